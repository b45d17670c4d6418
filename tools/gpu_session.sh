#!/bin/bash
# One GPU-box pass for a development step: parity suite, HVI scan A/B, GEMM shape probe and
# the bench line.  Stops at the first step that faults, aborts or times out (exit status
# other than 0 or 1); a failing test (1) still lets the timing steps run.
# usage: bash tools/gpu_session.sh <tag> [steps...]   steps: pytest ab gemm bench (default all)
set -o pipefail
TAG=${1:-s}
shift
STEPS=${*:-pytest ab gemm bench}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <name> <timeout_s> cmd...
  local name=$1 t=$2; shift 2
  echo "[$(date +%H:%M:%S)] $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%H:%M:%S)] $name rc=$rc"
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for st in $STEPS; do
  case $st in
    pytest) run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    ab) run ab 600 bash tools/hvi_ab.sh "$TAG/ab" ;;
    gemm) run gemm 300 python tools/gemm_shapes.py ;;
    bench) run bench 600 python bench.py ;;
    ask) run ask 300 python tools/profile_ask.py ;;
  esac
done
echo done
