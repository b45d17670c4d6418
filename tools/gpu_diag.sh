#!/bin/bash
# Diagnostics for one GPU call: selected parity tests, the ask's Python-level phases, the
# construction's synchronised probes, the diagonal-factor cycle split and the fit timing.
# usage: bash tools/gpu_diag.sh <tag> [pytest node ids...]     (outputs under gpurun_out/<tag>/)
set -o pipefail
TAG=${1:-diag}; shift
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> cmd...
  local name=$1 t=$2; shift 2
  echo "[$(date +%H:%M:%S)] $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%H:%M:%S)] $name rc=$rc"
  tail -3 "$O/$name.log"
  return $rc
}
if [ $# -gt 0 ]; then
  step pytest 400 python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread || exit 1
fi
step ask_phases 200 env EVR_MIN_STATS=1 python tools/ask_phases.py &&
step probes 200 python tools/construction_probes.py &&
step fit 200 python tools/bench_fit.py &&
step chol_prof 60 ./tools/_chol_prof &&
step timeline 200 rocprofv3 --kernel-trace --output-format csv -d "$O/tl" -o run -- python tools/ask_timeline.py &&
step timeline_report 60 python tools/ask_timeline.py --analyse "$O/tl"
echo "done rc=$?"
