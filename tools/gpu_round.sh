#!/bin/bash
# One GPU-box pass: parity tests, bench line, rocprofv3 kernel stats of the same bench
# command, and two PMC passes (FETCH_SIZE / WRITE_SIZE) for the HBM-traffic figure.
# usage: bash tools/gpu_round.sh <tag>     (outputs under gpurun_out/<tag>/)
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> cmd...
  local name=$1 t=$2; shift 2
  echo "[$(date +%H:%M:%S)] $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%H:%M:%S)] $name rc=$rc"
  return $rc
}
step pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
step bench 600 python bench.py &&
step prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
     python bench.py --no-cpu-baseline --no-eval-pass &&
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv \
     --kernel-include-regex "hvi_|kmat_kernel|qn_|kcross_grad|Cijk" -- python tools/loop_step.py 10 &&
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv \
     --kernel-include-regex "hvi_|kmat_kernel|qn_|kcross_grad|Cijk" -- python tools/loop_step.py 10 &&
step pmc_fetch20 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch20" -o run --output-format csv \
     --kernel-include-regex "hvi_|kmat_kernel|qn_|qs_|kcross_grad|Cijk" -- python tools/loop_step.py 10 20 &&
step pmc_write20 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write20" -o run --output-format csv \
     --kernel-include-regex "hvi_|kmat_kernel|qn_|qs_|kcross_grad|Cijk" -- python tools/loop_step.py 10 20 &&
python tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/hbm_traffic.json" &&
python tools/pmc_traffic.py "$OUT/pmc_fetch20" "$OUT/pmc_write20" "$OUT/hbm_traffic.json" "@b20" &&
step pmc_sq 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
     SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES -d "$OUT/pmc_sq" -o run --output-format csv \
     --kernel-include-regex "hvi_kd|qs_fwd|qs_bwd|chol_step" -- python tools/loop_step.py 10 &&
step pmc_sq20 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
     SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES -d "$OUT/pmc_sq20" -o run --output-format csv \
     --kernel-include-regex "hvi_kd|qs_fwd|qs_bwd" -- python tools/loop_step.py 10 20 &&
python tools/pmc_sq.py "$OUT/pmc_sq" "$OUT/sq_counters.json" b512 &&
python tools/pmc_sq.py "$OUT/pmc_sq20" "$OUT/sq_counters.json" b20
rc=$?
echo "done rc=$rc"
exit $rc
