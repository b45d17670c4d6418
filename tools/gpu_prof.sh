#!/bin/bash
# bench line + rocprofv3 kernel stats of the same bench command (no CPU baseline / eval pass)
# usage: bash tools/gpu_prof.sh <tag> [pytest-args...]
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval-pass --steps 10 > $O/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
     python bench.py --no-cpu-baseline --no-eval-pass --steps 10 > $O/prof.log 2>&1 &&
python tools/trace_summary.py $O/prof/run_kernel_trace.csv 20; echo rc=$?
