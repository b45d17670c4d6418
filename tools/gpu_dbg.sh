#!/bin/bash
# Determinism tests + kernel-level profile of the b = 20 restart loop (tools/profile_restart.py)
set -o pipefail
OUT=gpurun_out/${1:-dbg}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_determinism.py tests/test_gpu_baseline_sizes.py -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python tools/profile_restart.py > $OUT/restart.json 2> $OUT/restart.err
echo "prof rc=$?"
