#!/bin/bash
# Selected GPU tests + kernel-level profile of the b = 20 restart loop (tools/profile_restart.py)
# usage: tools/gpu_dbg.sh <tag> [test files ...]
set -o pipefail
OUT=gpurun_out/${1:-dbg}
shift
TESTS=${@:-tests/test_gpu_determinism.py tests/test_gpu_baseline_sizes.py}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest $TESTS -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -3 $OUT/pytest.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python tools/profile_restart.py > $OUT/restart.json 2> $OUT/restart.err
echo "prof rc=$?"
cat $OUT/restart.json
