# GPU parity suite only (one process), stops at the first failure
set -o pipefail
mkdir -p gpurun_out/t
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" > gpurun_out/t/pytest.log 2>&1
rc=$?
tail -40 gpurun_out/t/pytest.log
exit $rc
