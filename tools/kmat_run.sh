set -o pipefail
mkdir -p gpurun_out/kmat
timeout -k 10 300 python -u -m pytest tests/test_gpu_linalg.py tests/test_gpu_gp_qnehvi.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/kmat/pytest.log 2>&1 || { tail -30 gpurun_out/kmat/pytest.log; exit 1; }
tail -2 gpurun_out/kmat/pytest.log
timeout -k 10 120 python tools/bench_kmat.py || exit 1
