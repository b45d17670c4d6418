set -o pipefail
mkdir -p gpurun_out/s3
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_hvi_kd.py tests/test_gpu_proj.py tests/test_gpu_config4.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s3/pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/s3/bench.json 2> gpurun_out/s3/bench.err &&
EVR_KD3=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eval-pass --steps 10 > gpurun_out/s3/bench_nokd3.json 2> gpurun_out/s3/bench_nokd3.err
echo rc=$?
