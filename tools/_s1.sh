set -o pipefail
mkdir -p gpurun_out/s5
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_linalg.py tests/test_gpu_baseline_sizes.py tests/test_gpu_gp_qnehvi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s5/pytest.log 2>&1 &&
timeout -k 10 200 python -u tools/construction_probes.py > gpurun_out/s5/probes.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eval-pass --steps 10 > gpurun_out/s5/bench.json 2> gpurun_out/s5/bench.err
echo rc=$?
