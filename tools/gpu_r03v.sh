set -o pipefail
O=gpurun_out/r03v; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 60 ./tools/_chol_prof > $O/chol_pair.log 2>&1 &&
timeout -k 10 60 ./tools/_chol_prof_single > $O/chol_single.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_linalg.py tests/test_gpu_optim.py tests/test_gpu_fit.py tests/test_gpu_config4.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 200 env EVR_MIN_STATS=1 python tools/ask_phases.py > $O/ask_phases.log 2>&1 &&
timeout -k 10 200 env EVR_MIN_STATS=1 EVR_PRELAUNCH=0 python tools/ask_phases.py > $O/ask_phases_noprelaunch.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval-pass --steps 10 > $O/bench.log 2>&1 &&
timeout -k 10 300 env EVR_PRELAUNCH=0 python bench.py --no-cpu-baseline --no-eval-pass --steps 10 > $O/bench_noprelaunch.log 2>&1
echo rc=$?
