set -o pipefail
O=gpurun_out/r03i; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_linalg.py -x -v --timeout 120 --timeout-method thread > $O/pytest_linalg.log 2>&1 &&
timeout -k 10 60 ./tools/_chol_prof > $O/chol_prof.log 2>&1 &&
timeout -k 10 200 python tools/chol_bench.py > $O/chol_bench.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_hvi_kd.py tests/test_gpu_proj.py tests/test_gpu_categorical.py tests/test_gpu_fit.py tests/test_gpu_baseline_sizes.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu-baseline --no-eval-pass --steps 10 > $O/bench_fuse.log 2>&1 &&
EVR_KD_FUSE=0 timeout -k 10 200 python bench.py --no-cpu-baseline --no-eval-pass --steps 10 > $O/bench_nofuse.log 2>&1 &&
for e in 0 1 2; do EVR_KMAT_EPI=$e KMAT_CASES=cfg5_n2048_d32 timeout -k 10 120 python tools/bench_kmat.py > $O/kmat_epi$e.log 2>&1 || exit 1; done
echo rc=$?
