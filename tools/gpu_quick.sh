set -o pipefail
mkdir -p gpurun_out/${1:-quick}
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/${1:-quick}/pytest.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${1:-quick}/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-ask > gpurun_out/${1:-quick}/prof.log 2>&1
echo rc=$?
