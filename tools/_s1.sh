set -o pipefail
mkdir -p gpurun_out/s9
export TMPDIR=/tmp
EVR_MIN_STATS=1 timeout -k 10 200 python -u tools/ask_phases.py > gpurun_out/s9/phases_kdb.log 2>&1 &&
EVR_KDB=0 EVR_MIN_STATS=1 timeout -k 10 200 python -u tools/ask_phases.py > gpurun_out/s9/phases_kd3.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eval-pass --steps 10 > gpurun_out/s9/bench_kdb.json 2> gpurun_out/s9/bench.err &&
EVR_KDB=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eval-pass --steps 10 > gpurun_out/s9/bench_kd3.json 2>> gpurun_out/s9/bench.err
echo rc=$?
