set -o pipefail
export HVI_ONLY_KD=1 HVI_SIZES=512 TMPDIR=/tmp
mkdir -p gpurun_out/hpmc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/hpmc/p1 -o run --output-format csv --kernel-include-regex "hvi_kd" -- python tools/bench_hvi.py > gpurun_out/hpmc/p1.log 2>&1 || { tail -20 gpurun_out/hpmc/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS -d gpurun_out/hpmc/p2 -o run --output-format csv --kernel-include-regex "hvi_kd" -- python tools/bench_hvi.py > gpurun_out/hpmc/p2.log 2>&1 || { tail -20 gpurun_out/hpmc/p2.log; exit 1; }
echo ok
