#!/bin/bash
# kernel-matrix A/B: bench_kmat (config 5 + d=6 2048^2) and one SQ counter pass on config 5.
# usage: bash tools/kmat_run.sh <tag> [ENV=val ...]   (env applied to every step)
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
env "$@" KMAT_CASES=cfg5_n2048_d32,n2048_d6,cfg3_cross_b512,cfg3_cross_b20 timeout -k 10 120 python tools/bench_kmat.py > $O/kmat.json 2>$O/kmat.err || exit $?
cat $O/kmat.json
env "$@" KMAT_CASES=cfg5_n2048_d32 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES -d $O/sq -o run --output-format csv --kernel-include-regex "kmat" -- python tools/bench_kmat.py > $O/sq.log 2>&1 &&
python tools/pmc_sq.py $O/sq $O/sq.json cfg5 && cat $O/sq.json
