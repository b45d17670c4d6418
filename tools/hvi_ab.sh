#!/bin/bash
# A/B of the sparse HVI scan kernels on the bench state (same build): the default hvi_kd2
# vs hvi_kd (EVR_KD=1).  usage: bash tools/hvi_ab.sh <tag>   (outputs under gpurun_out/<tag>/)
set -o pipefail
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export HVI_ONLY_KD=1 HVI_SIZES=${HVI_SIZES:-20,128,512}
timeout -k 10 300 python tools/bench_hvi.py > "$OUT/kd2.json" 2> "$OUT/kd2.err" || exit 1
EVR_KD=1 timeout -k 10 300 python tools/bench_hvi.py > "$OUT/kd1.json" 2> "$OUT/kd1.err" || exit 1
cat "$OUT/kd2.json" "$OUT/kd1.json"
