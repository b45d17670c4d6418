set -o pipefail
export HVI_ONLY_KD=1 HVI_SIZES=20,512
timeout -k 10 300 python tools/bench_hvi.py || exit 1
for e in 1 2; do EVR_LIB_PATH=$PWD/everest_amd/_lib_exp$e/libeverest_amd.so timeout -k 10 300 python tools/bench_hvi.py || exit 1; done
