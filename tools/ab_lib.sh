#!/bin/bash
# A/B of the restart evaluation between the shipped library and an alternative build in
# everest_amd/_lib_ab (make -C everest_amd/csrc OUT=../_lib_ab BUILD=../_build_ab EXTRA=-D...):
# tools/restart_ab.py (scan / device chain / host round trip / minimize per evaluation) twice
# each, interleaved.  usage: bash tools/ab_lib.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:?tag}
mkdir -p "$OUT"
for i in 1 2; do
  timeout -k 10 300 python tools/restart_ab.py > "$OUT/ab_default_$i.json" 2> "$OUT/ab_default_$i.err" || exit 1
  EVR_LIB_PATH=everest_amd/_lib_ab/libeverest_amd.so timeout -k 10 300 python tools/restart_ab.py > "$OUT/ab_alt_$i.json" 2> "$OUT/ab_alt_$i.err" || exit 1
done
tail -n 1 "$OUT"/ab_*.json
