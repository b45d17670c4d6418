#!/bin/bash
# One GPU-box pass made of named steps, each under its own time limit; stops at the first
# step that faults, aborts or times out (exit status other than 0 or 1: a failing test still
# lets later steps run).  Output under gpurun_out/<tag>/.
# usage: bash tools/gpu_steps.sh <tag> step...
#   pytest      the -m gpu parity suite
#   pytestf     the test files named in $PYTEST_FILES
#   restartab   tools/restart_ab.py (restart-scan variants: scan / chain / round trip / optimiser per
#               evaluation) -> <tag>/restart_ab.json
#   kmat        tools/bench_kmat.py (kernel assembly: config 5 cross / symmetric train, fill ceiling)
#   asktl       device timeline of one ask (tools/ask_timeline.py under rocprofv3 --kernel-trace)
#               -> <tag>/ask_timeline.json
#   planprobe   tools/plan_setup_probe.py (restart plan creation / first / warm evaluation)
#   hostprof    tools/ask_host_profile.py (cProfile of 5 warm asks)
#   benchq      python bench.py --no-cpu-baseline --no-eval-pass (the ask line only)
#   benche      python bench.py --no-cpu-baseline --no-config1 (ask line + evaluation pass + qLog)
#   kmatab      bench_kmat.py with the shipped library and everest_amd/_lib_ab, twice interleaved
#   kmatprof    bench_kmat.py with EVR_KMAT_PROF builds in everest_amd/_libkm{1,2,3} (1: no kernel evaluation,
#               2: no stores, 3: neither, 4: staging only, 8: staging + norms + MFMA; KMAT_PROFS picks) beside
#               the shipped library
#   kmatsq      two SQ counter passes over bench_kmat.py's MFMA kernel-matrix launches (KMAT_CASES)
#   digest      tools/ask_digest.py with the shipped library and everest_amd/_lib_ab (bitwise-neutral changes: equal lines)
#   trsm        tools/bench_trsm.py (forward substitution at the operator's G = L_base^-1 E shape)
#   post        tools/bench_post.py (GP posterior at the metric's shape, HIP events) and its rocprofv3
#               --kernel-trace --stats pass -> <tag>/post_prof
#   postab      tools/bench_post.py with the shipped library and everest_amd/_lib_ab, twice interleaved
#   postv       the same over the shipped library and the builds everest_amd/<dir> named in $POST_LIBS
#   kmatwpc     bench_kmat.py at EVR_KMAT_WPC = 0 (one-shot grid) / 1 / 2 / 4 (persistent, workgroups per CU)
#   sharded     tools/sharded_ask_check.py (config-4 ask at 2 ranks vs 1 rank, same seed)
#   pmc20       FETCH_SIZE / WRITE_SIZE passes over the bench's restart batch (b = 20 at the
#               ask's optimised restart candidates) -> <tag>/hbm_traffic.json (keys op@b20)
#   pmc512      the same over the b = 512 evaluation pass (keys without suffix)
#   sq20        SQ wave-cycle split of the restart chain kernels (hvi_kdw, qs_fwd, qs_bwd) at b = 20
#   kdwaves     per-wave phase stamps of hvi_kd3 / hvi_kdb (EVR_KD_PROF=2 build in _libprof/)
#   kdwwaves    per-(sample, candidate) phase stamps of hvi_kdw (EVR_KD_PROF=2 build in _libkdprof/)
#   hpeval      tools/hp_eval.py (device vs the 60-digit truth, fused and split roots) -> <tag>/hp_eval.json
#   benchsplit  benchq with EVR_ROOT=split (benchfused: EVR_ROOT=fused)
#   hpdump      tools/hp_state_dump.py (config-3 state + device values for tools/hp_truth.py) -> <tag>/hp_state.json
#   fill        tools/_fill_probe (write-bandwidth ceiling of the 33.5 MB config-5 output: 8 / 16 / 32 B
#               per lane, cached / non-temporal; hipcc -O3 tools/micro/fill_probe.hip -o tools/_fill_probe)
#   bench       python bench.py (the driver's default command)
#   prof        rocprofv3 --kernel-trace --stats of the bench command
#   fitprof     the same over tools/fit_probe.py (tell(): the MLL plan's kernels per round)
#   cpufull     bench.py --cpu-full-ask (one full reference-structure ask on the host cores)
#   qsprof      per-workgroup phase stamps of qs_bwd at the bench shape (tools/_qs_prof: hipcc
#               --offload-arch=gfx950 -O3 -std=c++17 -DEVR_QS_PROF tools/qs_prof.hip -o tools/_qs_prof)
#   cholprof    phase cycles + result digest of the 64x64 diagonal factor (tools/_chol_prof_pair:
#               hipcc --offload-arch=gfx950 -O3 -DEVR_CHOL_PROF tools/chol_prof.hip everest_amd/csrc/gemm.hip -o ...)
set -o pipefail
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <name> <timeout_s> cmd...
  local name=$1 t=$2; shift 2
  echo "[$(date +%H:%M:%S)] $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%H:%M:%S)] $name rc=$rc"
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for st in "$@"; do
  case $st in
    pytest) run pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    pytestf) run pytestf 900 python -u -m pytest $PYTEST_FILES -x -q --timeout 300 --timeout-method thread ;;
    restartab) run restartab 300 python tools/restart_ab.py && cp "$OUT/restartab.log" "$OUT/restart_ab.json" ;;
    asktl)
      run asktl_trace 300 rocprofv3 --kernel-trace -d "$OUT/asktl" -o run --output-format csv -- python tools/ask_timeline.py
      run asktl_parse 60 python tools/ask_timeline.py --analyse "$OUT/asktl" "$OUT/asktl_trace.log" && cp "$OUT/asktl_parse.log" "$OUT/ask_timeline.json" ;;
    hpdump) run hpdump 300 python tools/hp_state_dump.py "$OUT/hp_state.json" ;;
    hpeval) run hpeval 300 python tools/hp_eval.py "$OUT/hp_eval.json" ;;
    benchsplit) EVR_ROOT=split run benchsplit 600 python bench.py --no-cpu-baseline --no-eval-pass ;;
    benchfused) EVR_ROOT=fused run benchfused 600 python bench.py --no-cpu-baseline --no-eval-pass ;;
    fill) run fill 60 tools/_fill_probe && cp "$OUT/fill.log" "$OUT/fill.json" ;;
    planprobe) run planprobe 300 python tools/plan_setup_probe.py ;;
    hostprof) run hostprof 300 python tools/ask_host_profile.py ;;
    benchq) run benchq 600 python bench.py --no-cpu-baseline --no-eval-pass ;;
    benche) run benche 600 python bench.py --no-cpu-baseline --no-config1 ;;
    kmat) KMAT_CASES=cfg5_n2048_d32,cfg5_train_sym,n2048_d6,fit_train_n512 run kmat 300 python tools/bench_kmat.py && cp "$OUT/kmat.log" "$OUT/kmat.json" ;;
    kmatab)
      for i in 1 2; do
        KMAT_CASES=cfg5_n2048_d32,cfg5_train_sym,n2048_d6 run kmat_new_$i 300 python tools/bench_kmat.py
        EVR_LIB_PATH=everest_amd/_lib_ab/libeverest_amd.so KMAT_CASES=cfg5_n2048_d32,cfg5_train_sym,n2048_d6 run kmat_ab_$i 300 python tools/bench_kmat.py
      done ;;
    kmatprof)
      for k in ${KMAT_PROFS:-0 1 2 3}; do
        lib=everest_amd/_lib/libeverest_amd.so; [ $k -gt 0 ] && lib=everest_amd/_libkm$k/libeverest_amd.so
        EVR_LIB_PATH=$lib KMAT_CASES=cfg5_n2048_d32,cfg5_train_sym run kmat_prof$k 300 python tools/bench_kmat.py
      done ;;
    kmatsq)
      run kmatsq_a 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex "kmat_mfma" -d "$OUT/kmatsq_a" -o run --output-format csv -- python tools/bench_kmat.py
      run kmatsq_b 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS --kernel-include-regex "kmat_mfma" -d "$OUT/kmatsq_b" -o run --output-format csv -- python tools/bench_kmat.py ;;
    digest)
      run digest_new 300 python tools/ask_digest.py
      EVR_LIB_PATH=everest_amd/_lib_ab/libeverest_amd.so run digest_ab 300 python tools/ask_digest.py ;;
    trsm) run trsm 120 python tools/bench_trsm.py ;;
    post)
      run post 120 python tools/bench_post.py
      run post_prof 180 rocprofv3 --kernel-trace --stats -d "$OUT/post_prof" -o run --output-format csv -- python tools/bench_post.py ;;
    postv)   # bench_post.py over the shipped library and the variant builds named in $POST_LIBS, twice
      for i in 1 2; do
        run post_lib$i 120 python tools/bench_post.py
        for L in $POST_LIBS; do EVR_LIB_PATH=everest_amd/$L/libeverest_amd.so run post_$L$i 120 python tools/bench_post.py; done
      done ;;
    postab)
      for i in 1 2; do
        run post_new$i 120 python tools/bench_post.py
        EVR_LIB_PATH=everest_amd/_lib_ab/libeverest_amd.so run post_ab$i 120 python tools/bench_post.py
      done ;;
    kmatwpc)
      for w in 0 1 2 4; do
        EVR_KMAT_WPC=$w KMAT_CASES=cfg5_n2048_d32,cfg5_train_sym run kmat_wpc$w 300 python tools/bench_kmat.py
      done ;;
    sharded) run sharded 600 python tools/sharded_ask_check.py --ranks 2 --asks 3 --out "$OUT/sharded" ;;
    pmc20)
      cp profiles/hbm_traffic.json "$OUT/hbm_traffic.json"
      run pmc20_fetch 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc20_f" -o run --output-format csv -- python tools/loop_step.py 10 20 ask
      run pmc20_write 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc20_w" -o run --output-format csv -- python tools/loop_step.py 10 20 ask
      run pmc20_parse 60 python tools/pmc_traffic.py "$OUT/pmc20_f" "$OUT/pmc20_w" "$OUT/hbm_traffic.json" @b20 ;;
    pmc512)
      [ -f "$OUT/hbm_traffic.json" ] || cp profiles/hbm_traffic.json "$OUT/hbm_traffic.json"
      run pmc512_fetch 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc512_f" -o run --output-format csv -- python tools/loop_step.py 10 512
      run pmc512_write 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc512_w" -o run --output-format csv -- python tools/loop_step.py 10 512
      run pmc512_parse 60 python tools/pmc_traffic.py "$OUT/pmc512_f" "$OUT/pmc512_w" "$OUT/hbm_traffic.json" ;;
    sq20)
      run sq20 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex "hvi_kd[bw]|qs_fwd|qs_bwd|kmat_kernel|qs_dx" -d "$OUT/sq20" -o run --output-format csv -- python tools/loop_step.py 10 20 ask
      run sq20_parse 60 python tools/pmc_sq.py "$OUT/sq20" "$OUT/sq_counters.json" ;;
    kdwwaves) EVR_LIB_PATH=everest_amd/_libkdprof/libeverest_amd.so run kdwwaves 300 python tools/kdw_waves.py ;;
    kdwaves) EVR_LIB_PATH=everest_amd/_libprof/libeverest_amd.so run kdwaves 300 python tools/kd3_waves.py ;;
    bench) run bench 900 python bench.py ;;
    fitprof) run fitprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/fitprof" -o run --output-format csv -- python tools/fit_probe.py ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 10 ;;
    cpufull) run cpufull 1100 python bench.py --no-eval-pass --steps 2 --warmup 1 --cpu-full-ask "$OUT/cpu_full_ask.json" ;;
    qsprof) run qsprof 60 tools/_qs_prof && run qsprof_tail 60 tools/_qs_prof tail ;;
    cholprof) run cholprof_pair 60 tools/_chol_prof_pair ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo done
