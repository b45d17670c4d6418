#!/bin/bash
# A/B of env knobs on the bench ask: bash tools/ab_env.sh <tag> "ENV=.. ENV2=.." ...
# (each argument is one variant; "" = defaults).  Outputs gpurun_out/<tag>/ab_<i>.log
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
i=0
for v in "$@"; do
  echo "[$(date +%H:%M:%S)] variant $i: $v"
  env $v timeout -k 10 240 python bench.py --no-cpu-baseline --no-eval-pass --steps 10 > $O/ab_$i.log 2>&1 || exit $?
  python - "$O/ab_$i.log" "$v" <<'P'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith("{")][-1]; d=json.loads(l)
a=d["ask"]; k=d["kernels"]
print(sys.argv[2] or "default", "ask_ms", d["ms_per_step"], "restarts_s", a["phases_last_ask"]["restarts_s"],
      "iters", a["phases_last_ask"]["optimizer_iterations"], "hvi_ms", k["hvi_fwd_bwd"]["launch_ms"], "tell", a["tell_s"],
      "chol2048", d["linalg"]["cholesky_n2048_b1"]["ms"], "cholinv", d["linalg"]["cholesky_inverse_n512_b5"]["ms"])
P
  i=$((i+1))
done
