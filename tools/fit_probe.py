"""tell() of the config-4 bench state (5 outputs, n = 512, d = 6): lock-step rounds, time in
the native MLL plan evaluation (evr_mll_plan_eval: graph launch + completion) vs the rest of
the round (Python: L-BFGS-B steps, MLL assembly), and the plan's device time per round from
HIP events; with the native driver (default; EVR_FIT_NATIVE=0: the Python loop) its wall time
and each member's L-BFGS-B evaluation / iteration counts.  usage: python tools/fit_probe.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import bench
from everest_amd import gp as gpm


def main():
    s, tells = bench.make_ask_strategy(512, 256, 1024, 20, 1)
    exps = s.experiments
    stats = {"rounds": 0, "plan_s": 0.0}
    orig = gpm.MLLBatch._eval_plan

    def timed(self, *a, **k):
        t0 = time.perf_counter()
        r = orig(self, *a, **k)
        stats["plan_s"] += time.perf_counter() - t0
        stats["rounds"] += 1
        return r

    gpm.MLLBatch._eval_plan = timed
    nat = {"s": 0.0, "nfev": [], "nit": []}
    orig_native = gpm._fit_rounds_native

    def native(ev, *a, **k):   # the native driver: wall time and per-member L-BFGS-B counts
        t0 = time.perf_counter()
        r = orig_native(ev, *a, **k)
        nat["s"] += time.perf_counter() - t0
        st = getattr(ev, "native_stats", {})
        nat["nfev"].append(st.get("nfev"))
        nat["nit"].append(st.get("nit"))
        return r

    gpm._fit_rounds_native = native
    out = []
    for _ in range(3):
        stats.update(rounds=0, plan_s=0.0)
        nat.update(s=0.0, nfev=[], nit=[])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.tell(exps, replace=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        out.append({"tell_s": round(dt, 4), "rounds": stats["rounds"],
                    "plan_us_per_round": round(1e6 * stats["plan_s"] / max(1, stats["rounds"]), 1),
                    "other_us_per_round": round(1e6 * (dt - stats["plan_s"]) / max(1, stats["rounds"]), 1),
                    "native_s": round(nat["s"], 4), "last_fit": dict(gpm.LAST_FIT_STATS)})
    print(json.dumps({"tells_make": [round(t, 3) for t in tells], "tells": out}))


if __name__ == "__main__":
    main()
