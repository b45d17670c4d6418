"""Where tell() spends its time at the bench shape (DTLZ2 d=6 m=5, n=512): cold and warm
tell wall time, batched MLL rounds / evaluations per output and the time per round, for
the lock-step batched fit and the per-output threaded fit (EVR_FIT_BATCH=0).  One JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import pandas as pd
import torch

import everest_amd.data_models as dm
from everest_amd import gp as gpm
from everest_amd import strategies
from everest_amd.benchmarks import DTLZ2


def main(n=512):
    bm = DTLZ2(dim=6, num_objectives=5)
    Xd = pd.DataFrame(np.random.default_rng(0).uniform(size=(n, 6)), columns=bm.domain.inputs.get_keys())
    exps = bm.f(Xd, return_complete=True)
    out = {}
    calls = {"rounds": 0, "members": 0, "s": 0.0}
    orig = gpm.MLLBatch.__call__

    def timed(self, idx, xs):
        t = time.perf_counter()
        r = orig(self, idx, xs)
        calls["s"] += time.perf_counter() - t
        calls["rounds"] += 1
        calls["members"] += len(idx)
        return r

    gpm.MLLBatch.__call__ = timed
    for mode in ("1", "0", "1"):
        os.environ["EVR_FIT_BATCH"] = mode
        s = strategies.map(dm.QnehviStrategy(domain=bm.domain, ref_point=bm.ref_point, seed=1))
        for k in calls:
            calls[k] = 0 if k != "s" else 0.0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.tell(exps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        key = f"batch{mode}" + ("_cold" if f"batch{mode}_cold" not in out else "")
        out[key] = {"tell_s": round(dt, 4), **({"mll_rounds": calls["rounds"], "mll_members": calls["members"],
                                               "ms_per_round": round(calls["s"] / max(1, calls["rounds"]) * 1e3, 3)}
                                             if mode == "1" else {})}
    print(json.dumps(out))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
