"""Time a full QnehviStrategy tell()/ask() on the config-4 shaped problem and print the
phase breakdown (fit, construction sub-phases, raw screening, restart optimisation)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import pandas as pd
import torch

import everest_amd.data_models as dm
from everest_amd import strategies
from everest_amd.benchmarks import DTLZ2


def main(n=512, S=256, raw=1024, restarts=20, asks=3):
    bench = DTLZ2(dim=6, num_objectives=5)
    X = pd.DataFrame(np.random.default_rng(0).uniform(size=(n, 6)), columns=bench.domain.inputs.get_keys())
    exps = bench.f(X, return_complete=True)
    s = strategies.map(dm.QnehviStrategy(domain=bench.domain, ref_point=bench.ref_point, seed=1,
                                         num_sobol_samples=S, num_raw_samples=raw, num_restarts=restarts))
    t0 = time.perf_counter()
    s.tell(exps)
    torch.cuda.synchronize()
    t_tell = time.perf_counter() - t0
    rows = []
    for i in range(asks):
        t0 = time.perf_counter()
        c = s.ask(1)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        st = s.last_ask_stats
        rows.append(dict(ask_s=round(dt, 4), construction=s.last_acqf.timings, raw_s=round(st.t_raw, 4),
                         opt_s=round(st.t_opt, 4), raw_evals=st.raw_evals, opt_evals=st.opt_evals,
                         opt_iters=st.opt_iters, chunks=st.chunks, n_base=s.last_acqf.nb, box_path=s.last_acqf.box_path,
                         cells=s.last_acqf.stats.total_cells, best=float(st.best_value)))
    print(json.dumps(dict(tell_s=round(t_tell, 3), asks=rows), default=float))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
