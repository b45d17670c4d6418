"""Where the restart phase of ask() spends its time (config-4 shape, b = 20 restarts):
device chain of one evaluation (graph replay between HIP events), one host round trip
(run_host: H2D + graph + D2H + sync), and the all-C++ L-BFGS-B loop, plus the construction
sub-phases of the acquisition.  Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

import bench


def main(b=20, reps=200):
    dev = torch.device("cuda", 0)
    X, Y, gp, hypers, acqf, t_fit, t_build = bench.build_state(512, 6, 5, 256, dev)
    out = {"construction": acqf.timings, "n_base": acqf.nb, "cells": acqf.stats.total_cells}
    rng = np.random.default_rng(0)
    x = rng.uniform(size=(b, 6))
    for bwd in (False, True):
        p = acqf.plan(b, bwd)
        p.X.copy_(torch.tensor(x, device=dev))
        for _ in range(5):
            p.run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            p.run()
        e1.record()
        torch.cuda.synchronize()
        out[f"chain_ms_{'fb' if bwd else 'f'}"] = round(e0.elapsed_time(e1) / reps, 4)
        t0 = time.perf_counter()
        for _ in range(reps):
            p.run_host(x)
        out[f"run_host_ms_{'fb' if bwd else 'f'}"] = round((time.perf_counter() - t0) / reps * 1e3, 4)
    p = acqf.plan(b, True)
    lb, ub = np.zeros(b * 6), np.ones(b * 6)
    t0 = time.perf_counter()
    xo, acq, info = p.minimize(x.reshape(-1), lb, ub, 2000)
    dt = time.perf_counter() - t0
    out["minimize"] = {"s": round(dt, 4), "iters": info[0], "evals": info[1], "ms_per_eval": round(dt / info[1] * 1e3, 4)}
    # the chain again at the optimised candidates (they dominate more cells: more scan terms)
    p.X.copy_(torch.tensor(np.asarray(xo).reshape(b, 6), device=dev))
    for _ in range(5):
        p.run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        p.run()
    e1.record()
    torch.cuda.synchronize()
    out["chain_ms_fb_optimised_x"] = round(e0.elapsed_time(e1) / reps, 4)
    print(json.dumps(out, default=float))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
