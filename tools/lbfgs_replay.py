"""Replay a recorded restart L-BFGS-B trajectory (tools/lbfgs_trace.py) through the native
optimiser's C-ABI on the host: feeds the recorded (f, g) in order, checks that every x it asks
for is bitwise the recorded one, and times the optimiser's own steps (FG: after an evaluation;
NEW_X: starting the next iteration — Cauchy point, subspace step, line-search start).
usage: python tools/lbfgs_replay.py TRACE.npz [repeats]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def replay(tr, lib, timed=True):
    x0, lb, ub, xs, fs, gs = (np.ascontiguousarray(tr[k], dtype=np.float64) for k in ("x0", "lb", "ub", "xs", "fs", "gs"))
    n = x0.size
    h = ctypes.c_void_p()
    assert lib.evr_lbfgsb_create(n, 10, lb.ctypes.data, ub.ctypes.data, ctypes.c_double(2.220446049250313e-09 / np.finfo(float).eps),
                                 ctypes.c_double(1e-5), 20, ctypes.byref(h)) == 0
    x = np.zeros(n)
    t_fg, t_nx = [], []
    try:
        task = lib.evr_lbfgsb_start(h, x0.ctypes.data, x.ctypes.data)
        e = 0
        g = np.zeros(n)
        f = 0.0
        ok = True
        while True:
            if task == 1:
                if e >= len(fs):
                    break
                ok &= bool(np.array_equal(x, xs[e]))
                f, g = float(fs[e]), np.ascontiguousarray(gs[e])
                e += 1
                t0 = time.perf_counter_ns()
                task = lib.evr_lbfgsb_step(h, ctypes.c_double(f), g.ctypes.data, x.ctypes.data)
                t_fg.append(time.perf_counter_ns() - t0)
            elif task == 2:
                t0 = time.perf_counter_ns()
                task = lib.evr_lbfgsb_step(h, ctypes.c_double(f), g.ctypes.data, x.ctypes.data)
                t_nx.append(time.perf_counter_ns() - t0)
            else:
                break
    finally:
        lib.evr_lbfgsb_destroy(h)
    return ok, e, np.array(t_fg) / 1e3, np.array(t_nx) / 1e3


def main(path, reps=20):
    from everest_amd import _native

    lib = _native.load()
    tr = dict(np.load(path))
    best = None
    for _ in range(reps):
        ok, e, fg, nx = replay(tr, lib)
        tot = fg.sum() + nx.sum()
        if best is None or tot < best[0]:
            best = (tot, ok, e, fg, nx)
    tot, ok, e, fg, nx = best
    print(json.dumps({"trajectory_bitwise": ok, "evals_replayed": e, "evals_recorded": int(len(tr["fs"])),
                      "fg_steps": int(fg.size), "fg_median_us": round(float(np.median(fg)), 2),
                      "newx_steps": int(nx.size), "newx_median_us": round(float(np.median(nx)), 2),
                      "host_optimizer_ms_per_ask": round(float(tot) / 1e3, 3)}))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
