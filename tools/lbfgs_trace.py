"""Record the restart L-BFGS-B trajectory of one warm bench ask (config 4): every evaluation's
x, f and gradient, through the Python-driven native L-BFGS-B (the plan's C++ loop has no
per-evaluation hook; the plan is switched off, so the op-by-op chain evaluates — bitwise the
plan, tests/test_gpu_proj.py).  tools/lbfgs_replay.py replays the (f, g) sequence on the
host to time and profile the optimiser's own step.  usage: python tools/lbfgs_trace.py OUT.npz"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(out):
    import bench
    from everest_amd import acquisition, optim

    s, _ = bench.make_ask_strategy(512, 256, 1024, 20, 1)
    s.ask(1)
    rec = {}
    orig = optim.minimize_lbfgsb

    def traced(fun, x0, lb, ub, **kw):
        xs, fs, gs = [], [], []

        def f2(x):
            v, g = fun(x)
            xs.append(np.array(x, dtype=np.float64))
            fs.append(float(v))
            gs.append(np.array(g, dtype=np.float64).reshape(-1))
            return v, g
        res = orig(f2, x0, lb, ub, **kw)
        rec.update(x0=np.asarray(x0, dtype=np.float64), lb=np.asarray(lb), ub=np.asarray(ub), xs=np.array(xs),
                   fs=np.array(fs), gs=np.array(gs), nit=res.nit)
        return res

    optim.minimize_lbfgsb = traced
    acquisition.QNEHVI.supports_plan = property(lambda self: False)
    s.ask(1)
    np.savez(out, **rec)
    print({"evals": len(rec["fs"]), "nit": int(rec["nit"]), "n": int(rec["x0"].size)})


if __name__ == "__main__":
    main(sys.argv[1])
