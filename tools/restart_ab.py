"""The restart-batch evaluation at the bench state: the config-4 QnehviStrategy after one ask
(bench.make_ask_strategy, seed 1), its optimised restart candidates (b = 20) and a Sobol batch:
the restart scan's device time (hvi_kdw, 10 launches in one HIP graph between HIP events), the
plan's device chain per evaluation (50 back-to-back device-mode graph launches between HIP
events), its host round trip per evaluation (plan.run_host: launch + chain + completion poll)
and the native L-BFGS-B's wall time per evaluation (plan.minimize from the Sobol start, 30
iterations: round trip + the optimiser's host step).  The forward operator is EVR_ROOT's
(split by default).  One JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import bench
from everest_amd import ops


def graph_ms(f, reps=10):
    f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            f()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda", 0)
    s, _ = bench.make_ask_strategy(512, 256, 1024, 20, 1, None, seed=1)
    s.ask(1)
    acqf = s.last_acqf
    Xopt = np.ascontiguousarray(s.last_ask_stats.restart_X.reshape(20, -1))
    out = {}
    for tag, X in (("opt", Xopt), ("sobol", bench.candidates(20, 6, seed=5, device=dev).cpu().numpy())):
        Xt = torch.tensor(X, device=dev)
        b = X.shape[0]
        R, P = ops.qnehvi_small_forward(acqf.state, acqf.model, acqf.gp.cross(Xt), b)
        G, L22, flags = ops.qnehvi_small_samples(acqf.state, R, P, b)
        for name in ("kdw",):
            scan = graph_ms(lambda: ops.hvi_restart_fb(acqf.state, G, b))
            acqf._plans = {}
            p = acqf.plan(b, True)
            p.X.copy_(Xt)
            for _ in range(3):
                p.run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                p.run()
            e1.record()
            torch.cuda.synchronize()
            chain = e0.elapsed_time(e1) / 50
            p.run_host(X)
            t0 = time.perf_counter()
            for _ in range(50):
                p.run_host(X)
            rt = (time.perf_counter() - t0) / 50
            rec = {"scan_us": round(scan * 1e3, 2), "chain_us": round(chain * 1e3, 2),
                   "eval_roundtrip_us": round(rt * 1e6, 2)}
            if tag == "sobol":
                t0 = time.perf_counter()
                _, _, info = p.minimize(X, np.zeros_like(X), np.ones_like(X), 30)
                rec["minimize_us_per_eval"] = round((time.perf_counter() - t0) / max(1, info[1]) * 1e6, 2)
                rec["minimize_evals"] = int(info[1])
            out[f"{tag}_{name}"] = rec
    acqf._plans = {}
    out["root"] = acqf.root
    out["construction"] = {k: round(v * 1e3, 3) for k, v in acqf.timings.items()}
    out["base_jitter"] = [float(v) for v in acqf.base_jitter.cpu()]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
