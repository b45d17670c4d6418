"""BASELINE config 5: mixed-categorical domain (4 continuous + 4 categoricals x 7 levels,
one-hot -> d_eff = 32), Matern-5/2 ARD SingleTaskGP, n_train = 2048, qEI (SOBO) on 1 GPU.
Reports the LDS-tiled K-matrix assembly (ms, GB/s), the 2048 Cholesky (+ inverse), the
device GP fit (tell), qEI forward+backward throughput and one ask() (categorical FREE)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import pandas as pd
import torch

import everest_amd.data_models as dm
from everest_amd import ops, strategies


def ev_ms(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def domain():
    cont = [dm.ContinuousInput(key=f"x{i}", bounds=(0, 1)) for i in range(4)]
    cats = [dm.CategoricalInput(key=f"c{i}", categories=[f"l{k}" for k in range(7)]) for i in range(4)]
    out = dm.Outputs(features=[dm.ContinuousOutput(key="y", objective=dm.MinimizeObjective(w=1.0))])
    return dm.Domain(inputs=dm.Inputs(features=cont + cats), outputs=out)


def f(df):
    rng = np.random.default_rng(123)
    w = rng.normal(size=(4, 7))
    x = df[[f"x{i}" for i in range(4)]].values
    y = ((x - 0.3) ** 2).sum(1) + np.sin(3 * x[:, 0]) * x[:, 1]
    for i in range(4):
        y = y + w[i][df[f"c{i}"].map(lambda s: int(s[1:])).values]
    return y


def main(n=2048, b=512, method="FREE"):
    dev = torch.device("cuda", 0)
    dom = domain()
    rnd = strategies.map(dm.RandomStrategy(domain=dom, seed=13))
    X = rnd.ask(n)
    exps = X.copy()
    exps["y"] = f(X)
    exps["valid_y"] = 1
    spec = dm.SingleTaskGPSurrogate(inputs=dom.inputs, outputs=dom.outputs, kernel=dm.MaternKernel(nu=2.5))
    s = strategies.map(dm.SoboStrategy(domain=dom, acquisition_function=dm.qEI(), seed=1,
                                       surrogate_specs=dm.BotorchSurrogates(surrogates=[spec]),
                                       categorical_method=method, num_raw_samples=1024, num_restarts=8))
    t0 = time.perf_counter()
    s.tell(exps)
    torch.cuda.synchronize()
    t_tell = time.perf_counter() - t0
    gp = s.model
    d = gp.Xn.shape[1]
    t_k = ev_ms(lambda: ops.kernel_matrix(gp.Xn, gp.Xn, gp.ls, gp.kind, diag_add=gp.noise))
    kbytes = 8.0 * (n * n + 2 * n * d + d)
    K = ops.kernel_matrix(gp.Xn, gp.Xn, gp.ls, gp.kind, diag_add=gp.noise)
    t_chol = ev_ms(lambda: ops.cholesky(K))
    t_cholinv = ev_ms(lambda: ops.cholesky_inverse(K))
    acqf = s._get_acqfs(1)[0]
    lo, hi = s._bounds()
    Xc = torch.as_tensor(lo + (hi - lo) * np.random.default_rng(5).uniform(size=(b, d)), device=dev)
    t_qei = ev_ms(lambda: acqf.forward_backward(Xc))
    t0 = time.perf_counter()
    cand = s.ask(1)
    torch.cuda.synchronize()
    t_ask = time.perf_counter() - t0
    st = s.last_ask_stats
    print(json.dumps({
        "config": f"mixed 4 cont + 4x7 cat (d_eff={d}), Matern-2.5, n={n}, qEI, categorical_method={method}",
        "tell_s": round(t_tell, 3),
        "kernel_matrix_ms": round(t_k, 4), "kernel_matrix_GBs": round(kbytes / (t_k * 1e-3) / 1e9, 1),
        "cholesky_ms": round(t_chol, 3), "cholesky_inverse_ms": round(t_cholinv, 3),
        "qei_fwd_bwd_ms_b512": round(t_qei, 4), "qei_candidates_per_s": round(b / (t_qei * 1e-3), 1),
        "ask_s": round(t_ask, 3), "ask_evals": st.raw_evals + st.opt_evals,
        "candidate": {k: (v if isinstance(v, str) else float(v)) for k, v in cand.iloc[0].items()}}))


if __name__ == "__main__":
    main(*[int(a) if a.isdigit() else a for a in sys.argv[1:]])
