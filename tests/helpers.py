"""Builders of matched (oracle CPU, device) problem instances for the parity tests."""
from __future__ import annotations

import math

import numpy as np
import torch

from oracle import gp as ogp
from oracle import qnehvi as oq


def dtlz2(X: np.ndarray, m: int) -> np.ndarray:
    """DTLZ2 restated from bofire/benchmarks/multi.py:95-132 (minimisation)."""
    k = X.shape[1] - m + 1
    Xm = X[..., -k:]
    g = ((Xm - 0.5) ** 2).sum(-1)
    fs = []
    for i in range(m):
        idx = m - 1 - i
        f = (1 + g) * np.cos(X[..., :idx] * math.pi / 2).prod(-1)
        if i > 0:
            f = f * np.sin(X[..., idx] * math.pi / 2)
        fs.append(f)
    return np.stack(fs, -1)


def make_problem(n=40, d=4, m=3, seed=0, kind=ogp.RBF, noise=1e-3, lo=None, hi=None):
    """Random DTLZ2 problem with fixed (not fitted) hyperparameters.  Returns raw X, Y,
    bounds and per-output hyperparameter dicts."""
    rng = np.random.default_rng(seed)
    lo = np.zeros(d) if lo is None else np.asarray(lo, dtype=np.float64)
    hi = np.ones(d) if hi is None else np.asarray(hi, dtype=np.float64)
    Xu = rng.uniform(size=(n, d))
    X = lo + (hi - lo) * Xu
    Y = dtlz2(Xu, m) + 0.01 * rng.normal(size=(n, m))
    hyp = []
    for j in range(m):
        hyp.append(dict(lengthscale=rng.uniform(0.3, 1.5, d), noise=noise * (1 + j), constant=0.1 * j))
    return X, Y, lo, hi, hyp


def oracle_states(X, Y, lo, hi, hyp, kind=ogp.RBF):
    Xn = torch.tensor((X - lo) / (hi - lo), dtype=torch.float64)
    out = []
    for j, h in enumerate(hyp):
        y = torch.tensor(Y[:, j], dtype=torch.float64)
        ym, ys = ogp.standardize_params(y.unsqueeze(-1))
        out.append(ogp.GPState(X=Xn, y=(y - ym) / ys, lengthscale=torch.tensor(h["lengthscale"], dtype=torch.float64),
                               noise=h["noise"], constant=h["constant"], y_mean=float(ym), y_std=float(ys),
                               kind=kind, lo=torch.tensor(lo), hi=torch.tensor(hi)))
    return out


def device_gp(X, Y, lo, hi, hyp, kind=0, device="cuda"):
    from everest_amd.gp import GPBatch, GPHyper, standardize_params

    hypers = []
    for j, h in enumerate(hyp):
        ym, ys = standardize_params(Y[:, j])
        hypers.append(GPHyper(lengthscale=np.asarray(h["lengthscale"]), noise=h["noise"], constant=h["constant"],
                              y_mean=ym, y_std=ys))
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=device)  # noqa: E731
    Xn = t((X - lo) / (hi - lo))
    return GPBatch(Xn, t(Y), hypers, kind, t(lo), t(hi))


def mixed_domain(n_cont: int = 4, n_cat: int = 4, levels: int = 7):
    """BASELINE configs[4]: 4 continuous inputs + 4 categoricals x 7 levels (one-hot ->
    d_eff = 32), one minimised output (same domain as tools/bench_config5.py)."""
    import everest_amd.data_models as dm

    cont = [dm.ContinuousInput(key=f"x{i}", bounds=(0, 1)) for i in range(n_cont)]
    cats = [dm.CategoricalInput(key=f"c{i}", categories=[f"l{k}" for k in range(levels)]) for i in range(n_cat)]
    out = dm.Outputs(features=[dm.ContinuousOutput(key="y", objective=dm.MinimizeObjective(w=1.0))])
    return dm.Domain(inputs=dm.Inputs(features=cont + cats), outputs=out)


def mixed_f(df, n_cont: int = 4, n_cat: int = 4, levels: int = 7):
    """Synthetic response of the mixed domain: a smooth continuous part plus a random
    per-category offset."""
    rng = np.random.default_rng(123)
    w = rng.normal(size=(n_cat, levels))
    x = df[[f"x{i}" for i in range(n_cont)]].values
    y = ((x - 0.3) ** 2).sum(1) + np.sin(3 * x[:, 0]) * x[:, 1]
    for i in range(n_cat):
        y = y + w[i][df[f"c{i}"].map(lambda s: int(s[1:])).values]
    return y
