"""High-precision truth of the GP posterior moments at the BASELINE config-3 state (the fitted
5-output model of tests/golden/hp_state.json) — the posterior the reference takes from
GPyTorch's exact prediction (bofire/surrogates/botorch.py:27,33; [upstream] posterior at
botorch.py:180), pinned here without GPyTorch.

Test infrastructure only; runs on the CPU of the build container (~5 min, 5 processes):
    python tests/golden/make_post_truth.py
Per output j, in 60-digit mpmath (make_hp_truth.py's Cholesky and solves, from the exact f64
inputs): K = k(X, X) + noise I, L = chol(K), alpha = K^-1 (y - c); at every candidate x of the
state's sets: mean = y_mean + y_std (c + k.alpha), variance = y_std^2 (1 - |L^-1 k|^2) (RBF:
k(x, x) = 1; no observation noise).  Writes tests/golden/post_truth.json."""
import json
import os
import sys
from multiprocessing import Pool

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_hp_truth as hp  # noqa: E402
from mpmath import mp, mpf, fdot, exp  # noqa: E402


def output_moments(args):
    j, st, cands = args
    mp.dps = hp.DPS
    X, Y = hp.state_inputs(st)
    h = st["hypers"][j]
    n, d = X.shape
    ls = [mpf(v) for v in h["lengthscale"]]
    Xs = [[mpf(float(X[i, t])) / ls[t] for t in range(d)] for i in range(n)]
    noise, c, ym, s = mpf(h["noise"]), mpf(h["constant"]), mpf(h["y_mean"]), mpf(h["y_std"])
    half = mpf(1) / 2

    def kvec(xs):
        return [exp(-half * fdot([(a - b) for a, b in zip(Xi, xs)], [(a - b) for a, b in zip(Xi, xs)])) for Xi in Xs]

    Ky = []
    for i in range(n):
        row = kvec(Xs[i])[:i + 1]
        row[i] = 1 + noise
        Ky.append(row)
    L = hp.chol(Ky)
    ytil = [(mpf(float(Y[i, j])) - ym) / s for i in range(n)]
    alpha = hp.bsolve_t(L, hp.fsolve(L, [yi - c for yi in ytil]))
    mean, var = [], []
    for x in cands:
        k = kvec([mpf(float(x[t])) / ls[t] for t in range(d)])
        v = hp.fsolve(L, k)
        mean.append(float(ym + s * (c + fdot(k, alpha))))
        var.append(float(s * s * (1 - fdot(v, v))))
    return j, mean, var


def main():
    with open(os.path.join(hp.GOLDEN, "hp_state.json")) as f:
        st = json.load(f)
    names = list(st["sets"].keys())
    cands = np.concatenate([np.asarray(st["sets"][k]) for k in names])
    with Pool(min(st["m"], os.cpu_count() or 1)) as pool:
        res = sorted(pool.map(output_moments, [(j, st, cands) for j in range(st["m"])]), key=lambda r: r[0])
    out = dict(source="tests/golden/make_post_truth.py (mpmath dps=%d) over tests/golden/hp_state.json" % hp.DPS,
               sets={})
    i0 = 0
    for k in names:
        nk = len(st["sets"][k])
        out["sets"][k] = dict(mean=[r[1][i0:i0 + nk] for r in res], var=[r[2][i0:i0 + nk] for r in res])
        i0 += nk
    with open(os.path.join(hp.GOLDEN, "post_truth.json"), "w") as f:
        json.dump(out, f)
    print("points", cands.shape[0], "outputs", len(res))


if __name__ == "__main__":
    main()
