"""High-precision truth of qNEHVI / qLogNEHVI at the BASELINE config-3 state — the adjudicator
for the cases where the device and the f64 oracle disagree (the new point's variance given the
baseline samples, L22^2 = var - |L21|^2, cancels next to baseline points).

Test infrastructure only (like make_golden.py); runs on the CPU of the build container:
    python tests/golden/make_hp_truth.py            (~5 min on 5 worker processes)
Reads tests/golden/hp_state.json (written by tools/hp_state_dump.py on the GPU box: the
device fit's hyperparameters, the pruned baseline rows and the candidate sets) and writes
tests/golden/hp_truth.json.

What is computed in 60-digit mpmath arithmetic (mp.dps = 60), from the exact f64 inputs
(X and Y regenerated from bench.py's seed, the hyperparameters, the Sobol-normal base samples):
* per output j (reference: the ModelListGP of SingleTaskGPs, bofire/surrogates/
  single_task_gp.py:39-71; the joint posterior of BoTorch's sample_cached_cholesky, called
  through bofire/strategies/predictives/qnehvi.py:39-52 with cache_root=True):
  K = k(X, X) + s2 I (RBF, ARD), its Cholesky factor L, alpha = K^-1 (y - c),
  W = L^-1 K(X, X_b), Sigma_bb = K(X_b, X_b) - W^T W, L_b = chol(Sigma_bb);
  the baseline samples Y_b = mu_b + s L_b z_b (-> the per-sample Pareto sets and cells);
* per candidate x: k = k(X, x), v = L^-1 k, mu = c + k.alpha, Sigma_bx = k_b - W^T v,
  L21 = L_b^-1 Sigma_bx, L22^2 = 1 - |v|^2 - |L21|^2 (no jitter: exact L22^2 > 0), and
  their exact derivatives in x (dk = k * (X - x) / ls^2 by coordinate, carried through the
  same linear maps); the samples y_s = y_mean + s (mu + L21.z_b[s] + L22 z_n[s]) and dy_s/dx.
The samples are then rounded to f64 and the HVI / log-HVI and their y-gradients evaluated in
f64 by the oracle's per-cell forms (oracle/qnehvi.py), chained with dy/dx: given the samples
both are sums of positive (resp. smooth, well-conditioned) terms, so f64 holds them to ~1e-14;
all of the cancellation lives in L22 and is done at 60 digits.
"""
import json
import math
import os
import sys
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from mpmath import mp, mpf, fdot, exp, sqrt  # noqa: E402

DPS = 60
GOLDEN = os.path.join(ROOT, "tests", "golden")


def dtlz2(X, m):
    # bench.py:53-63 (the bench's synthetic DTLZ2 problem)
    k = X.shape[1] - m + 1
    g = ((X[..., -k:] - 0.5) ** 2).sum(-1)
    fs = []
    for i in range(m):
        idx = m - 1 - i
        f = (1 + g) * np.cos(X[..., :idx] * math.pi / 2).prod(-1)
        if i > 0:
            f = f * np.sin(X[..., idx] * math.pi / 2)
        fs.append(f)
    return np.stack(fs, -1)


def state_inputs(st):
    rng = np.random.default_rng(st["x_seed"])
    X = rng.uniform(size=(st["n"], st["d"]))
    Y = dtlz2(X, st["m"])
    return X, Y


def chol(A):
    """Row-oriented Cholesky of a list-of-rows symmetric matrix (lower triangle read)."""
    n = len(A)
    L = []
    for i in range(n):
        Li = []
        Ai = A[i]
        for k in range(i):
            Lk = L[k]
            Li.append((Ai[k] - fdot(Li, Lk)) / Lk[k])
        dd = Ai[i] - fdot(Li, Li)
        if dd <= 0:
            raise ArithmeticError(f"not p.d. at pivot {i}: {dd}")
        Li.append(sqrt(dd))
        L.append(Li)
    return L


def fsolve(L, b):
    """L v = b (forward substitution), L a list of lower rows."""
    v = []
    for i, Li in enumerate(L):
        v.append((b[i] - fdot(Li, v)) / Li[i])
    return v


def bsolve_t(L, b):
    """L^T v = b (back substitution), L a list of lower rows."""
    n = len(L)
    v = [mpf(0)] * n
    for i in range(n - 1, -1, -1):
        s = b[i]
        for k in range(i + 1, n):
            s -= L[k][i] * v[k]
        v[i] = s / L[i][i]
    return v


def output_truth(args):
    """Everything that needs the high precision, for one output j."""
    j, st, zb, zn, cands = args
    mp.dps = DPS
    X, Y = state_inputs(st)
    h = st["hypers"][j]
    n, d = X.shape
    base = st["base_rows"]
    nb = len(base)
    ls = [mpf(v) for v in h["lengthscale"]]
    Xs = [[mpf(float(X[i, t])) / ls[t] for t in range(d)] for i in range(n)]
    noise, c, ym, s = mpf(h["noise"]), mpf(h["constant"]), mpf(h["y_mean"]), mpf(h["y_std"])
    half = mpf(1) / 2

    def kvec(xs):
        return [exp(-half * fdot([(a - b) for a, b in zip(Xi, xs)], [(a - b) for a, b in zip(Xi, xs)])) for Xi in Xs]

    K = []
    for i in range(n):
        row = kvec(Xs[i][:])[:i + 1]
        row[i] = mpf(1)
        K.append(row)
    Ky = [r[:] for r in K]
    for i in range(n):
        Ky[i][i] = K[i][i] + noise
    L = chol(Ky)
    ytil = [(mpf(float(Y[i, j])) - ym) / s for i in range(n)]
    alpha = bsolve_t(L, fsolve(L, [yi - c for yi in ytil]))

    def Kfull(a, b):
        return K[a][b] if b <= a else K[b][a]

    # W = L^-1 K(X, X_b): one forward solve per baseline point
    W = [fsolve(L, [Kfull(i, bcol) for i in range(n)]) for bcol in base]      # nb x n
    Sbb = []
    for a in range(nb):
        Sbb.append([Kfull(base[a], base[b]) - fdot(W[a], W[b]) for b in range(a + 1)])
    Lb = chol(Sbb)
    mu_b = [c + fdot([Kfull(base[a], i) for i in range(n)], alpha) for a in range(nb)]
    # baseline samples (raw scale), S x nb
    Yb = []
    for zs in zb:
        Yb.append([float(ym + s * (mu_b[a] + fdot(Lb[a], zs))) for a in range(nb)])

    out = []
    for x in cands:
        xs = [mpf(float(x[t])) / ls[t] for t in range(d)]
        k = kvec(xs)
        # dk/dx_t = k * (X_t - x_t) / ls_t^2 = k * (Xs_t - xs_t) / ls_t
        dk = [[k[i] * (Xs[i][t] - xs[t]) / ls[t] for i in range(n)] for t in range(d)]
        vecs = [k] + dk
        vs = [fsolve(L, kk) for kk in vecs]
        mus = [fdot(kk, alpha) for kk in vecs]
        mus[0] += c
        Sbx = [[kk[base[a]] - fdot(W[a], vv) for a in range(nb)] for kk, vv in zip(vecs, vs)]
        L21 = [fsolve(Lb, sb) for sb in Sbx]
        l22sq = 1 - fdot(vs[0], vs[0]) - fdot(L21[0], L21[0])
        if l22sq <= 0:
            raise ArithmeticError(f"exact L22^2 <= 0 for output {j}: {l22sq}")
        L22 = sqrt(l22sq)
        dL22 = [(-2 * fdot(vs[0], vs[t + 1]) - 2 * fdot(L21[0], L21[t + 1])) / (2 * L22) for t in range(d)]
        ys, dys = [], []
        for zs, znv in zip(zb, zn):
            ys.append(float(ym + s * (mus[0] + fdot(L21[0], zs) + L22 * znv)))
            dys.append([float(s * (mus[t + 1] + fdot(L21[t + 1], zs) + dL22[t] * znv)) for t in range(d)])
        out.append(dict(y=ys, dy=dys, L22=float(s * L22), rel=float(l22sq), mu=float(ym + s * mus[0])))
    return j, Yb, out


def main():
    import torch

    from oracle import qnehvi as oq
    from oracle.multiobjective import nondominated_cells, pareto_above_ref

    with open(os.path.join(GOLDEN, "hp_state.json")) as f:
        st = json.load(f)
    m, S, nb = st["m"], st["S"], len(st["base_rows"])
    zb = oq.base_samples(S, nb, m, st["sampler_seed"]).numpy()                  # S x nb x m
    zn = oq.base_samples(S, nb + 1, m, st["sampler_seed"])[:, nb].numpy()       # S x m
    names = list(st["sets"].keys())
    cands = np.concatenate([np.asarray(st["sets"][k]) for k in names])
    jobs = [(j, st, [[mpf(float(v)) for v in zb[si, :, j]] for si in range(S)],
             [mpf(float(zn[si, j])) for si in range(S)], cands) for j in range(m)]
    cache = os.environ.get("HP_TRUTH_CACHE")        # optional: keep the 60-digit part between runs
    if cache and os.path.exists(cache):
        with open(cache) as f:
            res = json.load(f)
    else:
        with Pool(min(m, os.cpu_count() or 1)) as pool:
            res = sorted(pool.map(output_truth, jobs), key=lambda r: r[0])
        if cache:
            with open(cache, "w") as f:
                json.dump(res, f)
    # baseline samples -> objective (minimise all: g = -y) -> per-sample cells (f64)
    Yb = torch.tensor(np.stack([np.asarray(r[1]) for r in res], -1))            # S x nb x m
    ref = torch.full((m,), st["ref"], dtype=torch.float64)
    base_obj = -Yb
    cells = [nondominated_cells(pareto_above_ref(base_obj[si], ref), ref) for si in range(S)]
    total_cells = sum(cc.shape[1] for cc in cells)
    b = cands.shape[0]
    y = torch.tensor([[[res[j][2][ci]["y"][si] for j in range(m)] for ci in range(b)] for si in range(S)])
    dy = torch.tensor([[[res[j][2][ci]["dy"][si] for j in range(m)] for ci in range(b)] for si in range(S)])
    # y: S x b x m, dy: S x b x m x d.  Per-sample forward + backward (one sample's graph at a
    # time): qNEHVI = mean_s HVI_s, qLogNEHVI = logmeanexp_s lse_s (d/d lse_s = softmax weight)
    def hvi_s(si, ys):
        lo, hi = cells[si][0], cells[si][1]
        ln = (torch.minimum((-ys).unsqueeze(-2), hi) - lo).clamp_min(0.0)       # b x C x m
        return ln.prod(-1).sum(-1)

    def lse_s(si, ys):
        return oq.log_hvi_cells(-ys, cells[si][0], cells[si][1], oq.TAU_RELU, oq.TAU_MAX_MO)

    gy = torch.zeros_like(y)
    gly = torch.zeros_like(y)
    vals = torch.zeros(S, b, dtype=torch.float64)
    with torch.no_grad():
        lses = torch.stack([lse_s(si, y[si]) for si in range(S)])              # S x b
    lval = oq.logmeanexp(lses, 0)
    wts = torch.softmax(lses, 0)
    for si in range(S):
        ys = y[si].clone().requires_grad_(True)
        v = hvi_s(si, ys)
        vals[si] = v.detach()
        v.sum().backward()
        gy[si] = ys.grad / S
        ys = y[si].clone().requires_grad_(True)
        (lse_s(si, ys) * wts[si]).sum().backward()
        gly[si] = ys.grad
    val = vals.mean(0)
    grad = torch.einsum("sbj,sbjt->bt", gy, dy)
    lgrad = torch.einsum("sbj,sbjt->bt", gly, dy)
    out = dict(source="tests/golden/make_hp_truth.py (mpmath dps=%d) over tests/golden/hp_state.json" % DPS,
               total_cells=int(total_cells), sets={})
    i0 = 0
    for k in names:
        nk = len(st["sets"][k])
        sl = slice(i0, i0 + nk)
        out["sets"][k] = dict(
            qnehvi=val.detach()[sl].tolist(), qnehvi_grad=grad[sl].tolist(),
            qlog=lval.detach()[sl].tolist(), qlog_grad=lgrad[sl].tolist(),
            L22=[[res[j][2][ci]["L22"] for ci in range(i0, i0 + nk)] for j in range(m)],
            rel=[[res[j][2][ci]["rel"] for ci in range(i0, i0 + nk)] for j in range(m)],
            mu=[[res[j][2][ci]["mu"] for ci in range(i0, i0 + nk)] for j in range(m)])
        i0 += nk
    with open(os.path.join(GOLDEN, "hp_truth.json"), "w") as f:
        json.dump(out, f)
    print("cells", total_cells, "(device", st["total_cells"], ")")


if __name__ == "__main__":
    main()
