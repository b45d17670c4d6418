"""CPU: pin the oracle before trusting it — cross-checks against independent mathematics
(SURVEY.md §7 step 1): exact hypervolume, scipy Cholesky posterior, finite differences,
torch autograd, and the psd_safe_cholesky ladder."""
import json
import math
import os

import numpy as np
import pytest
import torch

from oracle import gp as ogp
from oracle import multiobjective as omo
from oracle import qnehvi as oq
from tests.helpers import make_problem, oracle_states


@pytest.mark.parametrize("seed", range(12))
def test_box_cells_match_exact_hypervolume(seed):
    rng = np.random.default_rng(seed)
    m = int(rng.integers(2, 6))
    n = int(rng.integers(0, 9))
    Y = torch.tensor(rng.uniform(0, 1, (n, m)))
    ref = torch.tensor(rng.uniform(-0.2, 0.3, m))
    P = omo.pareto_above_ref(Y, ref) if n else torch.zeros(0, m, dtype=torch.float64)
    cells = omo.nondominated_cells(P, ref)
    for _ in range(6):
        y = rng.uniform(-0.1, 1.2, m)
        h_cells = omo.hvi_from_cells(torch.tensor(y), cells).item()
        Pn = P.numpy()
        h_ie = omo.hv_inclusion_exclusion(np.vstack([Pn, y[None]]), ref.numpy()) - (
            omo.hv_inclusion_exclusion(Pn, ref.numpy()) if len(Pn) else 0.0)
        h_sl = omo.hv_slicing(np.vstack([Pn, y[None]]), ref.numpy()) - omo.hv_slicing(Pn, ref.numpy())
        assert abs(h_cells - h_ie) < 1e-12 and abs(h_cells - h_sl) < 1e-12


def test_is_non_dominated_dedup():
    Y = torch.tensor([[1.0, 2.0], [1.0, 2.0], [0.5, 3.0], [0.4, 1.0]], dtype=torch.float64)
    assert omo.is_non_dominated(Y).tolist() == [True, False, True, False]
    assert omo.is_non_dominated(Y, deduplicate=False).tolist() == [True, True, True, False]


def test_posterior_vs_scipy_and_mll_grad_fd():
    X, Y, lo, hi, hyp = make_problem(n=30, d=3, m=1, seed=2)
    st = oracle_states(X, Y, lo, hi, hyp)[0]
    Xs = torch.rand(20, 3, dtype=torch.float64)
    m1, v1 = ogp.posterior(st, Xs, observation_noise=True)
    m2, v2 = ogp.posterior_scipy(st, Xs, observation_noise=True)
    assert np.allclose(m1.numpy(), m2, rtol=1e-10) and np.allclose(v1.numpy(), v2, rtol=1e-8)
    prior = ogp.dim_scaled_lognormal(3)
    x0 = torch.tensor([2e-3, 0.1, -0.2, 0.3, 0.0], requires_grad=True)
    v = ogp.mll_value(st.X, st.y, x0[2:], x0[0], x0[1], ogp.RBF, prior)
    v.backward()
    for k in range(5):
        e = torch.zeros(5, dtype=torch.float64)
        e[k] = 1e-6
        fp = ogp.mll_value(st.X, st.y, (x0 + e)[2:], (x0 + e)[0], (x0 + e)[1], ogp.RBF, prior).item()
        fm = ogp.mll_value(st.X, st.y, (x0 - e)[2:], (x0 - e)[0], (x0 - e)[1], ogp.RBF, prior).item()
        assert abs((fp - fm) / 2e-6 - x0.grad[k].item()) < 1e-5 * max(1.0, abs(x0.grad[k].item()))


def test_psd_safe_cholesky_ladder():
    V = torch.randn(20, 4, dtype=torch.float64, generator=torch.Generator().manual_seed(0))
    A = V @ V.T                                            # rank 4
    L, jit = ogp.psd_safe_cholesky(A)
    assert jit.item() in (1e-8, 1e-7, 1e-6)
    with pytest.raises(ogp.NotPSDError):
        ogp.psd_safe_cholesky(-torch.eye(3, dtype=torch.float64))


def test_sobol_normal_samples_pinned():
    """The Sobol-normal base samples that both sides consume (torch SobolEngine, scrambled)."""
    z = oq.draw_sobol_normal_samples(6, 4, seed=123)
    z2 = oq.draw_sobol_normal_samples(6, 4, seed=123)
    assert torch.equal(z, z2) and z.shape == (4, 6)
    assert abs(z.mean().item()) < 1.5


def test_qnehvi_oracle_hvi_equals_hv_difference():
    """qNEHVI for one sample equals HV(P_s U {y_s}) - HV(P_s) computed by slicing."""
    X, Y, lo, hi, hyp = make_problem(n=12, d=3, m=3, seed=4)
    st = oracle_states(X, Y, lo, hi, hyp)
    obj = oq.Objective(-torch.ones(3, dtype=torch.float64), torch.zeros(3, dtype=torch.float64))
    ref = torch.full((3,), -1.1, dtype=torch.float64)
    Xn = torch.tensor((X - lo) / (hi - lo))
    zb = oq.base_samples(4, 12, 3, 1)
    zn = oq.base_samples(4, 13, 3, 1)
    q = oq.QNEHVI(st, Xn, obj, ref, zb, zn[:, 12:13, :])
    xc = torch.rand(3, 1, 3, dtype=torch.float64)
    g = q.obj(q.samples(xc))
    per = q.hvi_per_sample(g)
    for s in range(4):
        P = omo.pareto_above_ref(q.base_obj[s], ref).numpy()
        for c in range(3):
            y = g[s, c, 0].numpy()
            ex = omo.hv_slicing(np.vstack([P, y[None]]), ref.numpy()) - omo.hv_slicing(P, ref.numpy())
            assert abs(per[s, c].item() - ex) < 1e-12


def test_prune_keeps_only_possible_pareto_points():
    X, Y, lo, hi, hyp = make_problem(n=30, d=3, m=2, seed=5)
    st = oracle_states(X, Y, lo, hi, hyp)
    obj = oq.Objective(-torch.ones(2, dtype=torch.float64), torch.zeros(2, dtype=torch.float64))
    idx, probs = oq.prune_baseline(st, torch.tensor((X - lo) / (hi - lo)), obj,
                                   torch.full((2,), -1.1, dtype=torch.float64), oq.base_samples(256, 30, 2, 3))
    assert set(idx.tolist()) == set(np.nonzero(probs.numpy())[0].tolist())
    assert 0 < len(idx) < 30


def test_qehvi_oracle_equals_exact_hv_difference():
    """qEHVI restatement: per-sample HVI over the fixed partition equals
    HV(P u {y_s}) - HV(P) computed by inclusion-exclusion (independent math)."""
    import numpy as np
    from oracle import qnehvi as oq
    from oracle.multiobjective import hv_inclusion_exclusion, pareto_above_ref
    from tests.helpers import make_problem, oracle_states

    X, Y, lo, hi, hyp = make_problem(n=20, d=3, m=3, seed=2)
    ost = oracle_states(X, Y, lo, hi, hyp)
    a, b, ref = -np.ones(3), np.zeros(3), -1.1 * np.ones(3)
    obj = oq.Objective(torch.tensor(a), torch.tensor(b))
    Yp = torch.tensor(Y * a + b)
    acq = oq.QEHVI(ost, Yp, obj, torch.tensor(ref), oq.base_samples(8, 1, 3, 5))
    Xc = torch.tensor(np.random.default_rng(0).uniform(size=(4, 1, 3)))
    v = acq.forward(Xc).numpy()
    smp = obj(acq.samples(Xc)).numpy()
    P = pareto_above_ref(Yp, torch.tensor(ref)).numpy()
    hv0 = hv_inclusion_exclusion(P, ref)
    ind = np.zeros(4)
    for s in range(8):
        for c in range(4):
            y = smp[s, c, 0]
            if (y > ref).all():
                P2 = pareto_above_ref(torch.tensor(np.vstack([P, y])), torch.tensor(ref)).numpy()
                ind[c] += hv_inclusion_exclusion(P2, ref) - hv0
    assert np.allclose(v, ind / 8, rtol=1e-9, atol=1e-12)   # HV differences cancel O(1) volumes
    assert (v > 0).any()


def test_log_hvi_oracle_tends_to_log_qnehvi():
    """The fat-smoothed log HVI restatement (qLogNEHVI / qLogEHVI) equals log(qNEHVI) /
    log(qEHVI) as tau_relu, tau_max -> 0, and stays within 1e-5 at the defaults here."""
    import numpy as np
    from oracle import qnehvi as oq
    from tests.helpers import make_problem, oracle_states

    X, Y, lo, hi, hyp = make_problem(n=20, d=3, m=3, seed=2)
    ost = oracle_states(X, Y, lo, hi, hyp)
    a, b, ref = -np.ones(3), np.zeros(3), -1.1 * np.ones(3)
    obj = oq.Objective(torch.tensor(a), torch.tensor(b))
    Xn = torch.tensor((X - lo) / (hi - lo))
    zb, zn = oq.base_samples(16, 20, 3, 7), oq.base_samples(16, 21, 3, 7)[:, 20:21]
    Xc = torch.tensor(np.random.default_rng(0).uniform(size=(6, 1, 3)))
    v = oq.QNEHVI(ost, Xn, obj, torch.tensor(ref), zb, zn).forward(Xc)
    tiny = oq.QLogNEHVI(ost, Xn, obj, torch.tensor(ref), zb, zn, tau_relu=1e-12, tau_max=1e-12).forward(Xc)
    dflt = oq.QLogNEHVI(ost, Xn, obj, torch.tensor(ref), zb, zn).forward(Xc)
    assert torch.allclose(tiny, v.log(), rtol=1e-10, atol=1e-10)
    assert torch.allclose(dflt, v.log(), rtol=1e-5, atol=1e-5)
    z = oq.base_samples(16, 1, 3, 5)
    e = oq.QEHVI(ost, torch.tensor(Y * a + b), obj, torch.tensor(ref), z).forward(Xc)
    le = oq.QLogEHVI(ost, torch.tensor(Y * a + b), obj, torch.tensor(ref), z, tau_relu=1e-12,
                     tau_max=1e-12).forward(Xc)
    assert torch.allclose(le, e.log(), rtol=1e-10, atol=1e-10)
    # fat tails: a candidate with zero HVI in every sample still gets a finite value
    far = torch.full((1, 1, 3), 1.0)
    lv = oq.QLogNEHVI(ost, Xn, obj, torch.tensor(ref), zb, zn).forward(far)
    assert torch.isfinite(lv).all()


@pytest.mark.parametrize("q,npend", [(1, 0), (3, 0), (2, 2)])
def test_qei_is_one_objective_qehvi_over_best_f_cell(q, npend):
    """The identity QEIJoint rests on: with one objective, qEHVI over the partition of
    {best_f} (a single cell [best_f, inf) above any ref < best_f) equals qEI with that best_f
    on the same base samples, pending points included."""
    X, Y, lo, hi, hyp = make_problem(n=20, d=3, m=1, seed=q + 3 * npend)
    st = oracle_states(X, Y, lo, hi, hyp)
    a, b0 = -1.0, 0.0
    Xn = torch.tensor((X - lo) / (hi - lo))
    mean, _ = ogp.posterior(st[0], Xn)
    best_f = float((a * mean + b0).max())
    qq = q + npend
    z = oq.base_samples(64, qq, 1, 5)                                   # S x qq x 1
    rng = np.random.default_rng(1)
    Xp = torch.tensor(rng.uniform(size=(npend, 3))) if npend else None
    f64 = dict(dtype=torch.float64)
    qe = oq.QEHVI(st, torch.tensor([[best_f]], **f64), oq.Objective(torch.tensor([a], **f64), torch.tensor([b0], **f64)),
                  torch.tensor([best_f - 1.0], **f64), z, X_pending=Xp)
    Xc = torch.tensor(rng.uniform(size=(9, q, 3)))
    v_hvi = qe.forward(Xc)
    Xf = torch.cat([Xc, Xp.unsqueeze(0).expand(9, npend, 3)], 1) if npend else Xc
    v_ei = oq.qei(st, Xf, best_f, z[..., 0], a=a, bconst=b0)
    # inclusion-exclusion over the q-subsets cancels terms: equal up to rounding
    assert torch.allclose(v_hvi, v_ei, rtol=1e-10, atol=1e-13)


def test_log_fatplus_cutoff_is_exact():
    """hvi_log.hip drops exp(x) / log1p(exp(x)) from log fatplus below x = -60: on a dense
    grid to -1e8 both F = softplus(x) + 0.1 / (1 + x^2) and the derivative numerator
    sigmoid(x) - 0.2 x / (1 + x^2)^2 round to the same doubles without the exp term."""
    x = -np.concatenate([np.linspace(60.0, 745.0, 400001), np.geomspace(60.0, 1e8, 200001)])
    e = np.exp(x)
    c = 1.0 / (1.0 + x * x)
    assert np.array_equal(np.log1p(e) + 0.1 * c, 0.0 + 0.1 * c)
    assert np.array_equal(e / (1.0 + e) - 0.2 * x * c * c, 0.0 - 0.2 * x * c * c)


@pytest.mark.parametrize("q", [1, 2, 3])
def test_log_qehvi_subsets_tend_to_log_exact_hvi(q):
    """The q-subset log restatement (log_qehvi_cells: logsumexp per subset size, odd minus
    even by logdiffexp) tends to log of the exact inclusion–exclusion HVI as the
    temperatures go to 0, equals log_hvi_cells at q = 1, and a log feasibility of 0 changes
    nothing."""
    import itertools

    g = torch.Generator().manual_seed(q)
    m = 3
    P = torch.rand(12, m, dtype=torch.float64, generator=g)
    ref = torch.zeros(m, dtype=torch.float64)
    lo, hi = omo.nondominated_cells(omo.pareto_above_ref(P, ref), ref)
    obj = torch.rand(6, q, m, dtype=torch.float64, generator=g) * 1.2
    la = oq.log_qehvi_cells(obj, lo, hi, 1e-10, 1e-7)
    ex = torch.zeros(6, dtype=torch.float64)
    for i in range(1, q + 1):
        for sub in itertools.combinations(range(q), i):
            ov = obj[:, list(sub)].min(1).values
            ex += (-1) ** (i + 1) * (torch.minimum(ov.unsqueeze(1), hi) - lo).clamp_min(0).prod(-1).sum(-1)
    pos = ex > 1e-6
    assert pos.sum() >= 2
    assert torch.allclose(la.exp()[pos], ex[pos], rtol=1e-5)
    assert (la.exp()[~pos] < 1e-5).all()
    if q == 1:
        assert torch.equal(oq.log_qehvi_cells(obj, lo, hi, 1e-6, 1e-3), oq.log_hvi_cells(obj[:, 0], lo, hi, 1e-6, 1e-3))
    zero = torch.zeros(6, q, dtype=torch.float64)
    assert torch.equal(oq.log_qehvi_cells(obj, lo, hi, 1e-6, 1e-3, zero), oq.log_qehvi_cells(obj, lo, hi, 1e-6, 1e-3))
    # a log feasibility lf on every point scales the single-point areas by exp(lf): q = 1 shifts by lf
    if q == 1:
        lf = torch.full((6, 1), -0.7, dtype=torch.float64)
        assert torch.allclose(oq.log_qehvi_cells(obj, lo, hi, 1e-6, 1e-3, lf),
                              oq.log_qehvi_cells(obj, lo, hi, 1e-6, 1e-3) - 0.7, rtol=0, atol=1e-12)


def test_logdiffexp():
    a = torch.tensor([0.0, -1.0, 2.0, -math.inf, 1.0], dtype=torch.float64)
    b = torch.tensor([-1.0, -math.inf, 2.0, -math.inf, -1e-12], dtype=torch.float64)
    out = oq.logdiffexp(a, b)
    assert torch.allclose(out[:2], torch.log(torch.exp(a[:2]) - torch.exp(b[:2])))
    assert out[2] == -math.inf and out[3] == -math.inf
    assert torch.allclose(out[4], torch.log(-torch.expm1(b[4] - a[4])) + a[4])


def test_log_fatmoid_restatement():
    """safe_math.log_fatmoid as restated: exp of it is the two-branch Cauchy fatmoid, it is
    continuous (1/2) at 0 with a matching slope, tends to 1 for x -> +inf, decays as
    O(1/x^2) for x -> -inf, and the closed-form slope used by the device backward
    (qnehvi_general.hip qg_dlog_fatmoid) equals autograd's."""
    m = math.sqrt(1 / 3)
    cauchy = lambda z: 1 / (1 + z * z)  # noqa: E731
    x = torch.linspace(-50, 50, 20001, dtype=torch.float64)
    direct = torch.where(x < 0, 2 / 3 * cauchy(x - m), 1 - 2 / 3 * cauchy(x + m))
    lf = oq.log_fatmoid(x)
    assert torch.allclose(lf.exp(), direct, rtol=1e-14, atol=0)
    assert abs(float(oq.log_fatmoid(torch.tensor(0.0, dtype=torch.float64))) - math.log(0.5)) < 1e-15
    assert abs(float(oq.log_fatmoid(torch.tensor(-1e-12, dtype=torch.float64))) - math.log(0.5)) < 1e-11
    big = torch.tensor([-1e3, -1e4], dtype=torch.float64)
    ratio = oq.log_fatmoid(big).exp() * big.square()
    assert torch.allclose(ratio, torch.full_like(ratio, 2 / 3), rtol=1e-2)      # 2/3 / x^2 tail
    assert float(oq.log_fatmoid(torch.tensor(1e6, dtype=torch.float64))) > -1e-12
    xg = x.clone().requires_grad_(True)
    oq.log_fatmoid(xg).sum().backward()

    def dlog(v):
        if v < 0:
            u = v - m
            return -2 * u / (1 + u * u)
        u = v + m
        w = 1 + u * u
        c = (2 / 3) / w
        return 2 * u * c / (w * (1 - c))

    ref = torch.tensor([dlog(float(v)) for v in x], dtype=torch.float64)
    assert torch.allclose(xg.grad, ref, rtol=1e-12, atol=1e-15)
    assert abs(dlog(-1e-15) - dlog(0.0)) < 1e-12                  # C^1 at 0


def test_log_feasibility_fat_default():
    """qLog* feasibility is fat by default; fat=False is the logistic form."""
    con = oq.OutputConstraints(out=[0], sign=[1.0], thr=[0.2], eta=[1e-3])
    Y = torch.tensor([[[0.0], [0.2], [0.5]]], dtype=torch.float64)
    lf = oq.log_feasibility(con, Y)
    assert torch.allclose(lf, oq.log_fatmoid(-(Y[..., 0] - 0.2) / 1e-3))
    ll = oq.log_feasibility(con, Y, fat=False)
    assert torch.allclose(ll, torch.nn.functional.logsigmoid(-(Y[..., 0] - 0.2) / 1e-3))
    assert float(lf[0, 2]) > float(ll[0, 2]) + 100          # fat tail: far less negative
