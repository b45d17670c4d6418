"""Results do not depend on what the torch caching allocator hands out: every kernel writes
before it reads its scratch, so evaluations after poisoning the cache with NaN / junk are
bitwise equal (the GP fit, the posterior and the qNEHVI chain)."""
import numpy as np
import pytest
import torch

from tests.helpers import device_gp, make_problem

pytestmark = pytest.mark.gpu


def _poison(val):
    junk = torch.full((96 << 20,), val, dtype=torch.float64, device="cuda")   # 768 MB
    del junk


@pytest.mark.parametrize("kind", [0, 3])
def test_mll_independent_of_scratch_contents(kind):
    from everest_amd.gp import MLLEvaluator

    rng = np.random.default_rng(1)
    Xn = torch.tensor(rng.uniform(size=(300, 8)), device="cuda")
    y = rng.normal(size=300)
    ev = MLLEvaluator(Xn, y, kind, ("lognormal", 2.0, 1.7), ("lognormal", -4.0, 1.0))
    x = np.r_[1e-3, 0.1, rng.normal(size=8)]
    out = []
    for val in (float("nan"), 1e300, -7.0):
        _poison(val)
        out.append(ev(x))
    for v, g in out[1:]:
        assert v == out[0][0] and np.array_equal(g, out[0][1])


def test_qnehvi_chain_independent_of_scratch_contents():
    from everest_amd.acquisition import QNEHVI

    X, Y, lo, hi, hyp = make_problem(n=50, d=4, m=3, seed=2)
    gp = device_gp(X, Y, lo, hi, hyp)
    Xc = torch.tensor(np.random.default_rng(3).uniform(size=(37, 4)), device="cuda")
    res = []
    for val in (float("nan"), 1e300):
        _poison(val)
        acqf = QNEHVI(gp, X, X, -1.1 * np.ones(3), -np.ones(3), np.zeros(3), S=32, prune_samples=64)
        a, g = acqf.forward_backward(Xc)
        a2, g2 = acqf.forward_backward(Xc.view(37, 1, 4))     # general path too
        res.append((a, g, a2, g2, acqf.stats.total_cells))
    for r in res[1:]:
        assert all(torch.equal(u, v) for u, v in zip(r[:4], res[0][:4])) and r[4] == res[0][4]


def test_fit_is_deterministic():
    from everest_amd.gp import fit_single

    rng = np.random.default_rng(5)
    X = torch.tensor(rng.uniform(size=(120, 5)), device="cuda")
    y = np.sin(3 * X[:, 0].cpu().numpy()) + 0.1 * rng.normal(size=120)
    hs = []
    for val in (float("nan"), 3.0):
        _poison(val)
        hs.append(fit_single(X, y, 3, ("lognormal", 2.2, 1.73), (-4.0, 1.0)))
    assert np.array_equal(hs[0].lengthscale, hs[1].lengthscale) and hs[0].noise == hs[1].noise


def test_mll_config5_shape_repeatable():
    """n = 2048, d_eff = 32 one-hot-like inputs, Matérn-5/2 (BASELINE configs[4])."""
    from everest_amd.gp import MLLEvaluator

    rng = np.random.default_rng(7)
    Xh = rng.uniform(size=(2048, 32))
    Xh[:, 4:] = (Xh[:, 4:] > 0.85).astype(np.float64)
    Xn = torch.tensor(Xh, device="cuda")
    y = rng.normal(size=2048)
    ev = MLLEvaluator(Xn, y, 3, ("lognormal", 3.1471, 1.7320508), ("lognormal", -4.0, 1.0))
    x = np.r_[2e-4, 0.05, np.log(np.expm1(rng.uniform(0.05, 3.0, size=32)))]
    out = []
    for val in (float("nan"), 1e300, -7.0):
        _poison(val)
        out.append(ev(x))
    for v, g in out[1:]:
        assert v == out[0][0] and np.array_equal(g, out[0][1]), (v - out[0][0], np.abs(g - out[0][1]).max())


def test_posterior_config5_shape_repeatable():
    from everest_amd.gp import GPBatch, GPHyper

    rng = np.random.default_rng(8)
    Xh = rng.uniform(size=(2048, 32))
    Xh[:, 4:] = (Xh[:, 4:] > 0.85).astype(np.float64)
    t = lambda a: torch.tensor(a, device="cuda")  # noqa: E731
    h = GPHyper(lengthscale=rng.uniform(0.05, 3.0, size=32), noise=2e-4, constant=0.1, y_mean=0.0, y_std=1.0)
    Xs = t(rng.uniform(size=(300, 32)))
    res = []
    for val in (float("nan"), 5.0):
        _poison(val)
        gp = GPBatch(t(Xh), t(rng.normal(size=(2048, 1)) * 0 + np.sin(Xh[:, :1] * 5)), [h], 3,
                     t(np.zeros(32)), t(np.ones(32)))
        res.append(gp.posterior(Xs))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
