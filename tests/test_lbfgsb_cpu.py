"""The native L-BFGS-B (everest_amd/csrc/lbfgsb.cpp, host-only) against scipy's L-BFGS-B,
the optimiser [upstream] gen_candidates_scipy runs for the acquisition restarts
(bofire/strategies/predictives/botorch.py:384-405): same optimum and — the algorithm being
the same — the same iteration and evaluation counts on smooth problems with active bounds."""
import numpy as np
import pytest
from scipy.optimize import minimize, rosen, rosen_der

from everest_amd.optim import minimize_lbfgsb


def _both(fun, x0, lb, ub, maxiter=2000):
    r1 = minimize(fun, x0, jac=True, method="L-BFGS-B", bounds=list(zip(lb, ub)), options={"maxiter": maxiter})
    r2 = minimize_lbfgsb(fun, x0, lb, ub, maxiter=maxiter)
    return r1, r2


def _rosen(x):
    return rosen(x), rosen_der(x)


@pytest.mark.parametrize("n", [2, 5, 10])
@pytest.mark.parametrize("upper", [2.0, 0.5])
def test_rosenbrock_matches_scipy(n, upper):
    x0 = np.random.default_rng(n).uniform(-2, 2, n)
    lb, ub = -2 * np.ones(n), upper * np.ones(n)
    r1, r2 = _both(_rosen, x0, lb, ub)
    assert r2.status == 0
    assert (r2.nit, r2.nfev) == (r1.nit, r1.nfev)
    assert np.allclose(r2.x, r1.x, atol=1e-7)
    assert abs(r2.fun - r1.fun) <= 1e-9 * max(1.0, abs(r1.fun))


def test_quadratic_with_active_bounds_matches_scipy():
    rng = np.random.default_rng(3)
    A = rng.normal(size=(20, 20))
    Q = A @ A.T + 0.1 * np.eye(20)
    c = 5 * rng.normal(size=20)
    fun = lambda x: (0.5 * x @ Q @ x + c @ x, Q @ x + c)  # noqa: E731
    r1, r2 = _both(fun, np.zeros(20), -np.ones(20), np.ones(20))
    assert (r2.nit, r2.nfev) == (r1.nit, r1.nfev)
    assert np.allclose(r2.x, r1.x, atol=1e-10)
    assert ((np.abs(r2.x) == 1.0).sum()) > 0          # some bounds are active at the optimum


def _multi(x):
    """-sum over restarts of a bimodal acquisition-like surface (the joint restart problem)."""
    X = x.reshape(-1, 3)
    e1 = np.exp(-((X - 0.3) ** 2).sum(-1) * 8)
    e2 = np.exp(-((X - 0.8) ** 2).sum(-1) * 20)
    g = -16 * (X - 0.3) * e1[:, None] - 20 * (X - 0.8) * e2[:, None]
    return -(e1 + 0.5 * e2).sum(), -g.reshape(-1)


def test_joint_restarts_match_scipy():
    x0 = np.random.default_rng(1).uniform(size=5 * 3)
    r1, r2 = _both(_multi, x0, np.zeros(15), np.ones(15))
    assert (r2.nit, r2.nfev) == (r1.nit, r1.nfev)
    assert np.allclose(r2.x, r1.x, atol=1e-8)


def test_maxiter_and_projection_of_x0():
    x0 = np.array([3.0, -3.0])                       # outside the box: projected first
    r = minimize_lbfgsb(_rosen, x0, -np.ones(2), np.ones(2), maxiter=3)
    assert r.status == 1 and r.nit == 3
    assert np.all(np.abs(r.x) <= 1.0)


def test_converged_at_start_and_fixed_variables():
    # projected gradient zero at a corner: converges before any iteration
    r = minimize_lbfgsb(lambda x: (float(x.sum()), np.ones(2)), np.zeros(2), np.zeros(2), np.ones(2))
    assert r.status == 0 and r.nit == 0 and r.nfev == 1
    # lb == ub fixes a variable
    r = minimize_lbfgsb(_rosen, np.array([0.0, 0.5]), np.array([-2.0, 0.5]), np.array([2.0, 0.5]))
    assert r.x[1] == 0.5 and r.status == 0


def test_bad_bounds_raise():
    with pytest.raises(RuntimeError):
        minimize_lbfgsb(_rosen, np.zeros(2), np.ones(2), np.zeros(2))


@pytest.mark.parametrize("which", ["value", "gradient"])
def test_nonfinite_trial_points_are_rejected(which):
    """A line-search trial whose value or gradient is not finite (an overflowing MLL
    gradient during the GP fit) is rejected and the search retried with a shorter step: no
    NaN reaches an iterate, the optimum of the finite region is found."""
    seen = []

    def fun(x):
        seen.append(x.copy())
        f, g = float(np.sum((x - 3.0) ** 2)), 2.0 * (x - 3.0)
        if np.any(x > 2.5):
            if which == "value":
                f = float("nan")
            else:
                g = np.full_like(x, np.inf)
        else:
            f += float(np.sum(np.exp(-20.0 * (2.5 - x))))       # a wall at 2.5
            g = g - 20.0 * np.exp(-20.0 * (2.5 - x)) * -1.0
        return f, g

    x0 = np.zeros(3)
    r = minimize_lbfgsb(fun, x0, np.full(3, -np.inf), np.full(3, np.inf), maxiter=200)
    assert all(np.all(np.isfinite(x)) for x in seen)
    assert np.all(np.isfinite(r.x)) and np.isfinite(r.fun)
    assert np.all(r.x <= 2.5) and np.all(r.x > 2.0)


def test_raw_sample_prefetch_equals_direct_draw():
    """optim.prefetch_raw_samples peeks at the generator's next seed and draws the raw Sobol
    samples on a worker thread; the future optimize_acqf takes holds exactly the direct draw,
    and the real generator is not advanced by the peek."""
    import numpy as np
    import torch

    from everest_amd import optim

    g = torch.Generator().manual_seed(11)
    state = g.get_state()
    bounds = np.array([[0.0, -1.0, 2.0], [1.0, 1.0, 5.0]])
    optim.prefetch_raw_samples(bounds, 256, g, q=2)
    assert torch.equal(g.get_state(), state)
    seed = int(torch.randint(10_000_000, (1,), generator=g).item())
    fut = optim._RAW_PREFETCHED.pop(optim._raw_key(bounds, 256, seed, 2))
    assert np.array_equal(fut.result(), optim.draw_sobol_samples(bounds, 256, seed, 2))
