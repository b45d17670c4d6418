"""The restart optimiser on the device acquisition: the all-C++ L-BFGS-B loop over the
native plan (evr_qnehvi_plan_minimize) against the same L-BFGS-B driven from Python through
eval_host, and against scipy's L-BFGS-B (the optimiser [upstream] gen_candidates_scipy runs,
bofire/strategies/predictives/botorch.py:384-405)."""
import numpy as np
import pytest
import torch

from tests.helpers import device_gp, make_problem

pytestmark = pytest.mark.gpu


class _NoPlan:
    """The same acquisition without ``plan``: optimize_acqf falls back to the Python-driven
    native L-BFGS-B over eval_host."""

    def __init__(self, a):
        self.a, self.dev = a, a.dev

    def forward(self, X):
        return self.a.forward(X)

    def forward_backward(self, X):
        return self.a.forward_backward(X)

    def eval_host(self, x, backward):
        return self.a.eval_host(x, backward)


def _acqf():
    from everest_amd.acquisition import QNEHVI

    X, Y, lo, hi, hyp = make_problem(n=60, d=6, m=3, seed=4)
    gp = device_gp(X, Y, lo, hi, hyp)
    m = 3
    return QNEHVI(gp, X, X, -1.1 * np.ones(m), -np.ones(m), np.zeros(m), S=64, sampler_seed=3, prune_seed=5), lo, hi


def test_plan_minimize_equals_python_driven_lbfgsb():
    from everest_amd.optim import optimize_acqf

    acqf, lo, hi = _acqf()
    bounds = np.stack([lo, hi])
    opts = {"batch_limit": 8, "maxiter": 2000}
    x1, v1, s1 = optimize_acqf(acqf, bounds, 8, 256, opts, torch.Generator().manual_seed(1))
    x2, v2, s2 = optimize_acqf(_NoPlan(acqf), bounds, 8, 256, opts, torch.Generator().manual_seed(1))
    assert s1.chunks[0]["driver"] == "native-plan" and s2.chunks[0]["driver"] == "native"
    assert np.array_equal(x1, x2) and v1 == v2
    assert s1.chunks[0]["evals"] == s2.chunks[0]["evals"] and s1.chunks[0]["nit"] == s2.chunks[0]["nit"]
    assert v1 > 0


def test_native_lbfgsb_tracks_scipy_on_the_acquisition():
    from everest_amd.optim import optimize_acqf

    acqf, lo, hi = _acqf()
    bounds = np.stack([lo, hi])
    x1, v1, s1 = optimize_acqf(acqf, bounds, 4, 128, {"batch_limit": 4, "maxiter": 2000},
                               torch.Generator().manual_seed(2))
    x2, v2, s2 = optimize_acqf(acqf, bounds, 4, 128, {"batch_limit": 4, "maxiter": 2000, "optimizer": "scipy"},
                               torch.Generator().manual_seed(2))
    # same algorithm: the optimum agrees to the line-search tolerance scale
    assert abs(v1 - v2) <= 1e-6 * max(1.0, abs(v2))
    assert np.allclose(x1, x2, atol=1e-4)


@pytest.mark.parametrize("backward", [False, True])
def test_plan_eval_host_matches_device_evaluation(backward):
    """evr_qnehvi_plan_eval_host (x from / [acq | dX] to pinned host memory inside the graph,
    completion word instead of a stream synchronise) returns exactly the device chain's
    values, evaluation after evaluation."""
    acqf, lo, hi = _acqf()
    rng = np.random.default_rng(9)
    b, d = 8, len(lo)
    p = acqf.plan(b, backward)
    for _ in range(5):
        x = lo + (hi - lo) * rng.uniform(size=(b, d))
        out = p.run_host(x).copy()
        Xd = torch.tensor(x, device="cuda")
        if backward:
            a, g = acqf.forward_backward(Xd)
            assert np.array_equal(out[b:].reshape(b, d), g.cpu().numpy())
        else:
            a = acqf.forward(Xd)
        assert np.array_equal(out[:b], a.cpu().numpy())


def test_recycled_host_graph_matches_device_chain():
    """A restart plan built after another plan of the same shape was destroyed takes over its
    pinned buffers and graph executable (hipGraphExecUpdate with the new chain's arguments):
    its host evaluations equal the new acquisition's device-mode chain bitwise."""
    import gc

    from everest_amd.acquisition import QNEHVI

    X, Y, lo, hi, hyp = make_problem(n=60, d=6, m=3, seed=4)
    gp = device_gp(X, Y, lo, hi, hyp)
    x = np.random.default_rng(1).uniform(lo, hi, size=(8, 6))
    m = 3
    a1 = QNEHVI(gp, X, X, -1.1 * np.ones(m), -np.ones(m), np.zeros(m), S=64, sampler_seed=3, prune_seed=5)
    a1.plan(8, True).run_host(x)
    a1._plans.clear()
    del a1
    gc.collect()
    a2 = QNEHVI(gp, X, X, -1.1 * np.ones(m), -np.ones(m), np.zeros(m), S=64, sampler_seed=11, prune_seed=7)
    out = a2.plan(8, True).run_host(x).copy()
    acq, dX = a2.forward_backward(torch.tensor(x, device="cuda"))
    assert np.array_equal(out[:8], acq.cpu().numpy())
    assert np.array_equal(out[8:8 + 48].reshape(8, 6), dX.cpu().numpy())
    out2 = a2.plan(8, True).run_host(x)
    assert np.array_equal(out2[:56], out[:56])
