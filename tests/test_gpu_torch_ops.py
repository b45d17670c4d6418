"""The PyTorch-ROCm custom-operator boundary (TORCH_LIBRARY(everest_amd)):
torch.ops.everest_amd.* give the same results as the ctypes C-ABI path, and the
acquisition's autograd wrapper (acqf(X), torch.autograd.Function over qnehvi_forward /
qnehvi_backward) reproduces forward_backward.  Also the surrogate dumps/loads round trip
(bofire/surrogates/botorch.py:66-77; the build's versioned blob)."""
import numpy as np
import pytest
import torch

from tests.helpers import device_gp, make_problem

pytestmark = pytest.mark.gpu


def _ops():
    from everest_amd import torch_ops

    return torch_ops.load()


def test_kernel_matrix_and_cholesky_ops_match_ctypes():
    from everest_amd import ops

    rng = np.random.default_rng(0)
    X1 = torch.tensor(rng.uniform(size=(70, 5)), device="cuda")
    X2 = torch.tensor(rng.uniform(size=(33, 5)), device="cuda")
    ls = torch.tensor(rng.uniform(0.3, 1.2, size=(3, 5)), device="cuda")
    for kind in (0, 1, 2, 3):
        K = _ops().kernel_matrix(X1, X2, ls, kind)
        assert torch.equal(K, ops.kernel_matrix(X1, X2, ls, kind))
    A = ops.kernel_matrix(X1, X1, ls, 0, diag_add=torch.full((3,), 1e-3, dtype=torch.float64, device="cuda"))
    L, jit, info = _ops().cholesky(A, 1e-8, 3)
    L2, jit2, info2 = ops.cholesky(A, 1e-8, 3)
    assert torch.equal(L, L2) and torch.equal(jit, jit2) and int(info.abs().sum()) == 0
    assert torch.allclose(L @ L.transpose(-1, -2), A, rtol=1e-12, atol=1e-13)
    with pytest.raises(RuntimeError):
        _ops().kernel_matrix(X1.float(), X2, ls, 0)      # TORCH_CHECK on dtype


def test_gp_posterior_op_is_the_product_path():
    from everest_amd import ops

    X, Y, lo, hi, hyp = make_problem(n=64, d=4, m=3, seed=1)
    gp = device_gp(X, Y, lo, hi, hyp)
    Xs = torch.tensor(np.random.default_rng(2).uniform(size=(50, 4)), device="cuda")
    for obs in (False, True):
        mean, var = gp.posterior(Xs, observation_noise=obs)            # torch.ops.everest_amd.gp_posterior
        m2, v2 = ops.gp_posterior(gp.Xn, Xs, gp.lo, gp.inv_range, gp.ls, gp.M, gp.kind, gp.const, gp.ym, gp.ys,
                                  gp.kxx, gp.noise if obs else None)
        assert torch.equal(mean, m2) and torch.equal(var, v2)


def _acqf(q_general=False):
    from everest_amd.acquisition import QNEHVI

    X, Y, lo, hi, hyp = make_problem(n=40, d=4, m=3, seed=40)
    gp = device_gp(X, Y, lo, hi, hyp)
    objective = None
    constraints = ()
    if q_general:
        objective = [(0, 0, -1.0, 0.0), (1, 1, 0.5, 1.5)]
        constraints = [(2, -1.0, 0.3, 0.05)]
        ref = [-1.1, -1.0]
    else:
        ref = -1.1 * np.ones(3)
    return QNEHVI(gp, X, X, ref, -np.ones(3), np.zeros(3), S=32, prune_samples=64, objective=objective,
                  constraints=constraints), lo, hi


@pytest.mark.parametrize("general,q", [(False, 1), (False, 2), (True, 1), (True, 3)])
def test_qnehvi_autograd_function(general, q):
    acqf, lo, hi = _acqf(general)
    rng = np.random.default_rng(q)
    shape = (17, 4) if q == 1 and not general else (17, q, 4)
    Xc = torch.tensor(lo + (hi - lo) * rng.uniform(size=shape), device="cuda")
    a_ref, g_ref = acqf.forward_backward(Xc)
    X = Xc.clone().requires_grad_(True)
    w = torch.tensor(rng.uniform(0.5, 2.0, size=17), device="cuda")
    val = acqf(X)
    assert val.grad_fn is not None
    assert torch.allclose(val.detach(), a_ref, rtol=1e-12, atol=0)
    (w * val).sum().backward()
    wshape = (-1,) + (1,) * (X.dim() - 1)
    assert torch.allclose(X.grad, g_ref * w.view(wshape), rtol=1e-12, atol=1e-30)


def test_autograd_launches_the_chain_once_and_caches_plans():
    """acqf(X).sum().backward() runs ONE device chain (qnehvi_forward_backward in the
    autograd forward, the saved dX scaled in backward), the torch-side acquisition caches its
    plan across calls, and it keeps the device state alive on its own."""
    import gc

    acqf, lo, hi = _acqf(False)
    rng = np.random.default_rng(9)
    Xc = torch.tensor(lo + (hi - lo) * rng.uniform(size=(11, 4)), device="cuda")
    a_ref, g_ref = acqf.forward_backward(Xc)
    tacq = acqf._torch_acq(1, True)
    n0 = tacq.evals()
    for k in range(3):
        X = Xc.clone().requires_grad_(True)
        acqf(X).sum().backward()
        assert tacq.evals() == n0 + k + 1          # one chain per forward + backward
        assert torch.equal(X.grad, g_ref)
    assert tacq.cached_plans() == 1
    with torch.no_grad():
        v = acqf(Xc)                                # value only: no gradient chain
    assert torch.equal(v, a_ref) and tacq.evals() == n0 + 4 and tacq.cached_plans() == 2
    # the torch object owns its state: drop every Python reference to the acquisition
    ops = __import__("everest_amd.torch_ops", fromlist=["load"]).load()
    del acqf
    gc.collect()
    torch.cuda.empty_cache()
    junk = torch.randn(1 << 22, dtype=torch.float64, device="cuda")   # reuse freed memory
    a2, g2 = ops.qnehvi_forward_backward(tacq, Xc)
    assert torch.equal(a2, a_ref) and torch.equal(g2, g_ref)
    del junk


def test_surrogate_dumps_loads_round_trip():
    import everest_amd.data_models as dm
    from everest_amd import strategies, surrogates
    from everest_amd.benchmarks import DTLZ2

    bench = DTLZ2(dim=4, num_objectives=2)
    X = strategies.map(dm.RandomStrategy(domain=bench.domain, seed=1)).ask(20)
    exps = bench.f(X, return_complete=True)
    spec = dm.SingleTaskGPSurrogate(inputs=bench.domain.inputs,
                                    outputs=dm.Outputs(features=[bench.domain.outputs.get_by_key("f_0")]))
    s = surrogates.map(spec)
    s.fit(exps)
    blob = s.dumps()
    assert isinstance(blob, str)
    s2 = surrogates.map(spec)
    s2.loads(blob)
    Xq = strategies.map(dm.RandomStrategy(domain=bench.domain, seed=2)).ask(25)
    p1, p2 = s.predict(Xq), s2.predict(Xq)
    assert np.array_equal(p1.values, p2.values)
    with pytest.raises(ValueError):
        s2.loads("e30=")                                   # "{}": unknown format
