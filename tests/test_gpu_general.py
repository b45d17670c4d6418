"""GPU parity of the general qNEHVI / qEHVI evaluation (qnehvi_general.hip) against the
torch-CPU oracle: q > 1 joint batches (inclusion–exclusion over q-subsets, joint q x q
new-block Cholesky), objectives over selected outputs incl. CloseToTarget, output
constraints with sigmoid feasibility weights, qEHVI pending points.

Reference semantics: optimize_acqf(q=candidate_count) (bofire/strategies/predictives/
botorch.py:385), get_multiobjective_objective / get_output_constraints
(bofire/utils/torch_tools.py:258-402, 699-727), constraints / eta at
bofire/strategies/predictives/qnehvi.py:28-48.  Tolerances: values 1e-6 relative,
gradients 1e-5 relative vs oracle autograd (north star: 1e-3 on qNEHVI values)."""
import numpy as np
import pytest
import torch

from oracle import qnehvi as oq
from tests.helpers import device_gp, make_problem, oracle_states

pytestmark = pytest.mark.gpu


def _setup(n, d, m, S, seed, q, prune, objective=None, constraints=None, ref=None, nprune=64, ls_scale=1.0):
    """Matched device / oracle qNEHVI with base samples for q new points."""
    from everest_amd.acquisition import QNEHVI

    X, Y, lo, hi, hyp = make_problem(n=n, d=d, m=m, seed=seed)
    for h in hyp:
        h["lengthscale"] = h["lengthscale"] * ls_scale
    ost = oracle_states(X, Y, lo, hi, hyp)
    gp = device_gp(X, Y, lo, hi, hyp)
    if objective is None:
        objective = [(j, 0, -1.0, 0.0) for j in range(m)]
    mo = len(objective)
    ref = -1.1 * np.ones(mo) if ref is None else np.asarray(ref, dtype=np.float64)
    oobj = oq.GeneralObjective(*[list(t) for t in zip(*objective)])
    ocon = None if not constraints else oq.OutputConstraints(*[list(t) for t in zip(*constraints)])
    Xn = torch.tensor((X - lo) / (hi - lo))
    idx = torch.arange(n)
    zp = oq.base_samples(nprune, n, m, 11)
    if prune:
        idx, _ = oq.prune_baseline(ost, Xn, oobj, torch.tensor(ref), zp, constraints=ocon)
    nb = idx.shape[0]
    zb = oq.base_samples(S, nb, m, 7)
    zn = oq.base_samples(S, nb + q, m, 7)
    orc = oq.QNEHVI(ost, Xn[idx], oobj, torch.tensor(ref), zb, zn[:, nb:nb + q, :], constraints=ocon)
    dq = QNEHVI(gp, X, X, ref, None, None, S=S, prune_baseline=prune, z_prune=zp, z_base_full=zb, z_new_full=zn,
                prune_samples=nprune, objective=objective, constraints=constraints or ())
    return X, lo, hi, orc, dq, idx


def _check(dq, orc, lo, hi, Xc, rtol=1e-6, gtol=1e-5):
    acq, dX = dq.forward_backward(torch.tensor(Xc, device="cuda"))
    xt = torch.tensor(Xc, requires_grad=True)
    xn = (xt - torch.tensor(lo)) / torch.tensor(hi - lo)
    ref = orc.forward(xn if xn.dim() == 3 else xn.unsqueeze(1))
    ref.sum().backward()
    a, r = acq.cpu(), ref.detach()
    assert (r > 0).sum() >= 2, r
    assert torch.allclose(a, r, rtol=rtol, atol=1e-9 * r.abs().max()), (a - r).abs().max()
    g = dX.cpu()
    assert g.shape == xt.grad.shape
    assert torch.allclose(g, xt.grad, rtol=gtol, atol=1e-7 * xt.grad.abs().max()), (g - xt.grad).abs().max()
    fwd = dq.forward(torch.tensor(Xc, device="cuda"))
    assert torch.allclose(fwd, acq, rtol=1e-12, atol=0)
    return a, r


def test_general_q1_equals_fast_path():
    """The general kernels at q = 1 with affine objectives on every output reproduce the
    fused fast path (same samples, same scan; the Gram / Cholesky order differs)."""
    X, lo, hi, orc, dq, _ = _setup(40, 4, 3, 32, seed=40, q=1, prune=True)
    assert dq.supports_plan
    Xc = lo + (hi - lo) * np.random.default_rng(2).uniform(size=(23, 4))
    Xt = torch.tensor(Xc, device="cuda")
    a_fast, g_fast = dq.forward_backward(Xt)
    a_gen, g_gen = dq._general(Xt.unsqueeze(1), True)
    assert torch.allclose(a_gen, a_fast, rtol=1e-9, atol=1e-12 * a_fast.abs().max())
    assert torch.allclose(g_gen[:, 0], g_fast, rtol=1e-7, atol=1e-10 * g_fast.abs().max())


@pytest.mark.parametrize("q", [2, 3])
@pytest.mark.parametrize("n,d,m,S", [(30, 3, 2, 16), (50, 5, 3, 24)])
def test_qnehvi_joint_batches(q, n, d, m, S):
    X, lo, hi, orc, dq, _ = _setup(n, d, m, S, seed=n + q, q=q, prune=True)
    rng = np.random.default_rng(q)
    Xc = lo + (hi - lo) * rng.uniform(size=(11, q, d))
    _check(dq, orc, lo, hi, Xc)


def test_qnehvi_q4():
    """q = 4 (15 subsets).  The candidates must not repeat baseline points: a baseline point in
    a q-batch has zero conditional variance, and the psd_safe_cholesky jitter rung chosen for
    the singular block — here and in the reference — is decided by rounding noise."""
    X, lo, hi, orc, dq, _ = _setup(30, 4, 2, 12, seed=4, q=4, prune=True, ls_scale=0.5)
    Xc = lo + (hi - lo) * np.random.default_rng(104).uniform(size=(5, 4, 4))
    _check(dq, orc, lo, hi, Xc)


@pytest.mark.parametrize("q", [1, 2])
def test_qnehvi_constraints_close_to_target(q):
    """3 model outputs: Minimize on output 0, CloseToTarget(0.5, e=1.5) on output 1,
    output 2 constraint-only (MaximizeSigmoid tp=0.3 -> c = -(y - 0.3), eta 0.05) plus a
    MinimizeSigmoid-style bound on output 0 (c = y - 0.9, eta 0.1)."""
    objective = [(0, 0, -1.0, 0.0), (1, 1, 0.5, 1.5)]
    constraints = [(2, -1.0, 0.3, 0.05), (0, 1.0, 0.9, 0.1)]
    X, lo, hi, orc, dq, idx = _setup(45, 4, 3, 24, seed=9 + q, q=q, prune=True, objective=objective,
                                     constraints=constraints, ref=[-1.1, -1.0])
    assert not dq.supports_plan
    assert np.array_equal(np.sort(dq.base_rows), idx.numpy())
    assert dq.stats.total_cells == sum(c.shape[1] for c in orc.cells)
    rng = np.random.default_rng(7)
    Xc = lo + (hi - lo) * rng.uniform(size=(13, q, 4) if q > 1 else (13, 4))
    _check(dq, orc, lo, hi, Xc)


def test_qehvi_joint_batch_with_pending():
    """qEHVI: the pending point joins every candidate's joint batch (q = 2 + 1 pending)."""
    from everest_amd.acquisition import QEHVI

    n, d, m, S, q = 30, 3, 2, 16, 2
    X, Y, lo, hi, hyp = make_problem(n=n, d=d, m=m, seed=12)
    ost = oracle_states(X, Y, lo, hi, hyp)
    gp = device_gp(X, Y, lo, hi, hyp)
    a, b = -np.ones(m), np.zeros(m)
    ref = -1.1 * np.ones(m)
    Ypart = Y * a + b
    Ypart = Ypart[(Ypart > ref).all(-1)]
    Xp = lo + (hi - lo) * np.random.default_rng(3).uniform(size=(1, d))
    z = oq.base_samples(S, q + 1, m, 5)
    dq = QEHVI(gp, Ypart, ref, a, b, S=S, X_pending_raw=Xp)
    dq.set_new_point_samples(q + 1, z)
    orc = oq.QEHVI(ost, torch.tensor(Ypart), oq.Objective(torch.tensor(a), torch.tensor(b)), torch.tensor(ref), z,
                   X_pending=torch.tensor((Xp - lo) / (hi - lo)))
    Xc = lo + (hi - lo) * np.random.default_rng(8).uniform(size=(9, q, d))
    _check(dq, orc, lo, hi, Xc)


@pytest.mark.parametrize("q", [9, 10])
def test_qnehvi_joint_batch_above_eight(q):
    """q > 8 (the reference passes optimize_acqf(q=candidate_count) with no cap): 2^q - 1
    subsets through the same kernels (QG Q = 9..12), against the oracle's inclusion-exclusion."""
    X, lo, hi, orc, dq, _ = _setup(24, 3, 2, 8, seed=90 + q, q=q, prune=True, ls_scale=0.5)
    Xc = lo + (hi - lo) * np.random.default_rng(q).uniform(size=(3, q, 3))
    _check(dq, orc, lo, hi, Xc)


def test_joint_batch_limit_message():
    """Beyond the device limit the error names the limit (the subset count is 2^q - 1)."""
    from everest_amd import ops

    X, lo, hi, orc, dq, _ = _setup(20, 3, 2, 8, seed=3, q=2, prune=False)
    q = ops.QNG_MAX_Q + 1
    Xc = torch.tensor(lo + (hi - lo) * np.random.default_rng(0).uniform(size=(1, q, 3)), device="cuda")
    with pytest.raises(ValueError, match=f"device limit of {ops.QNG_MAX_Q}"):
        dq.forward(Xc)
