"""GPU parity of the log-space acquisition functions (qLogNEHVI — MoboStrategy's default —
and qLogEHVI) against the torch-CPU oracle (oracle/qnehvi.py QLogNEHVI / QLogEHVI, autograd
for the gradients) on identical base samples and cells.

The oracle restates BoTorch's fat-smoothed log HVI (fatplus, fatmax/_pareto, logmeanexp) —
parity against BoTorch itself is unpinned (not installable offline); tests/test_oracle.py
checks that the restatement tends to log(qNEHVI) as the temperatures go to 0.
Tolerances: log values 1e-9 absolute (+1e-9 relative), gradients rtol 1e-6."""
import numpy as np
import pytest
import torch

import everest_amd.data_models as dm
from everest_amd import strategies
from everest_amd.benchmarks import DTLZ2
from oracle import qnehvi as oq
from tests.helpers import device_gp, make_problem, oracle_states

pytestmark = pytest.mark.gpu


def _matched(n, d, m, S, seed, prune, nprune=64, ehvi=False):
    from everest_amd.acquisition import QLogEHVI, QLogNEHVI

    X, Y, lo, hi, hyp = make_problem(n=n, d=d, m=m, seed=seed)
    ost = oracle_states(X, Y, lo, hi, hyp)
    gp = device_gp(X, Y, lo, hi, hyp)
    a, b = -np.ones(m), np.zeros(m)
    ref = -1.1 * np.ones(m)
    objective = oq.Objective(torch.tensor(a), torch.tensor(b))
    if ehvi:
        z = oq.base_samples(S, 1, m, 17)
        orc = oq.QLogEHVI(ost, torch.tensor(Y * a + b), objective, torch.tensor(ref), z)
        dq = QLogEHVI(gp, Y * a + b, ref, a, b, S=S, z=z[:, 0, :])
        return X, lo, hi, orc, dq
    Xn = torch.tensor((X - lo) / (hi - lo))
    idx = torch.arange(n)
    zp = oq.base_samples(nprune, n, m, 11)
    if prune:
        idx, _ = oq.prune_baseline(ost, Xn, objective, torch.tensor(ref), zp)
    nb = idx.shape[0]
    zb = oq.base_samples(S, nb, m, 7)
    zn = oq.base_samples(S, nb + 1, m, 7)
    orc = oq.QLogNEHVI(ost, Xn[idx], objective, torch.tensor(ref), zb, zn[:, nb:nb + 1, :])
    dq = QLogNEHVI(gp, X, X, ref, a, b, S=S, prune_baseline=prune, z_prune=zp, z_base_full=zb, z_new_full=zn,
                   prune_samples=nprune)
    return X, lo, hi, orc, dq


def _check(X, lo, hi, orc, dq, d, nc=40, seed=5):
    rng = np.random.default_rng(seed)
    Xc = lo + (hi - lo) * rng.uniform(size=(nc, d))
    Xc[1] = 0.5 * (lo + hi) + 0.45 * (hi - lo)       # far corner: dominated in most samples
    acq, dX = dq.forward_backward(torch.tensor(Xc, device="cuda"))
    xt = torch.tensor(Xc, requires_grad=True)
    ref = orc.forward(((xt - torch.tensor(lo)) / torch.tensor(hi - lo)).unsqueeze(1))
    ref.sum().backward()
    assert torch.isfinite(ref).all() and torch.isfinite(acq).all()
    assert torch.allclose(acq.cpu(), ref.detach(), rtol=1e-9, atol=1e-9), (acq.cpu() - ref.detach()).abs().max()
    assert torch.allclose(dX.cpu(), xt.grad, rtol=1e-6, atol=1e-9 * xt.grad.abs().max()), \
        (dX.cpu() - xt.grad).abs().max()
    fwd = dq.forward(torch.tensor(Xc, device="cuda"))
    assert torch.allclose(fwd, acq, rtol=1e-13, atol=1e-13)       # forward-only plan == fused
    return acq


@pytest.mark.parametrize("n,d,m,S,prune", [(20, 3, 2, 16, False), (40, 4, 3, 32, True), (60, 6, 5, 16, True)])
def test_qlognehvi_forward_backward_parity(n, d, m, S, prune):
    X, lo, hi, orc, dq = _matched(n, d, m, S, seed=n, prune=prune)
    assert dq.state.log_hvi == 1 and dq.log_acqf
    _check(X, lo, hi, orc, dq, d)


@pytest.mark.parametrize("n,d,m,S", [(24, 3, 2, 32), (50, 5, 4, 16)])
def test_qlogehvi_forward_backward_parity(n, d, m, S):
    X, lo, hi, orc, dq = _matched(n, d, m, S, seed=n, prune=False, ehvi=True)
    _check(X, lo, hi, orc, dq, d)


def test_qlognehvi_batch_sizes_and_splits():
    """Small batches split the cell range over workgroups (merged online log-sum-exp
    states): values independent of the batch composition up to rounding."""
    X, lo, hi, orc, dq = _matched(64, 6, 5, 32, seed=2, prune=True)
    rng = np.random.default_rng(9)
    Xc = torch.tensor(lo + (hi - lo) * rng.uniform(size=(300, 6)), device="cuda")
    full = dq.forward(Xc)
    part = torch.cat([dq.forward(Xc[i:i + 7]) for i in range(0, 300, 50)])
    assert torch.allclose(full.view(-1)[[i + k for i in range(0, 300, 50) for k in range(7)]], part,
                          rtol=1e-12, atol=1e-12)
    assert torch.equal(dq.forward(Xc), full)                       # bitwise reproducible


def test_mobo_default_qlognehvi_tell_ask():
    """MoboStrategy() with its default acquisition function (qLogNEHVI) end to end."""
    bench = DTLZ2(dim=6, num_objectives=2)
    rnd = strategies.map(dm.RandomStrategy(domain=bench.domain, seed=4))
    exps = bench.f(rnd.ask(12), return_complete=True)
    s = strategies.map(dm.MoboStrategy(domain=bench.domain, ref_point=bench.ref_point, seed=5,
                                       num_raw_samples=256, num_restarts=4))
    assert isinstance(s.acquisition_function, dm.qLogNEHVI)
    s.tell(exps)
    cand = s.ask(1)
    assert len(cand) == 1
    for k in bench.domain.inputs.get_keys():
        assert 0.0 <= cand[k].iloc[0] <= 1.0
    vals = s.calc_acquisition(cand[bench.domain.inputs.get_keys()])
    assert np.isfinite(vals).all()
