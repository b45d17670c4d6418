"""GPU parity of qEHVI (QehviStrategy / MoboStrategy(qEHVI)) and the MoboStrategy end to end.

The device qEHVI runs the qNEHVI kernels with nb = 0 and no H^T rows (state.no_h = 1); its
values and gradients are compared with the torch-CPU oracle (oracle/qnehvi.py QEHVI, itself
checked against exact HV differences in tests/test_oracle.py) on identical base samples.
Tolerances: values rtol 1e-6 (north-star bar 1e-3), gradients rtol 1e-5."""
import numpy as np
import pandas as pd
import pytest
import torch

import everest_amd.data_models as dm
from everest_amd import strategies
from everest_amd.benchmarks import DTLZ2
from oracle import qnehvi as oq
from tests.helpers import device_gp, make_problem, oracle_states

pytestmark = pytest.mark.gpu


def _matched_qehvi(n, d, m, S, seed, ref_scale=1.1, shift_ref=False):
    from everest_amd.acquisition import QEHVI

    X, Y, lo, hi, hyp = make_problem(n=n, d=d, m=m, seed=seed)
    ost = oracle_states(X, Y, lo, hi, hyp)
    gp = device_gp(X, Y, lo, hi, hyp)
    a, b = -np.ones(m), np.zeros(m)
    ref = -ref_scale * np.ones(m)
    if shift_ref:                  # a reference point that most observations fail (7 of 40 pass)
        ref = np.quantile(Y * a + b, 0.3, axis=0)
    Yp = Y * a + b
    z = oq.base_samples(S, 1, m, 17)
    orc = oq.QEHVI(ost, torch.tensor(Yp), oq.Objective(torch.tensor(a), torch.tensor(b)), torch.tensor(ref), z)
    dq = QEHVI(gp, Yp, ref, a, b, S=S, z=z[:, 0, :])
    return X, lo, hi, orc, dq


@pytest.mark.parametrize("n,d,m,S,shift", [(20, 3, 2, 16, False), (40, 4, 3, 32, True), (64, 6, 5, 64, False)])
def test_qehvi_forward_backward_parity(n, d, m, S, shift):
    X, lo, hi, orc, dq = _matched_qehvi(n, d, m, S, seed=n, shift_ref=shift)
    assert dq.state.no_h == 1 and dq.Rr == n + 1
    assert dq.stats.total_cells == S * orc.cell.shape[1]       # one partition, replicated per sample
    rng = np.random.default_rng(4)
    Xc = lo + (hi - lo) * rng.uniform(size=(45, d))
    acq, dX = dq.forward_backward(torch.tensor(Xc, device="cuda"))
    xt = torch.tensor(Xc, requires_grad=True)
    ref = orc.forward(((xt - torch.tensor(lo)) / torch.tensor(hi - lo)).unsqueeze(1))
    ref.sum().backward()
    assert (ref > 0).any()
    assert torch.allclose(acq.cpu(), ref.detach(), rtol=1e-6, atol=1e-10)
    assert torch.allclose(dX.cpu(), xt.grad, rtol=1e-5, atol=1e-8)
    # op-by-op chain and native plan agree
    a2, d2 = dq.forward_backward_ops(torch.tensor(Xc, device="cuda"))
    assert torch.allclose(a2, acq, rtol=1e-12, atol=1e-15)
    assert torch.allclose(d2, dX, rtol=1e-10, atol=1e-13)


def test_qehvi_empty_front_single_cell():
    """Empty Pareto set (no observation better than ref): one cell [ref, inf) per sample, the
    acquisition is the expected volume dominated by the sample above ref."""
    from everest_amd.acquisition import QEHVI

    X, Y, lo, hi, hyp = make_problem(n=24, d=3, m=2, seed=5)
    ost = oracle_states(X, Y, lo, hi, hyp)
    gp = device_gp(X, Y, lo, hi, hyp)
    a, b = np.ones(2), np.zeros(2)
    ref = np.quantile(Y, 0.5, axis=0)
    z = oq.base_samples(32, 1, 2, 3)
    dq = QEHVI(gp, np.zeros((0, 2)), ref, a, b, S=32, z=z[:, 0, :])
    assert dq.box_path == "none"
    orc = oq.QEHVI(ost, torch.zeros(0, 2, dtype=torch.float64), oq.Objective(torch.tensor(a), torch.tensor(b)),
                   torch.tensor(ref), z)
    Xc = torch.tensor(lo + (hi - lo) * np.random.default_rng(0).uniform(size=(9, 3)))
    v = dq.forward(Xc.cuda()).cpu()
    r = orc.forward(((Xc - torch.tensor(lo)) / torch.tensor(hi - lo)).unsqueeze(1))
    assert torch.allclose(v, r, rtol=1e-9, atol=1e-14)
    assert (r > 0).any()


def _dtlz2_experiments(n=12, dim=6, m=2, seed=0):
    bench = DTLZ2(dim=dim, num_objectives=m)
    rnd = strategies.map(dm.RandomStrategy(domain=bench.domain, seed=seed))
    X = rnd.ask(n)
    return bench, bench.f(X, return_complete=True)


def _check_candidate(bench, cand):
    assert len(cand) == 1
    for k in bench.domain.inputs.get_keys():
        assert 0.0 <= cand[k].iloc[0] <= 1.0
    for k in bench.domain.outputs.get_keys():
        for suf in ("_pred", "_sd", "_des"):
            assert f"{k}{suf}" in cand.columns


def test_qehvi_strategy_tell_ask():
    """QehviStrategy (bofire/strategies/predictives/qehvi.py): partition of the masked
    observations better than the reference point; ask -> candidate with predictions."""
    bench, exps = _dtlz2_experiments()
    s = strategies.map(dm.QehviStrategy(domain=bench.domain, ref_point=bench.ref_point, seed=3,
                                        num_sobol_samples=128, num_raw_samples=256, num_restarts=4))
    s.tell(exps)
    cand = s.ask(1)
    _check_candidate(bench, cand)
    acqf = s.last_acqf
    assert acqf.state.no_h == 1 and acqf.S == 128
    vals = s.calc_acquisition(pd.concat([cand[bench.domain.inputs.get_keys()], exps.iloc[:3]], ignore_index=True))
    assert vals.shape == (4,) and (vals >= 0).all() and vals[0] > 0


@pytest.mark.parametrize("acqf", ["qEHVI", "qNEHVI"])
def test_mobo_strategy_tell_ask(acqf):
    """MoboStrategy with the device acquisition functions (bofire/strategies/predictives/mobo.py:44-90)."""
    bench, exps = _dtlz2_experiments(seed=1)
    af = getattr(dm, acqf)(n_mc_samples=64)
    s = strategies.map(dm.MoboStrategy(domain=bench.domain, ref_point=bench.ref_point, seed=5,
                                       acquisition_function=af, num_raw_samples=256, num_restarts=4))
    s.tell(exps)
    cand = s.ask(1)
    _check_candidate(bench, cand)
    assert s.last_acqf.S == 64
    assert s.last_ask_stats.raw_evals == 256
