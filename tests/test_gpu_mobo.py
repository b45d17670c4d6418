"""Re-expressions of the reference's MoboStrategy tests (tests/bofire/strategies/
test_mobo.py:78-160) on the device acquisitions: the acquisition class per data model,
with and without a reference point, and on the constrained C2DTLZ2 benchmark the one output
constraint with eta = 1e-3 and the adjusted reference point [-1.1, -1.1].  Beyond the
reference's type checks, the constrained acquisitions' values are compared with the oracle on
the same states, base samples and cells (qLog*: the fat-tailed log feasibility)."""
import numpy as np
import pytest
import torch

import everest_amd.data_models as dm
from everest_amd import strategies
from everest_amd.acquisition import QEHVI, QNEHVI, QLogEHVI, QLogNEHVI
from everest_amd.benchmarks import C2DTLZ2, DTLZ2
from oracle import gp as ogp
from oracle import qnehvi as oq

pytestmark = pytest.mark.gpu

ACQFS = [(dm.qEHVI, QEHVI), (dm.qLogEHVI, QLogEHVI), (dm.qNEHVI, QNEHVI), (dm.qLogNEHVI, QLogNEHVI)]


def _exact(acqf, cls):
    # QLogNEHVI subclasses QNEHVI: compare the exact type
    return type(acqf) is cls


@pytest.mark.parametrize("use_ref_point", [True, False])
@pytest.mark.parametrize("acqf_dm,cls", ACQFS)
def test_mobo(use_ref_point, acqf_dm, cls):
    """test_mobo.py:78-120: DTLZ2(dim=6), 10 random experiments, _get_acqfs(2)."""
    bm = DTLZ2(dim=6)
    rnd = strategies.map(dm.RandomStrategy(domain=bm.domain, seed=2))
    exps = bm.f(rnd.ask(candidate_count=10), return_complete=True)
    s = strategies.map(dm.MoboStrategy(domain=bm.domain, ref_point=bm.ref_point if use_ref_point else None,
                                       acquisition_function=acqf_dm(n_mc_samples=64), seed=4))
    s.tell(exps)
    acqf = s._get_acqfs(2)[0]
    assert _exact(acqf, cls)
    assert acqf.constraints == [] and acqf.eta is None
    if use_ref_point:
        assert torch.allclose(acqf.ref_point.cpu(), torch.tensor([-1.1, -1.1], dtype=torch.float64))


def _oracle_states(s):
    out = []
    for sur in s.surrogates.surrogates:
        st = sur.state
        y = torch.tensor(st["y"])
        out.append(ogp.GPState(X=torch.tensor((st["X"] - st["lo"]) / (st["hi"] - st["lo"])),
                               y=(y - st["y_mean"]) / st["y_std"], lengthscale=torch.tensor(st["lengthscale"]),
                               noise=st["noise"], constant=st["constant"], y_mean=st["y_mean"], y_std=st["y_std"],
                               kind=st["kind"], lo=torch.tensor(st["lo"]), hi=torch.tensor(st["hi"])))
    return out


@pytest.mark.parametrize("acqf_dm,cls", ACQFS)
def test_mobo_constraints(acqf_dm, cls):
    """test_mobo.py:123-160: C2DTLZ2(dim=4), ref {f_0: 1.1, f_1: 1.1}: one constraint, eta 1e-3,
    ref point [-1.1, -1.1]; then the q = 1 acquisition values against the oracle."""
    bm = C2DTLZ2(dim=4)
    rnd = strategies.map(dm.RandomStrategy(domain=bm.domain, seed=5))
    exps = bm.f(rnd.ask(10), return_complete=True)
    s = strategies.map(dm.MoboStrategy(domain=bm.domain, ref_point={"f_0": 1.1, "f_1": 1.1},
                                       acquisition_function=acqf_dm(n_mc_samples=32), seed=7))
    s.tell(exps)
    acqf2 = s._get_acqfs(2)[0]
    assert _exact(acqf2, cls)
    assert float(acqf2.eta) == pytest.approx(1e-3, rel=1e-12)
    assert len(acqf2.constraints) == 1
    assert torch.allclose(acqf2.ref_point.cpu(), torch.tensor([-1.1, -1.1], dtype=torch.double))

    # values at q = 1 against the oracle with the same partition input / base samples
    acqf = s._get_acqfs(1)[0]
    ost = _oracle_states(s)
    keys = s.model.output_keys
    islack = keys.index("slack")
    obj_out = [keys.index("f_0"), keys.index("f_1")]
    oobj = oq.GeneralObjective(out=obj_out, kind=[0, 0], p0=[-1.0, -1.0], p1=[0.0, 0.0])
    (o, sg, t, e), = acqf.constraints
    assert o == islack
    ocon = oq.OutputConstraints(out=[o], sign=[sg], thr=[t], eta=[e])
    ref = acqf.ref_point.cpu()
    m = len(keys)
    if cls in (QNEHVI, QLogNEHVI):
        Xb = torch.tensor(s.model.X_raw[acqf.base_rows])
        zb = acqf.z_base_host()
        zn = acqf.zq.cpu().reshape(acqf.S, 1, m)
        ocls = oq.QNEHVI if cls is QNEHVI else oq.QLogNEHVI
        orc = ocls(ost, Xb, oobj, ref, zb, zn, constraints=ocon, raw=True)
        assert acqf.stats.total_cells == sum(c.shape[1] for c in orc.cells)
    else:
        # the oracle's qEHVI takes normalised inputs: Normalize bounds are the feature bounds
        # [0, 1] here (feature bounds U data), so raw = normalised
        for st in ost:
            assert torch.equal(st.lo, torch.zeros(4, dtype=torch.float64)) and torch.equal(st.hi, torch.ones(4, dtype=torch.float64))
        z = acqf.zq.cpu().reshape(acqf.S, 1, m)
        ocls = oq.QEHVI if cls is QEHVI else oq.QLogEHVI
        orc = ocls(ost, torch.tensor(acqf.Y_part), oobj, ref, z, constraints=ocon)
    Xc = np.random.default_rng(3).uniform(size=(9, 4))
    a = acqf.forward(torch.tensor(Xc, device="cuda")).cpu()
    r = orc.forward(torch.tensor(Xc).unsqueeze(1)).detach()
    assert torch.isfinite(a).all()
    tol = dict(rtol=1e-9, atol=1e-9) if cls in (QLogNEHVI, QLogEHVI) else dict(rtol=1e-6, atol=1e-10)
    assert torch.allclose(a, r, **tol), (a, r)
