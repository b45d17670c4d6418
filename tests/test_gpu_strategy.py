"""End-to-end BoFire-API tests on the MI355X: tell -> fit on device -> ask -> candidates,
mirroring tests/bofire/strategies/test_qehvi.py:133-193 and test_ask.py:85-147 of the
reference (types, shapes, ref point, constraint satisfaction), plus oracle parity of the
fitted posterior and of the device GP fit."""
import numpy as np
import pandas as pd
import pytest
import torch

import everest_amd.data_models as dm
from everest_amd import strategies
from everest_amd.benchmarks import DTLZ2, Detergent
from oracle import gp as ogp

pytestmark = pytest.mark.gpu


def _dtlz2_experiments(n=10, dim=6, m=2, seed=17):
    bench = DTLZ2(dim=dim, num_objectives=m)
    rnd = strategies.map(dm.RandomStrategy(domain=bench.domain, seed=seed))
    X = rnd.ask(n)
    return bench, bench.f(X, return_complete=True)


@pytest.mark.parametrize("use_ref_point", [True, False])
def test_qnehvi_tell_ask_dtlz2(use_ref_point):
    bench, exps = _dtlz2_experiments()
    data_model = dm.QnehviStrategy(domain=bench.domain, ref_point=bench.ref_point if use_ref_point else None,
                                   seed=42, num_sobol_samples=128, num_raw_samples=256, num_restarts=4)
    s = strategies.map(data_model)
    s.tell(exps)
    assert s.is_fitted
    ref = s.get_adjusted_refpoint()
    if use_ref_point:
        assert np.allclose(ref, [-1.1, -1.1])
    cand = s.ask(1)
    assert len(cand) == 1
    for k in bench.domain.inputs.get_keys():
        assert 0.0 <= cand[k].iloc[0] <= 1.0
    for k in bench.domain.outputs.get_keys():
        for suf in ("_pred", "_sd", "_des"):
            assert f"{k}{suf}" in cand.columns
    vals = s.calc_acquisition(pd.concat([cand[bench.domain.inputs.get_keys()], exps.iloc[:3]], ignore_index=True))
    assert vals.shape == (4,) and (vals >= 0).all()
    st = s.last_ask_stats
    assert st.raw_evals == 256 and st.opt_evals > 0


@pytest.mark.parametrize("mobo", [False, True])
def test_qnehvi_ask_approximate_partition(mobo):
    """QnehviStrategy(alpha=...) / MoboStrategy(qNEHVI(alpha=...)) at m = 3: the acquisition
    takes the approximate partition (bofire qnehvi.py:50, mobo.py:83) and ask() completes."""
    bench, exps = _dtlz2_experiments(n=14, m=3, seed=5)
    kw = dict(domain=bench.domain, ref_point=bench.ref_point, seed=4)
    if mobo:
        dmod = dm.MoboStrategy(acquisition_function=dm.qNEHVI(alpha=0.02, n_mc_samples=64), **kw)
    else:
        dmod = dm.QnehviStrategy(alpha=0.02, num_sobol_samples=64, num_raw_samples=128, num_restarts=2, **kw)
    s = strategies.map(dmod)
    s.tell(exps)
    cand = s.ask(1)
    assert len(cand) == 1 and s.last_acqf.box_path == "host-approx"
    for k in bench.domain.inputs.get_keys():
        assert 0.0 <= cand[k].iloc[0] <= 1.0


def test_qnehvi_ask_add_pending():
    """ask(add_pending=True) stores the candidate; the next ask() folds it into the baseline
    (X_pending, bofire/strategies/predictives/qnehvi.py:47), which removes its improvement."""
    bench, exps = _dtlz2_experiments(n=12, seed=3)
    s = strategies.map(dm.QnehviStrategy(domain=bench.domain, ref_point=bench.ref_point, seed=7,
                                         num_sobol_samples=128, num_raw_samples=256, num_restarts=4))
    s.tell(exps)
    c1 = s.ask(1, add_pending=True)
    assert s.candidates is not None and len(s.candidates) == 1
    keys = bench.domain.inputs.get_keys()
    before = s.last_acqf
    v_before = float(before.forward(torch.tensor(s._transform(c1), device=before.dev))[0])
    c2 = s.ask(1, add_pending=True)
    acqf = s.last_acqf
    assert acqf.n_pending == 1 and acqf.nb == len(acqf.base_rows) and acqf.base_rows[-1] == acqf.n
    v_after = float(acqf.forward(torch.tensor(s._transform(c1), device=acqf.dev))[0])
    assert v_before > 0 and v_after < 0.1 * v_before
    assert not np.allclose(c1[keys].values, c2[keys].values)
    assert len(s.candidates) == 2


def test_predict_matches_oracle_posterior():
    bench, exps = _dtlz2_experiments(n=30, m=3, seed=3)
    s = strategies.map(dm.QnehviStrategy(domain=bench.domain, seed=1))
    s.tell(exps)
    Xq = strategies.map(dm.RandomStrategy(domain=bench.domain, seed=5)).ask(50)
    pred = s.predict(Xq)
    for sur in s.surrogates.surrogates:
        st = sur.state
        key = sur.output_key
        o = ogp.GPState(X=torch.tensor((st["X"] - st["lo"]) / (st["hi"] - st["lo"])),
                        y=torch.tensor((st["y"] - st["y_mean"]) / st["y_std"]),
                        lengthscale=torch.tensor(st["lengthscale"]), noise=st["noise"], constant=st["constant"],
                        y_mean=st["y_mean"], y_std=st["y_std"])
        Xn = torch.tensor((Xq[bench.domain.inputs.get_keys()].values - st["lo"]) / (st["hi"] - st["lo"]))
        m, v = ogp.posterior(o, Xn, observation_noise=True)
        assert np.allclose(pred[f"{key}_pred"].values, m.numpy(), rtol=1e-9, atol=1e-9)
        assert np.allclose(pred[f"{key}_sd"].values, np.sqrt(v.numpy()), rtol=1e-7, atol=1e-9)
        assert np.allclose(pred[f"{key}_des"].values, -pred[f"{key}_pred"].values)


def test_device_fit_matches_oracle_fit():
    """fit_gpytorch_mll restated: device L-BFGS-B vs oracle L-BFGS-B (torch autograd) reach the
    same optimum (same start, same bounds; trajectories may differ by rounding)."""
    from everest_amd.gp import MLLEvaluator, fit_single

    bench, exps = _dtlz2_experiments(n=40, dim=4, m=2, seed=7)
    X = exps[bench.domain.inputs.get_keys()].values
    y = exps["f_0"].values
    prior = ogp.dim_scaled_lognormal(4)
    h = fit_single(torch.tensor(X, device="cuda"), y, 0, prior, (-4.0, 1.0))
    st, res = ogp.fit_gp(torch.tensor(X), torch.tensor(y), ogp.RBF, prior, (-4.0, 1.0))
    yy = (y - y.mean()) / y.std(ddof=1)
    ev = MLLEvaluator(torch.tensor(X, device="cuda"), yy, 0, prior, (-4.0, 1.0))
    x_dev = np.r_[h.noise, h.constant, np.log(np.expm1(h.lengthscale))]
    x_orc = np.r_[st.noise, st.constant, np.log(np.expm1(st.lengthscale.numpy()))]
    v_dev, _ = ev(x_dev)
    v_orc, _ = ev(x_orc)
    assert abs(v_dev - v_orc) <= 1e-6 * max(1.0, abs(v_orc))
    assert np.allclose(h.lengthscale, st.lengthscale.numpy(), rtol=2e-2)


def test_detergent_readme_loop():
    """README.md:82-104 loop (config 1): 2 initial random points + 4 ask/tell rounds with the
    two linear inequality constraints (SLSQP restarts on hit-and-run raw samples)."""
    bench = Detergent()
    rnd = strategies.map(dm.RandomStrategy(domain=bench.domain, seed=19))
    exps = bench.f(rnd.ask(2), return_complete=True)
    s = strategies.map(dm.QnehviStrategy(domain=bench.domain, seed=7, num_sobol_samples=64,
                                         num_raw_samples=128, num_restarts=4))
    s.tell(exps)
    for _ in range(4):
        c = s.ask(candidate_count=1)
        assert bench.domain.constraints.is_fulfilled(c, tol=1e-5).all()
        y = bench.f(c[bench.domain.inputs.get_keys()], return_complete=True)
        s.tell(y)
    assert s.num_experiments == 6


def test_sobo_qei_matern_parity():
    from everest_amd.acquisition import QEI
    from oracle import qnehvi as oq

    bench, exps = _dtlz2_experiments(n=25, dim=4, m=2, seed=11)
    dom = dm.Domain(inputs=bench.domain.inputs,
                    outputs=dm.Outputs(features=[dm.ContinuousOutput(key="f_0",
                                                                      objective=dm.MinimizeObjective(w=1.0))]))
    spec = dm.SingleTaskGPSurrogate(inputs=dom.inputs, outputs=dom.outputs, kernel=dm.MaternKernel(nu=2.5))
    s = strategies.map(dm.SoboStrategy(domain=dom, acquisition_function=dm.qEI(), seed=3,
                                       surrogate_specs=dm.BotorchSurrogates(surrogates=[spec]),
                                       num_raw_samples=64, num_restarts=2))
    s.tell(exps[dom.inputs.get_keys() + ["f_0", "valid_f_0"]])
    cand = s.ask(1)
    assert len(cand) == 1
    acqf = s._get_acqfs(1)[0]
    st = s.surrogates.surrogates[0].state
    o = ogp.GPState(X=torch.tensor(st["X"]), y=torch.tensor((st["y"] - st["y_mean"]) / st["y_std"]),
                    lengthscale=torch.tensor(st["lengthscale"]), noise=st["noise"], constant=st["constant"],
                    y_mean=st["y_mean"], y_std=st["y_std"], kind=ogp.MATERN25)
    Xc = np.random.default_rng(0).uniform(size=(20, 4))
    x = torch.tensor(Xc, requires_grad=True)
    ref = oq.qei([o], x.unsqueeze(1), acqf.best_f, acqf.z.cpu().unsqueeze(-1), a=-1.0, bconst=0.0)
    ref.sum().backward()
    acq, dX = acqf.forward_backward(torch.tensor(Xc, device="cuda"))
    assert torch.allclose(acq.cpu(), ref.detach(), rtol=1e-7, atol=1e-10)
    assert torch.allclose(dX.cpu(), x.grad, rtol=1e-6, atol=1e-9)


def _sobo_qei_strategy(seed=11):
    bench, exps = _dtlz2_experiments(n=25, dim=4, m=2, seed=seed)
    dom = dm.Domain(inputs=bench.domain.inputs,
                    outputs=dm.Outputs(features=[dm.ContinuousOutput(key="f_0",
                                                                      objective=dm.MinimizeObjective(w=1.0))]))
    spec = dm.SingleTaskGPSurrogate(inputs=dom.inputs, outputs=dom.outputs, kernel=dm.MaternKernel(nu=2.5))
    s = strategies.map(dm.SoboStrategy(domain=dom, acquisition_function=dm.qEI(n_mc_samples=128), seed=3,
                                       surrogate_specs=dm.BotorchSurrogates(surrogates=[spec]),
                                       num_raw_samples=64, num_restarts=2))
    s.tell(exps[dom.inputs.get_keys() + ["f_0", "valid_f_0"]])
    st = s.surrogates.surrogates[0].state
    o = ogp.GPState(X=torch.tensor(st["X"]), y=torch.tensor((st["y"] - st["y_mean"]) / st["y_std"]),
                    lengthscale=torch.tensor(st["lengthscale"]), noise=st["noise"], constant=st["constant"],
                    y_mean=st["y_mean"], y_std=st["y_std"], kind=ogp.MATERN25)
    return s, dom, o


@pytest.mark.parametrize("q,npend", [(3, 0), (1, 2), (2, 1)])
def test_qei_joint_batch_parity(q, npend):
    """qEI over joint batches (q > 1, pending points: sobo.py:51-90 with X_pending) through the
    m = 1 general qEHVI kernels vs the oracle's joint-posterior qEI (psd_safe q x q root,
    mean_s max_i (g - best_f)_+), values and gradients on the same base samples."""
    from everest_amd.acquisition import QEI, QEIJoint
    from oracle import qnehvi as oq

    s, dom, o = _sobo_qei_strategy()
    X_train, _ = s.get_acqf_input_tensors()
    rng = np.random.default_rng(q * 10 + npend)
    Xp = rng.uniform(size=(npend, 4)) if npend else None
    acqf = QEIJoint(s.model, X_train, -1.0, 0.0, S=128, seed=9, X_pending_raw=Xp)
    assert abs(acqf.best_f - QEI(s.model, X_train, -1.0, 0.0, S=8).best_f) == 0.0
    qq = q + npend
    z = acqf._zq(qq).reshape(128, qq).cpu()
    Xc = rng.uniform(size=(12, q, 4))
    x = torch.tensor(Xc, requires_grad=True)
    xf = torch.cat([x, torch.tensor(Xp).unsqueeze(0).expand(12, npend, 4)], 1) if npend else x
    ref = oq.qei([o], xf, acqf.best_f, z, a=-1.0, bconst=0.0)
    ref.sum().backward()
    acq, dX = acqf.forward_backward(torch.tensor(Xc, device="cuda"))
    assert torch.allclose(acq.cpu(), ref.detach(), rtol=1e-6, atol=1e-10)
    assert torch.allclose(dX.cpu().reshape(12, q, 4), x.grad, rtol=1e-5, atol=1e-8)


def test_sobo_ask_joint_and_pending():
    """SoboStrategy.ask(2) optimises one joint q = 2 batch; ask(add_pending=True) then folds the
    pending candidate into the next qEI (which no longer raises)."""
    s, dom, _ = _sobo_qei_strategy(seed=4)
    c2 = s.ask(2)
    assert len(c2) == 2
    v = s.calc_acquisition(c2[dom.inputs.get_keys()], combined=True)
    assert v.shape == (1,) and v[0] >= 0
    c1 = s.ask(1, add_pending=True)
    c1b = s.ask(1)
    assert len(c1b) == 1 and not np.allclose(c1[dom.inputs.get_keys()].values, c1b[dom.inputs.get_keys()].values)


def test_qnehvi_ask_joint_batch_and_combined_value():
    """ask(candidate_count=3): one joint q = 3 optimisation (optimize_acqf(q=...),
    bofire/strategies/predictives/botorch.py:385); calc_acquisition(combined=True) scores the
    batch as one q-batch (:196-225) and equals the acquisition's joint value."""
    bench, exps = _dtlz2_experiments(n=14, seed=5)
    s = strategies.map(dm.QnehviStrategy(domain=bench.domain, ref_point=bench.ref_point, seed=3,
                                         num_sobol_samples=64, num_raw_samples=128, num_restarts=4))
    s.tell(exps)
    cand = s.ask(3)
    assert len(cand) == 3
    keys = bench.domain.inputs.get_keys()
    assert ((cand[keys].values >= 0) & (cand[keys].values <= 1)).all()
    assert not np.allclose(cand[keys].values[0], cand[keys].values[1])
    joint = s.calc_acquisition(cand[keys], combined=True)
    single = s.calc_acquisition(cand[keys])
    assert joint.shape == (1,) and single.shape == (3,)
    # HVI of a union: at least the best single point, at most the sum
    assert single.max() - 1e-12 <= joint[0] <= single.sum() + 1e-12
    assert s.last_ask_stats.best_value > 0


def test_qnehvi_output_constraint_and_close_to_target():
    """Outputs: f_0 minimised, f_1 CloseToTarget(0.4, e=2), f_2 MaximizeSigmoid(tp=0.2) as an
    output constraint (get_output_constraints, bofire/utils/torch_tools.py:340-381)."""
    bench, exps = _dtlz2_experiments(n=16, m=3, seed=9)
    outs = dm.Outputs(features=[
        dm.ContinuousOutput(key="f_0", objective=dm.MinimizeObjective(w=1.0)),
        dm.ContinuousOutput(key="f_1", objective=dm.CloseToTargetObjective(target_value=0.4, exponent=2.0)),
        dm.ContinuousOutput(key="f_2", objective=dm.MaximizeSigmoidObjective(tp=0.2, steepness=50.0))])
    dom = dm.Domain(inputs=bench.domain.inputs, outputs=outs)
    s = strategies.map(dm.QnehviStrategy(domain=dom, seed=2, num_sobol_samples=64, num_raw_samples=128,
                                         num_restarts=4))
    s.tell(exps)
    objectives, constraints = s._objective_spec()
    assert [o[1] for o in objectives] == [0, 1] and constraints == [(2, -1.0, 0.2, 1.0 / 50.0)]
    acqf = s._get_acqfs(1)[0]
    assert not acqf.supports_plan and acqf.spec.m_obj == 2
    cand = s.ask(2)
    assert len(cand) == 2
    vals = s.calc_acquisition(cand[dom.inputs.get_keys()])
    assert np.isfinite(vals).all() and (vals >= 0).all()


def test_qehvi_pending_joint_batch():
    """qEHVI with a pending candidate: the pending point joins every candidate's joint batch
    ([upstream] concatenate_pending_points; QehviStrategy passes X_pending,
    bofire/strategies/predictives/qehvi.py:60-78)."""
    bench, exps = _dtlz2_experiments(n=12, seed=4)
    s = strategies.map(dm.QehviStrategy(domain=bench.domain, ref_point=bench.ref_point, seed=5,
                                        num_sobol_samples=64, num_raw_samples=128, num_restarts=4))
    s.tell(exps)
    c1 = s.ask(1, add_pending=True)
    c2 = s.ask(1, add_pending=True)
    acqf = s.last_acqf
    assert acqf.X_pending is not None and acqf.X_pending.shape[0] == 1
    # the pending point must reach the restarts' optimiser: not the pending-free q = 1 plan
    assert not acqf.supports_plan
    st = s.last_ask_stats
    assert st.chunks and all(ch["driver"] != "native-plan" for ch in st.chunks)
    v2 = acqf.forward(torch.tensor(s._transform(c2), device=acqf.dev))
    v1 = acqf.forward(torch.tensor(s._transform(c1), device=acqf.dev))
    assert torch.isfinite(v2).all() and float(v2[0]) > 0
    # the returned best value is the acquisition with the pending point at the candidate
    assert abs(float(v2[0]) - st.best_value) <= 1e-9 * max(1.0, abs(st.best_value))
    keys = bench.domain.inputs.get_keys()
    assert not np.allclose(c1[keys].values, c2[keys].values) or float(v2[0]) >= float(v1[0]) - 1e-12
    assert len(s.candidates) == 2


def test_qehvi_strategy_ignores_output_constraints():
    """QehviStrategy builds qExpectedHypervolumeImprovement without constraints / eta
    (bofire/strategies/predictives/qehvi.py:67-75) and its data model admits no constrained
    objective (data_models/strategies/predictives/qehvi.py:54-70); QnehviStrategy passes the
    output constraints (qnehvi.py:28-51)."""
    bench, exps = _dtlz2_experiments(n=16, m=3, seed=9)
    outs = dm.Outputs(features=[
        dm.ContinuousOutput(key="f_0", objective=dm.MinimizeObjective(w=1.0)),
        dm.ContinuousOutput(key="f_1", objective=dm.MinimizeObjective(w=1.0)),
        dm.ContinuousOutput(key="f_2", objective=dm.MaximizeSigmoidObjective(tp=0.2, steepness=50.0))])
    dom = dm.Domain(inputs=bench.domain.inputs, outputs=outs)
    kw = dict(domain=dom, seed=2, num_sobol_samples=64, num_raw_samples=128, num_restarts=2)
    with pytest.raises(ValueError):
        dm.QehviStrategy(**kw)
    s2 = strategies.map(dm.QnehviStrategy(**kw))
    s2.tell(exps)
    assert len(s2._get_acqfs(1)[0].spec.constraints) == 1
    # the plain two-objective QehviStrategy runs the fused q = 1 plan (affine objectives only)
    s = strategies.map(dm.QehviStrategy(domain=bench.domain, ref_point=bench.ref_point, seed=2,
                                        num_sobol_samples=64, num_raw_samples=128, num_restarts=2))
    s.tell(exps)
    acqf = s._get_acqfs(1)[0]
    assert acqf.spec.constraints == [] and acqf.supports_plan
