"""CPU: re-expressions of the reference's known-answer tests at the hot path's boundary
(SURVEY.md §4): reference-point mask / inference (tests/bofire/utils/test_multiobjective.py
:55-266 fixtures), adjusted ref point (tests/bofire/strategies/test_qehvi.py:114-130),
prior mapping (tests/bofire/priors/test_mapper.py:51-73), linear constraints in BoTorch form,
Normalize scaler bounds (tests/bofire/surrogates/test_utils.py:54-78)."""
import math

import numpy as np
import pandas as pd
import pytest

import everest_amd.data_models as dm
from everest_amd import strategies
from everest_amd.surrogates import SingleTaskGPSurrogate, map_prior

if1 = dm.ContinuousInput(key="if1", bounds=(0, 10))
if2 = dm.ContinuousInput(key="if2", bounds=(0, 20))
of1 = dm.ContinuousOutput(objective=dm.MaximizeObjective(w=1), key="of1")
of2 = dm.ContinuousOutput(objective=dm.MinimizeObjective(w=1), key="of2")
of3 = dm.ContinuousOutput(objective=dm.MaximizeObjective(w=1), key="of3")
of4 = dm.ContinuousOutput(objective=dm.MinimizeObjective(w=1), key="of4")
of7 = dm.ContinuousOutput(objective=dm.CloseToTargetObjective(w=1, target_value=5, exponent=1), key="of7")


def D(outs):
    return dm.Domain.from_lists(inputs=[if1, if2], outputs=outs)


valid_domains = [D([of1, of2]), D([of1, of3]), D([of1, of2, of3, of4]), D([of2, of4]), D([of2, of1, of3, of4]),
                 D([of1, of2, of7])]
base = {"if1": [3.0, 4.0, 5.0, 6.0], "if2": [10.0, 7.0, 8.0, 12.0], "of1": [1.0, 10.0, 4.0, 5.0]}
dfs = [pd.DataFrame({**base, "of2": [5.0, 3.0, 2.0, 5.0], "valid_of1": [1] * 4, "valid_of2": [1] * 4}),
       pd.DataFrame({**base, "of3": [5.0, 3.0, 2.0, 5.0], "valid_of1": [1] * 4, "valid_of3": [1] * 4}),
       pd.DataFrame({**base, "of2": [5.0, 3.0, 2.0, 5.0], "of7": [10.0, 0.0, 30.0, 6.0], "valid_of1": [1] * 4,
                     "valid_of2": [1] * 4, "valid_of7": [1] * 4})]


@pytest.mark.parametrize("domain, expected", [
    (valid_domains[0], [1.0, -1.0]), (valid_domains[1], [1.0, 1.0]), (valid_domains[2], [1.0, -1.0, 1.0, -1.0]),
    (valid_domains[3], [-1.0, -1.0]), (valid_domains[4], [1.0, -1.0, 1.0, -1.0]), (valid_domains[5], [1.0, -1.0, -1.0])])
def test_get_ref_point_mask(domain, expected):
    assert np.allclose(strategies.get_ref_point_mask(domain), expected)


def test_ref_point_mask_subset_and_invalid():
    assert np.allclose(strategies.get_ref_point_mask(valid_domains[2], ["of1", "of2", "of3"]), [1, -1, 1])
    with pytest.raises(ValueError):
        strategies.get_ref_point_mask(D([of1]))


@pytest.mark.parametrize("domain, experiments, return_masked, expected", [
    (valid_domains[0], dfs[0], True, {"of1": 1.0, "of2": -5.0}),
    (valid_domains[0], dfs[0], False, {"of1": 1.0, "of2": 5.0}),
    (valid_domains[1], dfs[1], True, {"of1": 1.0, "of3": 2.0}),
    (valid_domains[1], dfs[1], False, {"of1": 1.0, "of3": 2.0}),
    (valid_domains[5], dfs[2], True, {"of1": 1.0, "of2": -5.0, "of7": -25.0}),
    (valid_domains[5], dfs[2], False, {"of1": 1.0, "of2": 5.0, "of7": 25.0})])
def test_infer_ref_point(domain, experiments, return_masked, expected):
    rp = strategies.infer_ref_point(domain, experiments, return_masked)
    for k, v in expected.items():
        assert np.isclose(rp[k], v)


@pytest.mark.parametrize("domain, ref_point, experiments, expected", [
    (valid_domains[0], {"of1": 0.5, "of2": 10.0}, dfs[0], [0.5, -10.0]),
    (valid_domains[1], {"of1": 0.5, "of3": 0.5}, dfs[1], [0.5, 0.5]),
    (valid_domains[0], None, dfs[0], [1.0, -5.0]),
    (valid_domains[1], None, dfs[1], [1.0, 2.0])])
def test_qehvi_get_adjusted_refpoint(domain, ref_point, experiments, expected):
    s = strategies.map(dm.QnehviStrategy(domain=domain, ref_point=ref_point))
    s.set_experiments(experiments)   # as the reference test: no training
    rp = s.get_adjusted_refpoint()
    assert isinstance(rp, list) and np.allclose(rp, expected)


def test_dimensionality_scaled_prior_map():
    p = dm.DimensionalityScaledLogNormalPrior(loc=np.sqrt(2), loc_scaling=0.5, scale=np.sqrt(3), scale_scaling=0.0)
    fam, loc, scale = map_prior(p, d=6)
    assert fam == "lognormal"
    assert loc == np.sqrt(2) + math.log(6) * 0.5
    assert scale == (3 + math.log(6) * 0.0) ** 0.5
    assert np.isclose(map_prior(dm.DimensionalityScaledLogNormalPrior(), 32)[1], 3.1471, atol=1e-4)


def test_linear_constraints_botorch_form():
    from everest_amd.benchmarks import Detergent

    d = Detergent().domain
    ineq = strategies.get_linear_constraints(d, dm.LinearInequalityConstraint)
    assert len(ineq) == 2
    idx, coef, rhs = ineq[0]
    assert list(idx) == [0, 1, 2, 3, 4] and np.allclose(coef, 1.0) and rhs == 0.2     # -(-1) x >= -(-0.2)
    idx, coef, rhs = ineq[1]
    assert np.allclose(coef, -1.0) and rhs == -0.4


def test_normalize_bounds_known_answer():
    """get_scaler(NORMALIZE): offset = lower bound, coefficient = range over (feature bounds U data)."""
    inputs = dm.Inputs(features=[dm.ContinuousInput(key=f"x{i}", bounds=(-4, 4)) for i in range(2)])
    outputs = dm.Outputs(features=[dm.ContinuousOutput(key="y")])
    sur = SingleTaskGPSurrogate(dm.SingleTaskGPSurrogate(inputs=inputs, outputs=outputs))
    X = pd.DataFrame({"x0": [-1.0, 2.0], "x1": [0.0, 5.0]})
    lo, hi = sur._bounds(X)
    assert np.allclose(lo, [-4.0, -4.0]) and np.allclose(hi - lo, [8.0, 9.0])


@pytest.mark.parametrize("domain, ref_point, experiments, expected", [
    (valid_domains[0], {"of1": 0.5, "of2": 10.0}, dfs[0], [0.5, -10.0]),
    (valid_domains[1], {"of1": 0.5, "of3": 0.5}, dfs[1], [0.5, 0.5]),
    (valid_domains[0], None, dfs[0], [1.0, -5.0]),
    (valid_domains[1], None, dfs[1], [1.0, 2.0])])
def test_mobo_get_adjusted_refpoint(domain, ref_point, experiments, expected):
    """tests/bofire/strategies/test_mobo.py:59-75."""
    s = strategies.map(dm.MoboStrategy(domain=domain, ref_point=ref_point))
    s.set_experiments(experiments)   # as the reference test: no training
    rp = s.get_adjusted_refpoint()
    assert isinstance(rp, list) and np.allclose(rp, expected)


def test_c2dtlz2_slack_restatement():
    """C2DTLZ2 (bofire/benchmarks/multi.py:227-272): the slack output against a direct
    per-row evaluation of the reference's gather formula; its objective is a sigmoid
    constraint with eta = 1e-3."""
    from everest_amd.benchmarks import C2DTLZ2

    bm = C2DTLZ2(dim=4)
    X = pd.DataFrame(np.random.default_rng(0).uniform(size=(16, 4)), columns=bm.domain.inputs.get_keys())
    Y = bm.f(X)
    f = Y[["f_0", "f_1"]].values
    r = 0.2
    for i, row in enumerate(f):
        m = len(row)
        min1 = min((row[a] - 1) ** 2 + sum(row[b] ** 2 - r ** 2 for b in range(m) if b != a) for a in range(m))
        min2 = sum((row[a] - 1 / math.sqrt(m)) ** 2 - r ** 2 for a in range(m))
        assert np.isclose(Y["slack"].values[i], -min(min1, min2), rtol=1e-14, atol=1e-15)
    assert (Y["valid_slack"] == 1).all()
    obj = bm.domain.outputs.get_by_key("slack").objective
    assert isinstance(obj, dm.MaximizeSigmoidObjective) and obj.tp == 0 and np.isclose(1 / obj.steepness, 1e-3)
