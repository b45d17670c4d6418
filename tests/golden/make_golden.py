"""Generate golden vectors by importing the REFERENCE's own data-model / benchmark layer.

Run in the build container only (the reference never travels to the GPU box):
    PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
Writes tests/golden/reference_datamodels.json (inputs + expected outputs only).
Only modules importable without BoTorch/GPyTorch are used.
"""
import json
import os

import numpy as np
import pandas as pd

from bofire.benchmarks.detergent import Detergent
from bofire.data_models.domain.api import Domain, Inputs, Outputs
from bofire.data_models.features.api import CategoricalInput, ContinuousInput, ContinuousOutput
from bofire.data_models.enum import CategoricalEncodingEnum
from bofire.data_models.kernels.api import MaternKernel, RBFKernel
from bofire.data_models.objectives.api import MaximizeObjective, MinimizeObjective
from bofire.data_models.priors.api import DimensionalityScaledLogNormalPrior, LogNormalPrior
from bofire.data_models.strategies.predictives.qnehvi import QnehviStrategy
from bofire.data_models.surrogates.api import SingleTaskGPSurrogate

out = {}

# Detergent: seeded designs and outputs (bofire/benchmarks/detergent.py:15-88)
det = Detergent()
rows = []
for seed in (0, 1, 2):
    X = det.domain.inputs.sample(6, seed=seed)
    Y = det.f(X)
    rows.append({"seed": seed, "X": X[det.domain.inputs.get_keys()].values.tolist(),
                 "Y": Y[det.domain.outputs.get_keys()].values.tolist()})
out["detergent"] = {"input_keys": det.domain.inputs.get_keys(), "output_keys": det.domain.outputs.get_keys(),
                    "designs": rows,
                    "constraints": [c.model_dump() for c in det.domain.constraints.constraints]}

# ContinuousInput.sample (bofire/data_models/features/continuous.py:108-122)
ci = ContinuousInput(key="a", bounds=[-1.0, 3.0])
out["continuous_sample"] = {"bounds": [-1.0, 3.0], "seed": 7, "n": 5, "values": ci.sample(5, seed=7).tolist()}

# Inputs.get_bounds with experiments (features.py:628-679 -> continuous.py:134-167)
inp = Inputs(features=[ContinuousInput(key="x1", bounds=[0, 1]), ContinuousInput(key="x2", bounds=[-2, 2]),
                       CategoricalInput(key="c", categories=["a", "b", "c"], allowed=[True, False, True])])
ex = pd.DataFrame({"x1": [0.5, 1.7, -0.3], "x2": [0.0, 1.0, -1.0], "c": ["a", "c", "a"]})
lo, hi = inp.get_bounds(specs={"c": CategoricalEncodingEnum.ONE_HOT}, experiments=ex)
out["bounds_with_experiments"] = {"experiments": ex.to_dict(orient="list"), "lower": lo, "upper": hi,
                                  "keys": inp.get_keys()}
tr = inp.transform(ex, specs={"c": CategoricalEncodingEnum.ONE_HOT})
out["onehot_transform"] = {"columns": list(tr.columns), "values": tr.values.tolist()}

# objectives (bofire/data_models/objectives/identity.py)
x = np.array([-1.0, 0.0, 0.25, 2.0])
out["objectives"] = {
    "x": x.tolist(),
    "maximize_0_1": MaximizeObjective(w=1.0)(x).tolist(),
    "minimize_0_1": MinimizeObjective(w=1.0)(x).tolist(),
    "maximize_m1_3": MaximizeObjective(w=1.0, bounds=[-1, 3])(x).tolist(),
    "minimize_m1_3": MinimizeObjective(w=1.0, bounds=[-1, 3])(x).tolist(),
}

# strategy / surrogate defaults (data_models/strategies/predictives/{botorch,qehvi,qnehvi}.py,
# data_models/surrogates/single_task_gp.py)
s = QnehviStrategy(domain=det.domain)
sur = s.surrogate_specs.surrogates[0]
out["qnehvi_defaults"] = {
    "num_sobol_samples": s.num_sobol_samples, "num_restarts": s.num_restarts,
    "num_raw_samples": s.num_raw_samples, "maxiter": s.maxiter, "batch_limit": s.batch_limit, "alpha": s.alpha,
    "n_surrogates": len(s.surrogate_specs.surrogates), "kernel": json.loads(sur.kernel.model_dump_json()),
    "noise_prior": json.loads(sur.noise_prior.model_dump_json()), "scaler": sur.scaler.value,
    "output_scaler": sur.output_scaler.value,
}
s2 = QnehviStrategy(domain=det.domain, num_restarts=20, batch_limit=50)
out["batch_limit_clamp"] = {"num_restarts": 20, "batch_limit_in": 50, "batch_limit": s2.batch_limit}
p = DimensionalityScaledLogNormalPrior()
out["dim_scaled_prior"] = {"loc": p.loc, "loc_scaling": p.loc_scaling, "scale": p.scale,
                           "scale_scaling": p.scale_scaling}

# hypervolume strategies and acquisition-function data models
# (data_models/strategies/predictives/{qehvi,mobo}.py, data_models/acquisition_functions/acquisition_function.py)
from bofire.data_models.acquisition_functions.api import qEHVI, qEI, qLogEHVI, qLogNEHVI, qNEHVI
from bofire.data_models.strategies.predictives.mobo import MoboStrategy
from bofire.data_models.strategies.predictives.qehvi import QehviStrategy

out["acqf_dumps"] = {c.__name__: json.loads(c().model_dump_json()) for c in (qEHVI, qLogEHVI, qNEHVI, qLogNEHVI, qEI)}
mo = MoboStrategy(domain=det.domain)
out["mobo_defaults"] = {"acquisition_function": json.loads(mo.acquisition_function.model_dump_json()),
                        "ref_point": mo.ref_point, "num_restarts": mo.num_restarts,
                        "num_raw_samples": mo.num_raw_samples, "batch_limit": mo.batch_limit}
qe = QehviStrategy(domain=det.domain)
out["qehvi_defaults"] = {"num_sobol_samples": qe.num_sobol_samples, "ref_point": qe.ref_point,
                         "type": qe.type}


# objective callables and smoothed feasibility (the known-answer tests of
# tests/bofire/utils/test_torch_tools.py:105-139 and :1064-1104): the reference's own
# objective __call__ values on fixed samples.  The build's device objective g(y) must equal
# __call__ for the objectives get_objective_callable turns into MC objectives, and its
# feasibility weight exp(sum logsigmoid(-c/eta)) over the constraints
# constrained_objective2botorch makes must equal __call__ for the constrained ones.
from bofire.data_models.objectives.api import (CloseToTargetObjective, MaximizeSigmoidObjective,
                                               MinimizeSigmoidObjective, MovingMaximizeSigmoidObjective,
                                               TargetObjective)

rng = np.random.default_rng(105)
samples = rng.uniform(size=50) * 5.0                  # test_torch_tools.py:130: rand(50, 3) * 5, column 1
x_adapt = rng.uniform(size=10) * 3.0                  # :132
callables = []
for obj in (MaximizeObjective(w=0.5), MinimizeObjective(w=0.5), CloseToTargetObjective(target_value=2.0, exponent=1.0, w=0.5),
            CloseToTargetObjective(target_value=2.0, exponent=2.0, w=0.5),
            MaximizeObjective(w=1.0, bounds=[-1.0, 3.0]), MinimizeObjective(w=1.0, bounds=[0.5, 4.0]),
            MaximizeSigmoidObjective(steepness=1.0, tp=1.0, w=0.5), MinimizeSigmoidObjective(steepness=1.0, tp=1.0, w=0.5),
            TargetObjective(target_value=2.0, steepness=1.0, tolerance=1e-3, w=0.5),
            MovingMaximizeSigmoidObjective(steepness=1, tp=-1, w=1)):
    callables.append({"objective": json.loads(obj.model_dump_json()),
                      "values": np.asarray(obj(samples, x_adapt=x_adapt), dtype=np.float64).tolist()})
out["objective_callables"] = {"samples": samples.tolist(), "x_adapt": x_adapt.tolist(), "cases": callables}

xf = np.linspace(0, 30, 500)                           # :1079
xa = np.array([1.0, 2.0, 3.0])                         # :1074
feas = []
for obj in (MaximizeSigmoidObjective(w=1, tp=15, steepness=0.5), MinimizeSigmoidObjective(w=1, tp=15, steepness=0.5),
            TargetObjective(w=1, target_value=15, steepness=2, tolerance=5),
            MovingMaximizeSigmoidObjective(w=1, tp=-1, steepness=0.5)):
    feas.append({"objective": json.loads(obj.model_dump_json()),
                 "values": np.asarray(obj(xf, x_adapt=xa), dtype=np.float64).tolist()})
out["smoothed_feasibility"] = {"x": xf.tolist(), "x_adapt": xa.tolist(), "cases": feas}

# get_output_constraints etas (:546-581): outputs of1 Maximize, of2 MaximizeSigmoid(steepness 2),
# of3 Target(steepness 4) -> etas [0.5, 0.25, 0.25] (the test's literal; the etas are
# 1/steepness per constraint, two constraints for a TargetObjective)
of1 = ContinuousOutput(key="of1", objective=MaximizeObjective(w=1.0))
of2 = ContinuousOutput(key="of2", objective=MaximizeSigmoidObjective(w=1.0, tp=0, steepness=2))
of3 = ContinuousOutput(key="of3", objective=TargetObjective(w=1.0, tolerance=2, target_value=5, steepness=4))
out["output_constraint_etas"] = {
    "orders": [[json.loads(f.model_dump_json()) for f in fs] for fs in ((of1, of2, of3), (of2, of1, of3))],
    "etas": [0.5, 0.25, 0.25]}

with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_datamodels.json"), "w") as f:
    json.dump(out, f, indent=1)
print("wrote reference_datamodels.json")
