"""Workload generators with BoFire's benchmark API (``.domain``, ``.f(df, return_complete)``):
Detergent (bofire/benchmarks/detergent.py:15-88), DTLZ2 (bofire/benchmarks/multi.py:37-132)
and C2DTLZ2 (bofire/benchmarks/multi.py:227-272).
Numbers restated: Detergent's coefficient table is data of the reference benchmark."""
from __future__ import annotations

import math

import numpy as np
import pandas as pd

from .data_models import (ContinuousInput, ContinuousOutput, Domain, Inputs, LinearInequalityConstraint,
                          MaximizeSigmoidObjective, MinimizeObjective, Outputs)


class Benchmark:
    """bofire/benchmarks/benchmark.py:49-70."""

    def f(self, candidates: pd.DataFrame, return_complete: bool = False) -> pd.DataFrame:
        Y = self._f(candidates)
        if return_complete:
            return pd.concat([candidates, Y], axis=1)
        return Y

    @property
    def domain(self) -> Domain:
        return self._domain


class DTLZ2(Benchmark):
    def __init__(self, dim: int, num_objectives: int = 2):
        if dim <= num_objectives:
            raise ValueError(f"dim must be > num_objectives, but got {dim} and {num_objectives}.")
        self.num_objectives = num_objectives
        self.dim = dim
        self.k = dim - num_objectives + 1
        self._domain = Domain(
            inputs=Inputs(features=[ContinuousInput(key=f"x_{i}", bounds=(0, 1)) for i in range(dim)]),
            outputs=Outputs(features=[ContinuousOutput(key=f"f_{i}", objective=MinimizeObjective(w=1.0))
                                      for i in range(num_objectives)]),
        )
        self.ref_point = {f"f_{i}": 1.1 for i in range(num_objectives)}

    def _f(self, candidates: pd.DataFrame) -> pd.DataFrame:
        X = candidates[[f"x_{i}" for i in range(self.dim)]].values
        Xm = X[..., -self.k:]
        g1 = 1 + ((Xm - 0.5) ** 2).sum(axis=-1)
        fs = []
        for i in range(self.num_objectives):
            idx = self.num_objectives - 1 - i
            f = g1 * np.cos(X[..., :idx] * math.pi / 2).prod(axis=-1)
            if i > 0:
                f = f * np.sin(X[..., idx] * math.pi / 2)
            fs.append(f)
        keys = [f"f_{i}" for i in range(self.num_objectives)]
        Y = pd.DataFrame(np.stack(fs, axis=-1), columns=keys, index=candidates.index)
        for k in keys:
            Y[f"valid_{k}"] = 1
        return Y


class C2DTLZ2(DTLZ2):
    """Constrained DTLZ2 (bofire/benchmarks/multi.py:227-272): DTLZ2 plus the output ``slack``
    with MaximizeSigmoidObjective(tp=0, steepness=1e3) — feasible where slack >= 0, i.e. an
    output constraint with eta = 1e-3.  slack = -min(min_i [(f_i - 1)^2 + sum_{j != i}
    (f_j^2 - r^2)], sum_i [(f_i - 1/sqrt(m))^2 - r^2]) with r = 0.2."""

    def __init__(self, dim: int, num_objectives: int = 2):
        super().__init__(dim, num_objectives)
        self._domain = Domain(
            inputs=self._domain.inputs,
            outputs=Outputs(features=list(self._domain.outputs.features) + [
                ContinuousOutput(key="slack", objective=MaximizeSigmoidObjective(w=1.0, tp=0, steepness=1.0 / 1e-3))]),
        )

    @property
    def best_possible_hypervolume(self) -> float:
        return 0.3996406303723544

    def _f(self, candidates: pd.DataFrame) -> pd.DataFrame:
        r = 0.2
        Y = super()._f(candidates)
        f = Y[[f"f_{i}" for i in range(self.num_objectives)]].values
        m = f.shape[1]
        sq = f ** 2 - r ** 2
        term1 = (f - 1.0) ** 2
        term2 = sq.sum(axis=1, keepdims=True) - sq           # sum over j != i
        min1 = (term1 + term2).min(axis=1)
        min2 = ((f - 1.0 / math.sqrt(m)) ** 2 - r ** 2).sum(axis=1)
        Y["slack"] = -np.minimum(min1, min2)
        Y["valid_slack"] = 1
        return Y


DETERGENT_COEF = np.array([
    [0.4967, 0.0, 0.6477, 1.523, 0.0], [0.0, 4.7376, 2.3023, 0.0, 1.6277], [0.0, 0.0, 0.7259, 0.0, 0.0],
    [0.0, 0.0, 0.9427, 0.0, 0.0], [4.3969, 0.0, 0.2026, 0.0, 0.0], [0.3328, 0.0, 1.1271, 0.0, 0.0],
    [0.0, 16.6705, 0.0, 0.0, 7.4029], [0.0, 1.8798, 0.0, 0.0, 1.7718], [6.6462, 1.5423, 0.0, 0.0, 0.0],
    [0.0, 0.0, 9.5141, 3.0926, 0.0], [2.9168, 0.0, 0.0, 5.5051, 9.279], [8.3815, 0.0, 0.0, 2.9814, 8.7799],
    [0.0, 0.0, 0.0, 0.0, 7.3127], [12.2062, 0.0, 9.0318, 3.2547, 0.0], [3.2526, 13.8423, 0.0, 14.0818, 0.0],
    [7.3971, 0.7834, 0.0, 0.8258, 0.0], [0.0, 3.214, 13.301, 0.0, 0.0], [0.0, 8.2386, 2.9588, 0.0, 4.6194],
    [0.8737, 8.7178, 0.0, 0.0, 0.0], [0.0, 2.6651, 2.3495, 0.046, 0.0], [0.0, 0.0, 0.0, 0.0, 0.0],
])


class Detergent(Benchmark):
    """5 components, 5 second-order polynomial outputs (maximise), 2 linear inequalities."""

    def __init__(self):
        self.coef = DETERGENT_COEF
        self._domain = Domain.from_lists(
            inputs=[ContinuousInput(key="x1", bounds=(0.0, 0.2)), ContinuousInput(key="x2", bounds=(0.0, 0.3)),
                    ContinuousInput(key="x3", bounds=(0.02, 0.2)), ContinuousInput(key="x4", bounds=(0.0, 0.06)),
                    ContinuousInput(key="x5", bounds=(0.0, 0.04))],
            outputs=[ContinuousOutput(key=f"y{i + 1}") for i in range(5)],
            constraints=[LinearInequalityConstraint(features=["x1", "x2", "x3", "x4", "x5"], coefficients=[-1] * 5,
                                                    rhs=-0.2),
                         LinearInequalityConstraint(features=["x1", "x2", "x3", "x4", "x5"], coefficients=[1] * 5,
                                                    rhs=0.4)],
        )

    @staticmethod
    def _poly2(x):
        return np.concatenate([[1], x, np.outer(x, x)[np.triu_indices(5)]])

    def _f(self, X: pd.DataFrame) -> pd.DataFrame:
        x = np.atleast_2d(X[self.domain.inputs.get_keys()].values)
        xp = np.stack([self._poly2(xi) for xi in x], axis=0)
        Y = pd.DataFrame(xp @ self.coef, columns=self.domain.outputs.get_keys(), index=X.index)
        for k in self.domain.outputs.get_keys():
            Y[f"valid_{k}"] = 1
        return Y
