"""Domain data models (features, objectives, constraints) — the subset of BoFire's
pydantic data-model layer on the GP/qNEHVI path, with the same field names, defaults,
``type`` tags and JSON shape (bofire/data_models/{features,objectives,constraints,domain}).

Ordering follows BoFire: containers return features sorted by (order_id, key)
(bofire/data_models/features/feature.py:20-37; continuous input 1, categorical input 7,
continuous output 9)."""
from __future__ import annotations

import math
import warnings
from typing import Annotated, ClassVar, Dict, List, Literal, Optional, Sequence, Tuple, Type, Union

import numpy as np
import pandas as pd
from pydantic import BaseModel as _PBaseModel
from pydantic import ConfigDict, Field, field_validator, model_validator


class BaseModel(_PBaseModel):
    """bofire/data_models/base.py:6-17."""
    model_config = ConfigDict(validate_assignment=True, arbitrary_types_allowed=True, extra="forbid")


class ConstraintNotFulfilledError(Exception):
    pass


# ---------------------------------------------------------------------------------------
# objectives  (bofire/data_models/objectives/identity.py, target.py)
# ---------------------------------------------------------------------------------------
class Objective(BaseModel):
    type: str


class IdentityObjective(Objective):
    type: Literal["IdentityObjective"] = "IdentityObjective"
    w: Annotated[float, Field(gt=0, le=1)] = 1.0
    bounds: Tuple[float, float] = (0, 1)

    @property
    def lower_bound(self) -> float:
        return self.bounds[0]

    @property
    def upper_bound(self) -> float:
        return self.bounds[1]

    @field_validator("bounds")
    @classmethod
    def _lu(cls, b):
        if b[0] > b[1]:
            raise ValueError(f"lower bound must be <= upper bound, got {b[0]} > {b[1]}")
        return b

    def __call__(self, x, x_adapt=None):
        return (x - self.lower_bound) / (self.upper_bound - self.lower_bound)

    def affine(self) -> Tuple[float, float]:
        """g(y) = a*y + b (bofire/utils/torch_tools.py:389-398)."""
        s = 1.0 / (self.upper_bound - self.lower_bound)
        return s, -self.lower_bound * s


class MaximizeObjective(IdentityObjective):
    type: Literal["MaximizeObjective"] = "MaximizeObjective"


class MinimizeObjective(IdentityObjective):
    type: Literal["MinimizeObjective"] = "MinimizeObjective"

    def __call__(self, x, x_adapt=None):
        return -1.0 * (x - self.lower_bound) / (self.upper_bound - self.lower_bound)

    def affine(self) -> Tuple[float, float]:
        a, b = super().affine()
        return -a, -b


class CloseToTargetObjective(Objective):
    type: Literal["CloseToTargetObjective"] = "CloseToTargetObjective"
    w: Annotated[float, Field(gt=0, le=1)] = 1.0
    target_value: float
    exponent: float

    def __call__(self, x, x_adapt=None):
        return -1.0 * (np.abs(np.asarray(x) - self.target_value) ** self.exponent)


class ConstrainedObjective:
    """Objectives that become BoTorch output constraints
    (bofire/data_models/objectives/objective.py:36-37)."""


def _sigmoid(z):
    return 1.0 / (1.0 + np.exp(-z))


class SigmoidObjective(Objective, ConstrainedObjective):
    """bofire/data_models/objectives/sigmoid.py: steepness > 0, turning point tp."""
    steepness: Annotated[float, Field(gt=0)]
    tp: float
    w: Annotated[float, Field(gt=0, le=1)] = 1.0


class MaximizeSigmoidObjective(SigmoidObjective):
    type: Literal["MaximizeSigmoidObjective"] = "MaximizeSigmoidObjective"

    def __call__(self, x, x_adapt=None):
        return _sigmoid(self.steepness * (np.asarray(x) - self.tp))


class MinimizeSigmoidObjective(SigmoidObjective):
    type: Literal["MinimizeSigmoidObjective"] = "MinimizeSigmoidObjective"

    def __call__(self, x, x_adapt=None):
        return 1.0 - _sigmoid(self.steepness * (np.asarray(x) - self.tp))


class MovingMaximizeSigmoidObjective(SigmoidObjective):
    """Turning point relative to the best observed value: tp' = max(x_adapt) + tp."""
    type: Literal["MovingMaximizeSigmoidObjective"] = "MovingMaximizeSigmoidObjective"

    def get_adjusted_tp(self, x) -> float:
        return float(np.asarray(x).max()) + self.tp

    def __call__(self, x, x_adapt):
        return _sigmoid(self.steepness * (np.asarray(x) - self.get_adjusted_tp(x_adapt)))


class TargetObjective(Objective, ConstrainedObjective):
    """bofire/data_models/objectives/target.py: product of a rising sigmoid at
    target - tolerance and a falling one at target + tolerance."""
    type: Literal["TargetObjective"] = "TargetObjective"
    w: Annotated[float, Field(gt=0, le=1)] = 1.0
    target_value: float
    tolerance: Annotated[float, Field(ge=0)]
    steepness: Annotated[float, Field(gt=0)]

    def __call__(self, x, x_adapt=None):
        x = np.asarray(x)
        return (_sigmoid(self.steepness * (x - (self.target_value - self.tolerance))) *
                (1.0 - _sigmoid(self.steepness * (x - (self.target_value + self.tolerance)))))


AnyObjective = Annotated[Union[MaximizeObjective, MinimizeObjective, CloseToTargetObjective, MaximizeSigmoidObjective,
                               MinimizeSigmoidObjective, MovingMaximizeSigmoidObjective, TargetObjective],
                         Field(discriminator="type")]


# ---------------------------------------------------------------------------------------
# features
# ---------------------------------------------------------------------------------------
class Feature(BaseModel):
    type: str
    key: str
    order_id: ClassVar[int] = -1

    def __lt__(self, other) -> bool:
        if self.order_id == other.order_id:
            return self.key < other.key
        return self.order_id < other.order_id


class Input(Feature):
    pass


class Output(Feature):
    pass


class ContinuousInput(Input):
    type: Literal["ContinuousInput"] = "ContinuousInput"
    order_id: ClassVar[int] = 1
    bounds: Tuple[float, float]
    local_relative_bounds: Optional[Tuple[float, float]] = None
    stepsize: Optional[float] = None
    unit: Optional[str] = None

    @field_validator("bounds")
    @classmethod
    def _b(cls, b):
        if b[0] > b[1]:
            raise ValueError(f"lower bound must be <= upper bound, got {b[0]} > {b[1]}")
        return b

    @property
    def lower_bound(self) -> float:
        return self.bounds[0]

    @property
    def upper_bound(self) -> float:
        return self.bounds[1]

    def is_fixed(self) -> bool:
        return self.lower_bound == self.upper_bound

    def fixed_value(self, transform_type=None):
        return [self.lower_bound] if self.is_fixed() else None

    def sample(self, n: int, seed: Optional[int] = None) -> pd.Series:
        """bofire/data_models/features/continuous.py:108-122."""
        return pd.Series(name=self.key,
                         data=np.random.default_rng(seed=seed).uniform(self.lower_bound, self.upper_bound, n))

    def get_bounds(self, transform_type=None, values: Optional[pd.Series] = None,
                   reference_value: Optional[float] = None):
        """bofire/data_models/features/continuous.py:134-167."""
        if reference_value is not None and values is not None:
            raise ValueError("Only one can be used, `local_value` or `values`.")
        if values is None:
            if reference_value is None or self.is_fixed():
                return [self.lower_bound], [self.upper_bound]
            lrb = self.local_relative_bounds or (math.inf, math.inf)
            return ([max(reference_value - lrb[0], self.lower_bound)],
                    [min(reference_value + lrb[1], self.upper_bound)])
        return [min(self.lower_bound, float(values.min()))], [max(self.upper_bound, float(values.max()))]

    def validate_candidental(self, values: pd.Series) -> pd.Series:
        if not pd.api.types.is_numeric_dtype(values):
            raise ValueError(f"not all values of input feature `{self.key}` are numerical")
        values = values.astype("float64")
        tol = 1e-6
        if (values < self.lower_bound - tol).any() or (values > self.upper_bound + tol).any():
            raise ValueError(f"not all values of input feature `{self.key}` are inside the bounds "
                             f"[{self.lower_bound}, {self.upper_bound}]")
        return values


class CategoricalInput(Input):
    type: Literal["CategoricalInput"] = "CategoricalInput"
    order_id: ClassVar[int] = 7
    categories: List[str]
    allowed: Optional[List[bool]] = None

    @model_validator(mode="after")
    def _allowed(self):
        if self.allowed is None:
            self.__dict__["allowed"] = [True] * len(self.categories)
        if len(self.allowed) != len(self.categories):
            raise ValueError("allowed must have same length as categories")
        if not any(self.allowed):
            raise ValueError("no category is allowed")
        return self

    def is_fixed(self) -> bool:
        return sum(self.allowed) == 1

    def fixed_value(self, transform_type=None):
        if not self.is_fixed():
            return None
        return [self.categories[self.allowed.index(True)]]

    def get_allowed_categories(self):
        return [c for c, a in zip(self.categories, self.allowed) if a]

    def get_forbidden_categories(self):
        return [c for c, a in zip(self.categories, self.allowed) if not a]

    def to_onehot_encoding(self, values: pd.Series) -> pd.DataFrame:
        """bofire/data_models/features/categorical.py:182-196 (columns f"{key}_{cat}")."""
        return pd.DataFrame({f"{self.key}_{c}": values == c for c in self.categories}, dtype=float,
                            index=values.index)

    def from_onehot_encoding(self, values: pd.DataFrame) -> pd.Series:
        cols = [f"{self.key}_{c}" for c in self.categories]
        s = values[cols].idxmax(axis=1).str.slice(len(self.key) + 1)
        return s.rename(self.key)

    def sample(self, n: int, seed: Optional[int] = None) -> pd.Series:
        return pd.Series(name=self.key,
                         data=np.random.default_rng(seed=seed).choice(self.get_allowed_categories(), n))

    def get_bounds(self, transform_type=None, values=None, reference_value=None):
        """bofire/data_models/features/categorical.py:312-345 (ONE_HOT): optimisation bounds
        close forbidden categories; with data (model fitting) every column is [0, 1]."""
        if getattr(transform_type, "value", transform_type) != "ONE_HOT":
            raise ValueError(f"categorical `{self.key}` needs a ONE_HOT transform in this build")
        lower = [0.0] * len(self.categories)
        if values is None:
            upper = [1.0 if a else 0.0 for a in self.allowed]
        else:
            upper = [1.0] * len(self.categories)
        return lower, upper

    def validate_candidental(self, values: pd.Series) -> pd.Series:
        bad = ~values.isin(self.get_allowed_categories())
        if bad.any():
            raise ValueError(f"not all values of input feature `{self.key}` are allowed categories")
        return values


class ContinuousOutput(Output):
    type: Literal["ContinuousOutput"] = "ContinuousOutput"
    order_id: ClassVar[int] = 9
    objective: Optional[AnyObjective] = Field(default_factory=lambda: MaximizeObjective(w=1.0))
    unit: Optional[str] = None

    def __call__(self, values: pd.Series, values_adapt=None) -> pd.Series:
        if self.objective is None:
            return pd.Series(data=[np.nan] * len(values), index=values.index, name=values.name)
        return self.objective(values, values_adapt)


AnyInput = Annotated[Union[ContinuousInput, CategoricalInput], Field(discriminator="type")]
AnyOutput = Annotated[Union[ContinuousOutput], Field(discriminator="type")]


def _filter(features, includes=None, excludes=None, exact=False):
    def ok(f, types):
        types = types if isinstance(types, (list, tuple)) else [types]
        return any((type(f) is t) if exact else isinstance(f, t) for t in types)

    out = [f for f in features if (includes is None or ok(f, includes)) and (excludes is None or not ok(f, excludes))]
    return sorted(out)


class _Features(BaseModel):
    def get(self, includes=None, excludes=None, exact: bool = False):
        return self.__class__(features=_filter(self.features, includes, excludes, exact))

    def get_keys(self, includes=None, excludes=None, exact: bool = False) -> List[str]:
        return [f.key for f in self.get(includes, excludes, exact).features]

    def get_by_key(self, key: str):
        for f in self.features:
            if f.key == key:
                return f
        raise KeyError(key)

    def get_by_keys(self, keys: Sequence[str]):
        return self.__class__(features=sorted(self.get_by_key(k) for k in keys))

    def __len__(self):
        return len(self.features)

    def __iter__(self):
        return iter(sorted(self.features))

    @model_validator(mode="after")
    def _unique(self):
        keys = [f.key for f in self.features]
        if len(set(keys)) != len(keys):
            raise ValueError("Feature keys are not unique")
        return self


class Inputs(_Features):
    type: Literal["Inputs"] = "Inputs"
    features: List[AnyInput] = Field(default_factory=list)

    def get_fixed(self):
        return self.__class__(features=[f for f in self.features if f.is_fixed()])

    def _transform_info(self, specs: Dict[str, str]):
        """features2idx / features2names (bofire/data_models/domain/features.py _get_transform_info)."""
        f2i, f2n = {}, {}
        col = 0
        for feat in self.get().features:
            if isinstance(feat, CategoricalInput) and specs.get(feat.key) == "ONE_HOT":
                names = tuple(f"{feat.key}_{c}" for c in feat.categories)
            else:
                names = (feat.key,)
            f2n[feat.key] = names
            f2i[feat.key] = tuple(range(col, col + len(names)))
            col += len(names)
        return f2i, f2n

    def transform(self, experiments: pd.DataFrame, specs: Dict[str, str]) -> pd.DataFrame:
        """bofire/data_models/domain/features.py:493-533 (ONE_HOT only)."""
        feats = self.get().features
        if all(isinstance(f, ContinuousInput) for f in feats):
            return experiments[[f.key for f in feats]].astype("float64")
        parts = []
        for feat in feats:
            s = experiments[feat.key]
            if isinstance(feat, CategoricalInput):
                if specs.get(feat.key) != "ONE_HOT":
                    raise ValueError(f"unsupported transform for `{feat.key}`")
                parts.append(feat.to_onehot_encoding(s))
            else:
                parts.append(s.astype("float64"))
        return pd.concat(parts, axis=1)

    def inverse_transform(self, transformed: pd.DataFrame, specs: Dict[str, str]) -> pd.DataFrame:
        feats = self.get().features
        if all(isinstance(f, ContinuousInput) for f in feats):
            return transformed[[f.key for f in feats]]
        parts = []
        for feat in self.get().features:
            if isinstance(feat, CategoricalInput):
                parts.append(feat.from_onehot_encoding(transformed))
            else:
                parts.append(transformed[feat.key])
        return pd.concat(parts, axis=1)

    def get_bounds(self, specs: Dict[str, str], experiments: Optional[pd.DataFrame] = None,
                   reference_experiment: Optional[pd.Series] = None):
        """bofire/data_models/domain/features.py:628-679."""
        if reference_experiment is not None and experiments is not None:
            raise ValueError("Only one can be used, `reference_experiments` or `experiments`.")
        lower, upper = [], []
        for feat in self.get().features:
            lo, up = feat.get_bounds(
                transform_type=specs.get(feat.key),
                values=experiments[feat.key] if experiments is not None else None,
                reference_value=(reference_experiment[feat.key] if reference_experiment is not None else None),
            )
            lower += lo
            upper += up
        return lower, upper

    def sample(self, n: int = 1, seed: Optional[int] = None) -> pd.DataFrame:
        rng = np.random.default_rng(seed)
        return pd.concat([f.sample(n, seed=int(rng.integers(1, 1_000_000))) for f in self.get().features], axis=1)

    def validate_experiments(self, experiments: pd.DataFrame, strict: bool = False) -> pd.DataFrame:
        for feat in self.features:
            if feat.key not in experiments:
                raise ValueError(f"no col in experiments for feature {feat.key}")
            if experiments[feat.key].isnull().any():
                raise ValueError(f"there are null values in column {feat.key}")
            if isinstance(feat, ContinuousInput):
                if not pd.api.types.is_numeric_dtype(experiments[feat.key]):
                    raise ValueError(f"not all values of input feature `{feat.key}` are numerical")
                experiments[feat.key] = experiments[feat.key].astype("float64")
        return experiments

    def check_continuous_candidates(self, candidates: pd.DataFrame) -> np.ndarray:
        """validate_candidates of an all-continuous Inputs on arrays: the numeric-dtype and
        bound checks (same errors, same order), returning the n x d float64 values (one
        positional gather instead of DataFrame selections)."""
        feats = self.get().features
        cols = candidates.columns
        idx = cols.get_indexer([f.key for f in feats])
        for f, i in zip(feats, idx):
            if i < 0:
                raise ValueError(f"no col for input feature `{f.key}`")
        dts = candidates.dtypes.to_numpy()
        for f, i in zip(feats, idx):
            if not pd.api.types.is_numeric_dtype(dts[i]):
                raise ValueError(f"not all values of input feature `{f.key}` are numerical")
        if all(dt == np.float64 for dt in dts):
            vals = candidates.to_numpy(dtype=np.float64)[:, idx]
        else:
            vals = np.column_stack([candidates.iloc[:, i].to_numpy(dtype=np.float64) for i in idx])
        lo = np.array([f.lower_bound for f in feats]) - 1e-6
        hi = np.array([f.upper_bound for f in feats]) + 1e-6
        bad = ((vals < lo) | (vals > hi)).any(axis=0)
        for f, b in zip(feats, bad):
            if b:
                raise ValueError(f"not all values of input feature `{f.key}` are inside the bounds "
                                 f"[{f.lower_bound}, {f.upper_bound}]")
        return np.ascontiguousarray(vals)

    def validate_candidates(self, candidates: pd.DataFrame) -> pd.DataFrame:
        """Per-feature checks of ContinuousInput / CategoricalInput.validate_candidental, the
        continuous columns' bounds tested in one array pass (same errors, same order)."""
        feats = self.get().features
        for feat in feats:
            if feat.key not in candidates:
                raise ValueError(f"no col for input feature `{feat.key}`")
        if all(isinstance(f, ContinuousInput) for f in feats):
            vals = self.check_continuous_candidates(candidates)
            return pd.DataFrame(vals, columns=[f.key for f in feats], index=candidates.index)
        dtypes = candidates.dtypes
        cont = [f for f in feats if isinstance(f, ContinuousInput)]
        if cont:
            for f in cont:
                if not pd.api.types.is_numeric_dtype(dtypes[f.key]):
                    raise ValueError(f"not all values of input feature `{f.key}` are numerical")
            vals = candidates[[f.key for f in cont]].to_numpy(dtype=np.float64)
            lo = np.array([f.lower_bound for f in cont]) - 1e-6
            hi = np.array([f.upper_bound for f in cont]) + 1e-6
            bad = ((vals < lo) | (vals > hi)).any(axis=0)
            for f, b in zip(cont, bad):
                if b:
                    raise ValueError(f"not all values of input feature `{f.key}` are inside the bounds "
                                     f"[{f.lower_bound}, {f.upper_bound}]")
        for feat in feats:
            if isinstance(feat, ContinuousInput):
                if dtypes[feat.key] != np.float64:
                    candidates[feat.key] = candidates[feat.key].astype("float64")
            else:
                candidates[feat.key] = feat.validate_candidental(candidates[feat.key])
        return candidates[[f.key for f in feats]]


class Outputs(_Features):
    type: Literal["Outputs"] = "Outputs"
    features: List[AnyOutput] = Field(default_factory=list)

    def get_by_objective(self, includes=None, excludes=None, exact: bool = False):
        incl = includes if includes is not None else [Objective]
        incl = incl if isinstance(incl, (list, tuple)) else [incl]
        out = []
        for f in self.features:
            if f.objective is None:
                continue
            if not any(isinstance(f.objective, t) for t in incl):
                continue
            if excludes is not None:
                ex = excludes if isinstance(excludes, (list, tuple)) else [excludes]
                if any(isinstance(f.objective, t) for t in ex):
                    continue
            out.append(f)
        return Outputs(features=sorted(out))

    def get_keys_by_objective(self, includes=None, excludes=None, exact: bool = False) -> List[str]:
        return [f.key for f in self.get_by_objective(includes, excludes, exact).features]

    def __call__(self, experiments: pd.DataFrame, experiments_adapt=None, predictions: bool = False) -> pd.DataFrame:
        """Desirabilities (bofire/data_models/domain/features.py:783-848): objective values of
        every output with an objective, the adaptive objectives (MovingMaximizeSigmoid) fed
        with the non-null observed values of experiments_adapt.  The objectives run on the
        column arrays and the frame is built once (same values, same column names)."""
        if predictions and experiments_adapt is None:
            raise ValueError("If predictions are used, `experiments_adapt` has to be provided.")
        adapt = experiments if experiments_adapt is None else experiments_adapt
        col = (lambda k: experiments[f"{k}_pred"].to_numpy(dtype=np.float64)) if predictions else \
            (lambda k: experiments[k].to_numpy(dtype=np.float64))
        return pd.DataFrame(self.desirability_arrays(col, adapt), index=experiments.index)

    def desirability_arrays(self, values, adapt) -> Dict[str, np.ndarray]:
        """{key_des: objective(values(key))} for every output with an objective, in feature
        order; values(key) gives the output's value array, adapt the observed experiments the
        adaptive objectives (MovingMaximizeSigmoid) read."""
        cols = {}
        for feat in self.get().features:
            if feat.objective is None:
                continue
            xa = None
            if isinstance(feat.objective, MovingMaximizeSigmoidObjective):
                xa = adapt[feat.key].dropna().to_numpy(dtype=np.float64)
            cols[f"{feat.key}_des"] = np.asarray(feat.objective(values(feat.key), xa), dtype=np.float64)
        return cols

    def preprocess_experiments_all_valid_outputs(self, experiments: pd.DataFrame,
                                                 output_feature_keys: Optional[List[str]] = None) -> pd.DataFrame:
        """bofire/data_models/domain/features.py:951-974."""
        keys = output_feature_keys or self.get_keys()
        # one row mask (valid_<key> > 0 for every key that has the column, no NaN in the
        # output columns) and one selection instead of a filtered copy per key
        keep = np.ones(len(experiments), dtype=bool)
        for k in keys:
            vk = f"valid_{k}"
            if vk in experiments:
                keep &= np.asarray(experiments[vk] > 0, dtype=bool)
        keep &= ~experiments[list(keys)].isna().to_numpy().any(axis=1)
        return experiments if keep.all() else experiments[keep]

    def validate_experiments(self, experiments: pd.DataFrame) -> pd.DataFrame:
        for feat in self.features:
            if feat.key not in experiments:
                raise ValueError(f"no col in experiments for feature {feat.key}")
            if not pd.api.types.is_numeric_dtype(experiments[feat.key]):
                raise ValueError(f"not all values of output feature `{feat.key}` are numerical")
            vk = f"valid_{feat.key}"
            if vk not in experiments:
                experiments[vk] = True
            experiments[feat.key] = experiments[feat.key].astype("float64")
        return experiments


# ---------------------------------------------------------------------------------------
# constraints  (bofire/data_models/constraints/linear.py)
# ---------------------------------------------------------------------------------------
class LinearConstraint(BaseModel):
    type: str
    features: List[str]
    coefficients: List[float]
    rhs: float

    @model_validator(mode="after")
    def _len(self):
        if len(self.features) != len(self.coefficients):
            raise ValueError("must provide same number of features and coefficients")
        return self

    def lhs(self, df: pd.DataFrame) -> pd.Series:
        return (df[self.features] * np.asarray(self.coefficients)).sum(axis=1)


class LinearEqualityConstraint(LinearConstraint):
    type: Literal["LinearEqualityConstraint"] = "LinearEqualityConstraint"

    def is_fulfilled(self, df: pd.DataFrame, tol: float = 1e-6) -> pd.Series:
        return np.isclose(self.lhs(df), self.rhs, atol=tol)


class LinearInequalityConstraint(LinearConstraint):
    """sum_i c_i x_i <= rhs."""
    type: Literal["LinearInequalityConstraint"] = "LinearInequalityConstraint"

    def is_fulfilled(self, df: pd.DataFrame, tol: float = 1e-6) -> pd.Series:
        return (self.lhs(df) - self.rhs) <= tol


AnyConstraint = Annotated[Union[LinearEqualityConstraint, LinearInequalityConstraint], Field(discriminator="type")]


class Constraints(BaseModel):
    type: Literal["Constraints"] = "Constraints"
    constraints: List[AnyConstraint] = Field(default_factory=list)

    def get(self, includes=None, excludes=None):
        incl = includes if includes is None or isinstance(includes, (list, tuple)) else [includes]
        ex = excludes if excludes is None or isinstance(excludes, (list, tuple)) else [excludes]
        out = [c for c in self.constraints if (incl is None or any(isinstance(c, t) for t in incl))
               and (ex is None or not any(isinstance(c, t) for t in ex))]
        return Constraints(constraints=out)

    def is_fulfilled(self, df: pd.DataFrame, tol: float = 1e-6) -> pd.Series:
        if len(self.constraints) == 0:
            return pd.Series([True] * len(df), index=df.index)
        ok = np.ones(len(df), dtype=bool)
        for c in self.constraints:
            ok &= np.asarray(c.is_fulfilled(df, tol), dtype=bool)
        return pd.Series(ok, index=df.index)

    def __len__(self):
        return len(self.constraints)

    def __iter__(self):
        return iter(self.constraints)


class Domain(BaseModel):
    type: Literal["Domain"] = "Domain"
    inputs: Inputs = Field(default_factory=Inputs)
    outputs: Outputs = Field(default_factory=Outputs)
    constraints: Constraints = Field(default_factory=Constraints)

    @classmethod
    def from_lists(cls, inputs=None, outputs=None, constraints=None) -> "Domain":
        return cls(inputs=Inputs(features=inputs or []), outputs=Outputs(features=outputs or []),
                   constraints=Constraints(constraints=constraints or []))

    @model_validator(mode="after")
    def _keys(self):
        ik, ok = set(self.inputs.get_keys()), set(self.outputs.get_keys())
        if ik & ok:
            raise ValueError("Feature keys are not unique")
        for c in self.constraints:
            for f in c.features:
                if f not in ik:
                    raise ValueError(f"constraint feature `{f}` is not an input")
        return self

    def validate_experiments(self, experiments: pd.DataFrame, strict: bool = False) -> pd.DataFrame:
        """bofire/data_models/domain/domain.py:334-385."""
        if len(experiments) == 0:
            raise ValueError("no experiments provided (empty dataframe)")
        experiments = experiments.copy()
        experiments = self.inputs.validate_experiments(experiments, strict=strict)
        experiments = self.outputs.validate_experiments(experiments)
        return experiments

    def validate_candidates(self, candidates: pd.DataFrame, only_inputs: bool = False, tol: float = 1e-5,
                            raise_validation_error: bool = True, inputs_validated: bool = False) -> pd.DataFrame:
        """bofire/data_models/domain/domain.py:417-459.  inputs_validated: the caller has just
        validated this very frame's inputs (PredictiveStrategy.ask after Strategy.ask); without
        constraints the input checks are not repeated (the output columns still are)."""
        if inputs_validated and not len(self.constraints):
            pass
        elif all(isinstance(f, ContinuousInput) for f in self.inputs.get().features):
            # continuous inputs: the checks on one gathered array; the validated input frame is
            # only formed when constraints need it
            vals = self.inputs.check_continuous_candidates(candidates)
            cand = None
            if len(self.constraints):
                cand = pd.DataFrame(vals, columns=self.inputs.get_keys(), index=candidates.index)
        else:
            cand = self.inputs.validate_candidates(candidates.copy())
        if len(self.constraints) and not self.constraints.is_fulfilled(cand, tol=tol).all():
            if raise_validation_error:
                raise ConstraintNotFulfilledError(f"Constraints not fulfilled: {cand}")
            warnings.warn("Not all constraints are fulfilled.")
        if not only_inputs:
            for feat in self.outputs.get().features:
                for suffix in ("_pred", "_sd"):
                    if f"{feat.key}{suffix}" not in candidates:
                        raise ValueError(f"missing column {feat.key}{suffix}")
        return candidates
