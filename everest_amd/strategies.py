"""Functional strategies with BoFire's API — ``map(data_model)`` returns an object with
``tell / ask / predict / calc_acquisition`` (bofire/strategies/{strategy,random}.py,
bofire/strategies/predictives/{predictive,botorch,qehvi,qnehvi,sobo}.py).

The dense work (GP fit and posterior, qNEHVI / qEI construction and evaluation) runs on the
MI355X through ``everest_amd.gp`` / ``everest_amd.acquisition``; the orchestration (pandas,
scipy optimiser, box decomposition threads) runs on the host as in the reference.
Multi-GPU: pass ``dist=torch.distributed`` (one process per GPU, RCCL) to shard the
acquisition evaluations of ``ask()`` (everest_amd/optim.py).
"""
from __future__ import annotations

import os
import warnings
from typing import List, Optional, Sequence, Tuple

import numpy as np
import pandas as pd
import torch

from . import data_models as dm
from . import ops
from .acquisition import QEHVI, QEI, QEIJoint, QLogEHVI, QLogNEHVI, QNEHVI, prefetch_scramble
from .data_models.domain import CloseToTargetObjective, MaximizeObjective, MinimizeObjective
from .optim import (OptimizeStats, hit_and_run, host_values, optimize_acqf, optimize_acqf_mixed,
                    prefetch_raw_samples)
from .surrogates import BotorchSurrogates, device


# ---------------------------------------------------------------------------------------
# helpers restated from bofire/utils
# ---------------------------------------------------------------------------------------
def get_column_names(outputs) -> Tuple[List[str], List[str]]:
    """bofire/utils/naming_conventions.py:9-33 (continuous outputs)."""
    keys = outputs.get_keys(dm.ContinuousOutput)
    return [f"{k}_pred" for k in keys], [f"{k}_sd" for k in keys]


def get_ref_point_mask(domain, output_feature_keys=None) -> np.ndarray:
    """bofire/utils/multiobjective.py:18-55."""
    if output_feature_keys is None:
        output_feature_keys = domain.outputs.get_keys_by_objective(
            [MaximizeObjective, MinimizeObjective, CloseToTargetObjective])
    if len(output_feature_keys) < 2:
        raise ValueError("At least two output features have to be provided.")
    mask = []
    for key in output_feature_keys:
        obj = domain.outputs.get_by_key(key).objective
        if isinstance(obj, MaximizeObjective):
            mask.append(1.0)
        elif isinstance(obj, (MinimizeObjective, CloseToTargetObjective)):
            mask.append(-1.0)
        else:
            raise ValueError("Only `MaximizeObjective` and `MinimizeObjective` supported")
    return np.array(mask)


def multiobjective_values(outputs, Y: np.ndarray) -> np.ndarray:
    """get_multiobjective_objective (bofire/utils/torch_tools.py:699-727) on a numpy array of
    the objective outputs (columns in get_keys_by_objective order)."""
    cols = []
    feats = outputs.get_by_objective([MaximizeObjective, MinimizeObjective, CloseToTargetObjective]).features
    for j, f in enumerate(feats):
        cols.append(np.asarray(f.objective(Y[:, j]), dtype=np.float64))
    return np.stack(cols, axis=-1)


def infer_ref_point(domain, experiments: pd.DataFrame, return_masked: bool = False) -> dict:
    """bofire/utils/multiobjective.py:133-159."""
    keys = domain.outputs.get_keys_by_objective([MaximizeObjective, MinimizeObjective, CloseToTargetObjective])
    df = domain.outputs.preprocess_experiments_all_valid_outputs(experiments, output_feature_keys=keys)
    ref = multiobjective_values(domain.outputs, df[keys].values).min(axis=0)
    mask = get_ref_point_mask(domain)
    if return_masked is False:
        ref = ref / mask
    return {k: ref[i] for i, k in enumerate(keys)}


def get_linear_constraints(domain, constraint_type, unit_scaled: bool = False):
    """bofire/utils/torch_tools.py:45-102: BoTorch form (indices, coefficients, rhs) meaning
    sum coefficients * x[indices] >= rhs."""
    out = []
    keys = domain.inputs.get_keys(dm.domain.Input)
    for c in domain.constraints.get(constraint_type).constraints:
        idx, coef, rhs = [], [], 0.0
        for i, fk in enumerate(c.features):
            feat = domain.inputs.get_by_key(fk)
            if feat.is_fixed():
                rhs -= feat.fixed_value()[0] * c.coefficients[i]
            else:
                idx.append(keys.index(fk))
                coef.append(c.coefficients[i])
        out.append((np.asarray(idx), -np.asarray(coef, dtype=np.float64), -(rhs + c.rhs)))
    return out


# ---------------------------------------------------------------------------------------
# strategy base classes
# ---------------------------------------------------------------------------------------
class Strategy:
    """bofire/strategies/strategy.py:14-280."""

    def __init__(self, data_model):
        self.domain = data_model.domain
        # bofire/strategies/strategy.py:26: `seed or random` — a seed of 0 counts as no seed
        # (draws a random one), as in the reference
        self.seed = data_model.seed or int(np.random.default_rng().integers(1000))
        self.rng = np.random.default_rng(self.seed)
        self._experiments: Optional[pd.DataFrame] = None
        self._candidates: Optional[pd.DataFrame] = None

    @classmethod
    def from_spec(cls, data_model):
        return cls(data_model=data_model)

    def _get_seed(self) -> int:
        return int(self.rng.integers(1, 100000))

    @property
    def experiments(self) -> Optional[pd.DataFrame]:
        return self._experiments

    @property
    def candidates(self) -> Optional[pd.DataFrame]:
        return self._candidates

    def tell(self, experiments: pd.DataFrame, replace: bool = False) -> None:
        if len(experiments) == 0:
            return
        if replace:
            self.set_experiments(experiments)
        else:
            self.add_experiments(experiments)
        self._tell()

    def _tell(self) -> None:
        pass

    def ask(self, candidate_count: Optional[int] = None, add_pending: bool = False,
            raise_validation_error: bool = True) -> pd.DataFrame:
        if candidate_count is not None and candidate_count < 1:
            raise ValueError(f"Candidate_count has to be at least 1 but got {candidate_count}.")
        if not self.has_sufficient_experiments():
            raise ValueError("Not enough experiments available to execute the strategy.")
        candidates = self._ask(candidate_count=candidate_count)
        self.domain.validate_candidates(candidates=candidates, only_inputs=True,
                                        raise_validation_error=raise_validation_error)
        if candidate_count is not None and len(candidates) != candidate_count:
            warnings.warn(f"Expected {candidate_count} candidates, got {len(candidates)}", UserWarning)
        if add_pending:
            self.add_candidates(candidates)
        return candidates

    def has_sufficient_experiments(self) -> bool:
        raise NotImplementedError

    def _ask(self, candidate_count=None) -> pd.DataFrame:
        raise NotImplementedError

    def set_candidates(self, candidates: pd.DataFrame):
        c = self.domain.inputs.validate_experiments(candidates[self.domain.inputs.get_keys()].copy())
        self._candidates = c[self.domain.inputs.get_keys()]

    def add_candidates(self, candidates: pd.DataFrame):
        c = self.domain.inputs.validate_experiments(candidates[self.domain.inputs.get_keys()].copy())
        c = c[self.domain.inputs.get_keys()]
        self._candidates = c if self._candidates is None else pd.concat((self._candidates, c), ignore_index=True)

    def reset_candidates(self):
        self._candidates = None

    @property
    def num_candidates(self) -> int:
        return 0 if self._candidates is None else len(self._candidates)

    def set_experiments(self, experiments: pd.DataFrame):
        self._experiments = self.domain.validate_experiments(experiments)

    def add_experiments(self, experiments: pd.DataFrame):
        e = self.domain.validate_experiments(experiments)
        self._experiments = e if self._experiments is None else pd.concat((self._experiments, e), ignore_index=True)

    @property
    def num_experiments(self) -> int:
        return 0 if self._experiments is None else len(self._experiments)


class RandomStrategy(Strategy):
    """Uniform sampling in the bounds; polytope (hit-and-run) sampling with linear
    constraints (bofire/strategies/random.py:70-140)."""

    def has_sufficient_experiments(self) -> bool:
        return True

    def _ask(self, candidate_count: Optional[int] = None) -> pd.DataFrame:
        n = candidate_count or 1
        inputs = self.domain.inputs
        cont = inputs.get(dm.ContinuousInput)
        lin = self.domain.constraints.get([dm.LinearInequalityConstraint, dm.LinearEqualityConstraint])
        if len(lin) == 0:
            return inputs.sample(n, seed=self._get_seed())
        keys = cont.get_keys()
        lo = np.array([f.lower_bound for f in cont.features])
        hi = np.array([f.upper_bound for f in cont.features])
        ineq = get_linear_constraints(self.domain, dm.LinearInequalityConstraint)
        eq = get_linear_constraints(self.domain, dm.LinearEqualityConstraint)
        X = hit_and_run(np.stack([lo, hi]), ineq, eq, n, seed=self._get_seed(), n_burnin=1000, n_thinning=32)
        df = pd.DataFrame(X, columns=keys)
        others = inputs.get(excludes=dm.ContinuousInput)
        if len(others):
            df = pd.concat([df, others.sample(n, seed=self._get_seed())], axis=1)
        return df[inputs.get_keys()]


class PredictiveStrategy(Strategy):
    """bofire/strategies/predictives/predictive.py:20-216."""

    def __init__(self, data_model):
        super().__init__(data_model)
        self.is_fitted = False

    def ask(self, candidate_count: Optional[int] = None, add_pending: bool = False,
            raise_validation_error: bool = True) -> pd.DataFrame:
        candidates = super().ask(candidate_count=candidate_count, add_pending=add_pending,
                                 raise_validation_error=raise_validation_error)
        # Strategy.ask validated this frame's inputs (and constraints) a moment ago: only the
        # prediction columns are new to check
        self.domain.validate_candidates(candidates=candidates, raise_validation_error=raise_validation_error,
                                        inputs_validated=True)
        return candidates

    def tell(self, experiments: pd.DataFrame, replace: bool = False, retrain: bool = True):
        if len(experiments) == 0:
            return
        if replace:
            self.set_experiments(experiments)
        else:
            self.add_experiments(experiments)
        if retrain and self.has_sufficient_experiments():
            self.fit()
            self._tell()

    def predict(self, experiments: pd.DataFrame) -> pd.DataFrame:
        if self.is_fitted is not True:
            raise ValueError("Model not yet fitted.")
        preds, stds = self._predict(experiments)
        return self._predictions_frame(preds, stds, experiments.index)

    def _predictions_frame(self, preds: np.ndarray, stds: np.ndarray, index) -> pd.DataFrame:
        """[pred | sd | desirability] columns of predict() (the reference builds the
        prediction frame, evaluates the objectives on it and concatenates): one array, one
        frame."""
        pred_cols, sd_cols = get_column_names(self.domain.outputs)
        pos = {c: i for i, c in enumerate(pred_cols)}
        des = self.domain.outputs.desirability_arrays(lambda k: preds[:, pos[f"{k}_pred"]], self.experiments)
        data = np.hstack([preds, stds] + [v.reshape(-1, 1) for v in des.values()])
        return pd.DataFrame(data, columns=pred_cols + sd_cols + list(des), index=index)

    def fit(self):
        assert self.experiments is not None and len(self.experiments) > 0, "No fitting data available"
        self.domain.validate_experiments(self.experiments, strict=True)
        self._fit(self.experiments)
        self.is_fitted = True


class BotorchStrategy(PredictiveStrategy):
    """bofire/strategies/predictives/botorch.py:58-750 (continuous search spaces)."""

    def __init__(self, data_model, dist=None):
        super().__init__(data_model)
        self.num_restarts = data_model.num_restarts
        self.num_raw_samples = data_model.num_raw_samples
        self.maxiter = data_model.maxiter
        self.batch_limit = data_model.batch_limit
        self.surrogate_specs = data_model.surrogate_specs
        self.categorical_method = getattr(data_model.categorical_method, "value", data_model.categorical_method)
        self.surrogates: Optional[BotorchSurrogates] = None
        self.model = None
        self.dist = dist
        # torch.manual_seed(self.seed) in the reference (botorch.py:86); a private generator here
        self.gen = torch.Generator().manual_seed(int(self.seed))
        self.last_ask_stats: Optional[OptimizeStats] = None

    @property
    def input_preprocessing_specs(self):
        return {k: (v.value if hasattr(v, "value") else v)
                for k, v in self.surrogate_specs.input_preprocessing_specs.items()}

    def _get_optimizer_options(self) -> dict:
        return {"batch_limit": self.batch_limit, "maxiter": self.maxiter}

    def _fit(self, experiments: pd.DataFrame):
        self.surrogates = BotorchSurrogates(self.surrogate_specs)
        self.surrogates.fit(experiments)
        self.model = self.surrogates.compatibilize(self.domain.inputs, self.domain.outputs)

    def _transform(self, df: pd.DataFrame) -> np.ndarray:
        return self.domain.inputs.transform(df[self.domain.inputs.get_keys()],
                                            self.input_preprocessing_specs).values.astype(np.float64)

    def _predict(self, experiments: pd.DataFrame):
        X = torch.as_tensor(self._transform(experiments), dtype=torch.float64, device=self.model.device)
        mean, var = self.model.posterior(X, observation_noise=True)
        return mean.T.cpu().numpy(), np.sqrt(var.T.cpu().numpy())

    def _valid_experiments(self) -> pd.DataFrame:
        """preprocess_experiments_all_valid_outputs of the current experiments, computed once
        per experiments frame (tell / set / add replace the frame object)."""
        c = getattr(self, "_valid_cache", None)
        if c is not None and c[0] is self._experiments:
            return c[1]
        v = self.domain.outputs.preprocess_experiments_all_valid_outputs(self.experiments)
        self._valid_cache = (self._experiments, v)
        self._xtrain_cache = None
        return v

    def has_sufficient_experiments(self) -> bool:
        if self.experiments is None:
            return False
        return len(self._valid_experiments()) > 1

    def get_acqf_input_tensors(self):
        """bofire/strategies/predictives/botorch.py:696-724."""
        ex = self._valid_experiments()
        c = getattr(self, "_xtrain_cache", None)
        if c is not None and c[0] is ex:
            X_train = c[1]
        else:
            clean = ex.drop_duplicates(subset=self.domain.inputs.get_keys(), keep="first")
            X_train = self._transform(clean)
            self._xtrain_cache = (ex, X_train)
        X_pending = self._transform(self.candidates) if self.candidates is not None else None
        extra = getattr(self, "_extra_pending", None)
        if extra is not None and len(extra):
            X_pending = extra if X_pending is None else np.concatenate([X_pending, extra], 0)
        return X_train.copy(), X_pending

    def calc_acquisition(self, candidates: pd.DataFrame, combined: bool = False) -> np.ndarray:
        """bofire/strategies/predictives/botorch.py:196-225: one value per candidate, or with
        ``combined`` one joint value of the whole set as a q-batch."""
        acqf = self._get_acqfs(len(candidates) if combined else 1)[0]
        X = torch.as_tensor(self._transform(candidates), dtype=torch.float64, device=self.model.device)
        if combined:
            X = X.unsqueeze(0)
        return host_values(acqf.forward(X))

    def _bounds(self) -> np.ndarray:
        lo, hi = self.domain.inputs.get_bounds(specs=self.input_preprocessing_specs)
        return np.array([lo, hi], dtype=np.float64)

    def _ask(self, candidate_count: Optional[int] = None) -> pd.DataFrame:
        if candidate_count is None:
            candidate_count = 1
        assert candidate_count > 0, "candidate_count has to be larger than zero."
        if self.experiments is None:
            raise ValueError("No experiments have been provided yet.")
        q = int(candidate_count)
        ineq = get_linear_constraints(self.domain, dm.LinearInequalityConstraint)
        eq = get_linear_constraints(self.domain, dm.LinearEqualityConstraint)
        combos = self.get_categorical_combinations()
        if len(combos) > 1 and q > 1:
            # EXHAUSTIVE categoricals with a batch: [upstream] optimize_acqf_mixed(q > 1) is a
            # sequential greedy — q rounds of the q = 1 mixed optimisation, each round's winner
            # added to the acquisition's pending points (acq_function.set_X_pending) — so the
            # acquisition is rebuilt per round with the same seeds (the generator is rewound)
            # and the chosen rows as extra pending points
            x, val, stats = self._ask_mixed_sequential(q, combos, ineq, eq)
            stats.best_value = val
            self.last_ask_stats = stats
            return self._postprocess_candidates(x.reshape(q, -1))
        # only this call site runs optimize_acqf's raw screening: the acquisition builder may
        # start that draw early (calc_acquisition and the mixed paths never use it)
        self._prefetch_raw = len(combos) <= 1
        try:
            acqf = self._get_acqfs(q)[0]
        finally:
            self._prefetch_raw = False
        if len(combos) > 1:     # EXHAUSTIVE categorical method: optimize_acqf_mixed
            x, val, stats = optimize_acqf_mixed(acqf, self._bounds(), combos, self.num_restarts, self.num_raw_samples,
                                                self._get_optimizer_options(), self.gen, ineq, eq, dist=self.dist,
                                                q=q)
        else:
            # the next ask's first draws are known once the Boltzmann initialisation has drawn:
            # its prefetch overlaps the restart loop
            x, val, stats = optimize_acqf(acqf, self._bounds(), self.num_restarts, self.num_raw_samples,
                                          self._get_optimizer_options(), self.gen, ineq, eq, dist=self.dist,
                                          fixed_features=combos[0] or None, q=q, on_init=self._prefetch_next_ask)
        stats.best_value = val
        self.last_ask_stats = stats
        out = self._postprocess_candidates(x.reshape(q, -1))
        self._prefetch_next_ask()
        return out

    def _prefetch_next_ask(self) -> None:
        """Hook run at the end of ask(): strategies whose next acquisition starts with seed
        draws of a known size may start that work early (QnehviStrategy)."""

    def _ask_mixed_sequential(self, q: int, combos, ineq, eq):
        """optimize_acqf_mixed with q > 1 (botorch.optim.optimize_mixed, sequential branch):
        returns (q x d candidates, list of the rounds' values, stats of the last round)."""
        # The reference builds the acquisition once (its sampler / prune seeds are drawn from
        # the global generator then) and every round's optimiser draws follow those; here the
        # acquisition is rebuilt per round from the same seed state, and the optimiser stream
        # continues from where the previous round (round 1: the build) left it.
        seed_state = self.gen.get_state()
        opt_state = None
        chosen, values = [], []
        stats = None
        try:
            for _ in range(q):
                self.gen.set_state(seed_state)            # same acquisition seeds every round
                self._extra_pending = np.asarray(chosen) if chosen else None
                acqf = self._get_acqfs(1)[0]
                if opt_state is None:
                    opt_state = self.gen.get_state()      # round 1: the draws after the build
                self.gen.set_state(opt_state)             # the optimiser's draws continue
                x, v, stats = optimize_acqf_mixed(acqf, self._bounds(), combos, self.num_restarts,
                                                  self.num_raw_samples, self._get_optimizer_options(), self.gen, ineq,
                                                  eq, dist=self.dist, q=1)
                opt_state = self.gen.get_state()
                chosen.append(np.asarray(x, dtype=np.float64).reshape(-1))
                values.append(v)
        finally:
            self._extra_pending = None
        return np.stack(chosen), values, stats

    def get_fixed_features(self) -> dict:
        """bofire/strategies/predictives/botorch.py:530-595 (continuous / one-hot part):
        fixed inputs, and with the FREE categorical method the forbidden one-hot columns."""
        f2i, _ = self.domain.inputs._transform_info(self.input_preprocessing_specs)
        fixed = {}
        for feat in self.domain.inputs.get().features:
            fv = feat.fixed_value() if hasattr(feat, "fixed_value") else None
            if fv is not None:
                if isinstance(feat, dm.CategoricalInput):
                    enc = feat.to_onehot_encoding(pd.Series([fv[0]])).values[0]
                    for j, idx in enumerate(f2i[feat.key]):
                        fixed[idx] = float(enc[j])
                else:
                    fixed[f2i[feat.key][0]] = float(fv[0])
        if self.categorical_method == "FREE":
            for feat in self.domain.inputs.get([dm.CategoricalInput]).features:
                if self.input_preprocessing_specs.get(feat.key) == "ONE_HOT" and not feat.is_fixed():
                    for cat in feat.get_forbidden_categories():
                        j = feat.categories.index(cat)
                        fixed[f2i[feat.key][j]] = 0.0
        return fixed

    def get_categorical_combinations(self) -> list:
        """bofire/strategies/predictives/botorch.py:597-672 (ONE_HOT categoricals): with the
        EXHAUSTIVE categorical method every combination of allowed categories (itertools
        product in input order) becomes one fixed-feature dict on top of the fixed basis."""
        import itertools

        basis = self.get_fixed_features()
        if self.categorical_method == "FREE":
            return [basis]
        feats = [f for f in self.domain.inputs.get([dm.CategoricalInput]).features if not f.is_fixed()]
        if not feats:
            return [basis]
        f2i, _ = self.domain.inputs._transform_info(self.input_preprocessing_specs)
        out = []
        for combo in itertools.product(*[[(f, c) for c in f.get_allowed_categories()] for f in feats]):
            ff = dict(basis)
            for f, c in combo:
                enc = f.to_onehot_encoding(pd.Series([c])).values[0]
                for j, idx in enumerate(f2i[f.key]):
                    ff[idx] = float(enc[j])
            out.append(ff)
        return out

    def _postprocess_candidates(self, X: np.ndarray) -> pd.DataFrame:
        f2i, f2n = self.domain.inputs._transform_info(self.input_preprocessing_specs)
        keys = self.domain.inputs.get_keys()
        cols = [n for k in keys for n in f2n[k]]
        df = pd.DataFrame(X, columns=cols)
        if cols == keys:
            # continuous inputs: the transform is the identity, so X is the candidates' frame;
            # predictions on the transformed X directly, one frame for inputs + predictions
            if self.is_fitted is not True:
                raise ValueError("Model not yet fitted.")
            Xt = torch.as_tensor(np.ascontiguousarray(X, dtype=np.float64), device=self.model.device)
            mean, var = self.model.posterior(Xt, observation_noise=True)
            mv = torch.stack((mean, var)).cpu().numpy()      # one device -> host copy for both
            preds = self._predictions_frame(mv[0].T, np.sqrt(mv[1].T), df.index)
            return pd.DataFrame(np.hstack([np.asarray(X, dtype=np.float64), preds.to_numpy()]),
                                columns=keys + list(preds.columns))
        df = self.domain.inputs.inverse_transform(df, self.input_preprocessing_specs)
        preds = self.predict(df)
        return pd.concat((df, preds), axis=1)

    def _get_acqfs(self, n):
        raise NotImplementedError


def objective_term(objective, idx: int):
    """get_objective_callable (bofire/utils/torch_tools.py:384-402) as the device kernels'
    objective description (output, kind, p0, p1): Maximize / Minimize -> the affine
    g = a*y + b of (y - lb) / (ub - lb) (negated for Minimize), CloseToTarget ->
    g = -|y - target|^exponent."""
    if isinstance(objective, CloseToTargetObjective):
        return (int(idx), ops.OBJ_CLOSE_TO_TARGET, float(objective.target_value), float(objective.exponent))
    if isinstance(objective, (MaximizeObjective, MinimizeObjective)):
        a, b = objective.affine()
        return (int(idx), ops.OBJ_AFFINE, float(a), float(b))
    raise NotImplementedError(f"objective {type(objective).__name__} has no device kernel")


def constrained_objective_terms(objective, idx: int, x_adapt=None):
    """constrained_objective2botorch (bofire/utils/torch_tools.py:258-337) as the device
    kernels' constraint description: one (output, sign, threshold, eta) per BoTorch
    constraint callable c(Z) = sign * (Z[..., idx] - threshold), feasible for c <= 0, with
    eta = 1 / steepness; the device weight is exp(sum_c logsigmoid(-c / eta))
    ([upstream] compute_smoothed_feasibility_indicator, fat=False)."""
    if not isinstance(objective, dm.ConstrainedObjective) or not hasattr(objective, "steepness"):
        raise NotImplementedError(f"output constraint {type(objective).__name__} has no device kernel")
    eta = 1.0 / objective.steepness
    if isinstance(objective, dm.MovingMaximizeSigmoidObjective):
        if x_adapt is None:
            raise ValueError("MovingMaximizeSigmoidObjective needs x_adapt (the observed values)")
        return [(int(idx), -1.0, float(np.asarray(x_adapt).max()) + objective.tp, eta)]
    if isinstance(objective, dm.MaximizeSigmoidObjective):
        return [(int(idx), -1.0, float(objective.tp), eta)]
    if isinstance(objective, dm.MinimizeSigmoidObjective):
        return [(int(idx), 1.0, float(objective.tp), eta)]
    if isinstance(objective, dm.TargetObjective):
        return [(int(idx), -1.0, objective.target_value - objective.tolerance, eta),
                (int(idx), 1.0, objective.target_value + objective.tolerance, eta)]
    raise NotImplementedError(f"output constraint {type(objective).__name__} has no device kernel")


def get_output_constraints(outputs, experiments: pd.DataFrame, output_keys: Sequence[str]):
    """get_output_constraints (bofire/utils/torch_tools.py:340-381): the constraint terms of
    every output with a constrained objective, in output order, each over its model output
    index in ``output_keys``; a moving turning point adapts to that output's valid
    observations.  The etas are the terms' last field."""
    constraints = []
    for feat in outputs.get().features:
        obj = getattr(feat, "objective", None)
        if not isinstance(obj, dm.ConstrainedObjective):
            continue
        x_adapt = None
        if isinstance(obj, dm.MovingMaximizeSigmoidObjective):
            x_adapt = outputs.preprocess_experiments_one_valid_output(feat.key, experiments)[feat.key].values
        constraints += constrained_objective_terms(obj, list(output_keys).index(feat.key), x_adapt)
    return constraints


class _MultiobjectiveMixin:
    """Reference point and objective handling shared by the hypervolume strategies
    (bofire/strategies/predictives/qehvi.py:87-110, mobo.py:92-115)."""

    def get_adjusted_refpoint(self) -> List[float]:
        assert self.experiments is not None, "No experiments available."
        if self.ref_point is None:
            c = getattr(self, "_ref_cache", None)   # inferred once per experiments frame
            if c is not None and c[0] is self._experiments:
                ref_point = c[1]
            else:
                df = self._valid_experiments()
                ref_point = infer_ref_point(self.domain, experiments=df, return_masked=False)
                self._ref_cache = (self._experiments, ref_point)
        else:
            ref_point = self.ref_point
        keys = self.domain.outputs.get_keys_by_objective([MaximizeObjective, MinimizeObjective,
                                                          CloseToTargetObjective])
        return (self.ref_point_mask * np.array([ref_point[k] for k in keys])).tolist()

    def _objective_spec(self):
        """(objectives, constraints) over the model outputs for the device kernels:
        get_multiobjective_objective (bofire/utils/torch_tools.py:699-727; callables :384-402)
        and get_output_constraints (:340-381, constrained_objective2botorch :258-337)."""
        keys = list(self.model.output_keys)
        objectives, constraints = [], []
        for k in self.domain.outputs.get_keys_by_objective([MaximizeObjective, MinimizeObjective,
                                                            CloseToTargetObjective]):
            objectives.append(objective_term(self.domain.outputs.get_by_key(k).objective, keys.index(k)))
        constraints = get_output_constraints(self.domain.outputs, self.experiments, keys)
        return objectives, constraints

    def _objective_affine(self):
        """a, b of g_j = a_j y_j + b_j when every output carries one affine objective (the
        q = 1 fast path); None otherwise (the general kernels take the full description)."""
        objectives, constraints = self._objective_spec()
        if constraints or len(objectives) != len(self.model.output_keys) or any(
                o != j or k != ops.OBJ_AFFINE for j, (o, k, _, _) in enumerate(objectives)):
            return None, None
        return np.array([o[2] for o in objectives]), np.array([o[3] for o in objectives])

    def _observed_outputs(self) -> np.ndarray:
        """Valid observations of every model output (n x m, model output order)."""
        df = self._valid_experiments()
        return df[self.model.output_keys].values.astype(np.float64)

    def _draw_seed(self) -> int:
        return int(torch.randint(0, 1000000, (1,), generator=self.gen).item())


class QehviStrategy(_MultiobjectiveMixin, BotorchStrategy):
    """bofire/strategies/predictives/qehvi.py:24-85 — qEHVI on the device."""

    def __init__(self, data_model, dist=None, **kwargs):
        super().__init__(data_model, dist=dist)
        self.num_sobol_samples = data_model.num_sobol_samples
        self.ref_point = data_model.ref_point
        self.ref_point_mask = get_ref_point_mask(self.domain)
        self.last_acqf = None

    def _get_acqfs(self, n) -> List[QEHVI]:
        """bofire/strategies/predictives/qehvi.py:37-79: the partition is built from the
        masked observations better than the reference point (not objective-transformed).
        Like the reference (qehvi.py:67-75 passes objective and X_pending only), output
        constraints do not enter qEHVI here; QnehviStrategy and MoboStrategy pass them."""
        assert self.experiments is not None, "No experiments available."
        _, X_pending = self.get_acqf_input_tensors()
        objectives, _ = self._objective_spec()
        constraints = ()
        keys = self.domain.outputs.get_keys_by_objective([MaximizeObjective, MinimizeObjective,
                                                          CloseToTargetObjective])
        df = self._valid_experiments()
        train_obj = df[keys].values.astype(np.float64) * self.ref_point_mask
        ref = np.asarray(self.get_adjusted_refpoint(), dtype=np.float64)
        better = (train_obj > ref).all(axis=-1)
        acqf = QEHVI(self.model, train_obj[better], ref, None, None, S=self.num_sobol_samples,
                     sampler_seed=self._draw_seed(), objective=objectives, constraints=constraints,
                     X_pending_raw=X_pending)
        self.last_acqf = acqf
        return [acqf]


class QnehviStrategy(QehviStrategy):
    """bofire/strategies/predictives/qnehvi.py:16-53."""

    def __init__(self, data_model, dist=None, **kwargs):
        super().__init__(data_model, dist=dist)
        self.alpha = data_model.alpha

    def _prefetch_next_ask(self) -> None:
        """The next ask's first generator draws are its prune and sampler seeds (qnehvi.py
        draws them before anything else consumes the strategy's generator), so right after an
        ask they are known: peek at them on a copy of the generator and start the prune draw's
        host scrambling (n_train x m Sobol dimensions) on a worker thread.  The next
        acquisition takes the running future if its (dimension, seed) matches — a tell()
        between the asks changes neither the generator nor, with the same rows, the size —
        and otherwise starts its own; results are the same either way."""
        if os.environ.get("EVR_SCRAMBLE_PREFETCH", "1") == "0" or self.model is None:
            return
        try:
            X_train, _ = self.get_acqf_input_tensors()
        except Exception:   # noqa: BLE001 — a speculative prefetch never fails an ask
            return
        g = torch.Generator()
        g.set_state(self.gen.get_state())
        prune_seed = int(torch.randint(0, 1000000, (1,), generator=g).item())
        prefetch_scramble(int(X_train.shape[0]) * int(self.model.B), prune_seed)

    def _get_acqfs(self, n) -> List[QNEHVI]:
        """bofire/strategies/predictives/qnehvi.py:23-53."""
        assert self.experiments is not None, "No experiments available."
        X_train, X_pending = self.get_acqf_input_tensors()
        # RNG call order of the reference: prune sampler seed, then the acquisition sampler seed;
        # the prune draw's host scrambling (n_baseline x m dimensions) starts right away
        prune_seed = self._draw_seed()
        sampler_seed = self._draw_seed()
        if os.environ.get("EVR_SCRAMBLE_PREFETCH", "1") != "0":
            prefetch_scramble(int(X_train.shape[0]) * int(self.model.B), prune_seed)
        # optimize_acqf's raw-sample seed is the generator's next draw: its Sobol draw runs on a
        # worker thread while the acquisition is built (plain box bounds only; otherwise the
        # optimiser draws as usual)
        if (getattr(self, "_prefetch_raw", False)
                and not get_linear_constraints(self.domain, dm.LinearInequalityConstraint)
                and not get_linear_constraints(self.domain, dm.LinearEqualityConstraint)
                and len(self.get_categorical_combinations()) <= 1):
            prefetch_raw_samples(self._bounds(), self.num_raw_samples, self.gen, q=n)
        objectives, constraints = self._objective_spec()
        ref = self.get_adjusted_refpoint()
        acqf = QNEHVI(self.model, self.model.X_raw, X_train, ref, None, None, S=self.num_sobol_samples,
                      sampler_seed=sampler_seed, prune_baseline=True, prune_seed=prune_seed, X_pending_raw=X_pending,
                      objective=objectives, constraints=constraints, alpha=self.alpha)
        self.last_acqf = acqf
        return [acqf]


class MoboStrategy(_MultiobjectiveMixin, BotorchStrategy):
    """bofire/strategies/predictives/mobo.py:28-115: the acquisition function comes from the
    data model ([upstream] botorch.acquisition.factory.get_acquisition_function) — q(Log)EHVI
    over the FastNondominatedPartitioning of the objective-transformed observations, or
    q(Log)NEHVI with the data model's prune_baseline (qLogNEHVI is the default);
    mc_samples = n_mc_samples."""

    def __init__(self, data_model, dist=None, **kwargs):
        super().__init__(data_model, dist=dist)
        self.ref_point = data_model.ref_point
        self.ref_point_mask = get_ref_point_mask(self.domain)
        self.acquisition_function = data_model.acquisition_function
        self.last_acqf = None

    def _get_acqfs(self, n):
        assert self.is_fitted is True, "Model not trained."
        assert self.experiments is not None, "No experiments available."
        af = self.acquisition_function
        X_train, X_pending = self.get_acqf_input_tensors()
        objectives, constraints = self._objective_spec()
        ref = np.asarray(self.get_adjusted_refpoint(), dtype=np.float64)
        S = int(af.n_mc_samples)
        # mobo.py:83 passes the data model's alpha to get_acquisition_function
        kw = dict(objective=objectives, constraints=constraints, alpha=float(af.alpha))
        if isinstance(af, (dm.qEHVI, dm.qLogEHVI)):
            # [upstream] get_acquisition_function: partition of objective(Y) over the feasible rows
            spec = ops.GeneralSpec(len(self.model.output_keys), objectives, constraints)
            Y = self._observed_outputs()
            feas = np.ones(Y.shape[0], dtype=bool)
            for o, sg, t, _ in constraints:
                feas &= sg * (Y[:, o] - t) <= 0
            cls = QEHVI if isinstance(af, dm.qEHVI) else QLogEHVI
            acqf = cls(self.model, spec.host_objective(Y[feas]), ref, None, None, S=S,
                       sampler_seed=self._draw_seed(), X_pending_raw=X_pending, **kw)
        elif isinstance(af, (dm.qNEHVI, dm.qLogNEHVI)):
            prune_seed = self._draw_seed() if af.prune_baseline else 0
            sampler_seed = self._draw_seed()
            cls = QNEHVI if isinstance(af, dm.qNEHVI) else QLogNEHVI
            acqf = cls(self.model, self.model.X_raw, X_train, ref, None, None, S=S, sampler_seed=sampler_seed,
                       prune_baseline=af.prune_baseline, prune_seed=prune_seed, X_pending_raw=X_pending, **kw)
        else:
            raise NotImplementedError(f"{type(af).__name__} has no device kernel in this build")
        self.last_acqf = acqf
        return [acqf]


class SoboStrategy(BotorchStrategy):
    """bofire/strategies/predictives/sobo.py:40-120 — qEI on the device."""

    def __init__(self, data_model, dist=None, **kwargs):
        super().__init__(data_model, dist=dist)
        self.acquisition_function = data_model.acquisition_function
        self.last_acqf = None

    def _get_acqfs(self, n):
        if not isinstance(self.acquisition_function, dm.qEI):
            raise NotImplementedError(f"{type(self.acquisition_function).__name__} is out of scope; use qEI()")
        target = self.domain.outputs.get_by_objective([MaximizeObjective, MinimizeObjective]).features[0]
        if self.model.output_keys.index(target.key) != 0 or len(self.model.output_keys) != 1:
            raise NotImplementedError("single-output SOBO only")
        a, b = target.objective.affine()
        X_train, X_pending = self.get_acqf_input_tensors()
        seed = int(torch.randint(0, 1000000, (1,), generator=self.gen).item())
        S = int(self.acquisition_function.n_mc_samples)
        if X_pending is None and n == 1:
            acqf = QEI(self.model, X_train, a, b, S=S, seed=seed)
        else:
            # joint batches (q > 1) and pending points (sobo.py:72 passes X_pending)
            acqf = QEIJoint(self.model, X_train, a, b, S=S, seed=seed, X_pending_raw=X_pending)
        self.last_acqf = acqf
        return [acqf]


STRATEGY_MAP = {
    dm.QnehviStrategy: QnehviStrategy,
    dm.QehviStrategy: QehviStrategy,
    dm.MoboStrategy: MoboStrategy,
    dm.SoboStrategy: SoboStrategy,
    dm.RandomStrategy: RandomStrategy,
}


def map(data_model, **kwargs):
    """bofire/strategies/mapper.py:7-14."""
    cls = STRATEGY_MAP.get(type(data_model))
    if cls is None:
        raise NotImplementedError(f"{type(data_model).__name__} is out of scope for the MI355X build")
    return cls(data_model, **kwargs) if cls is not RandomStrategy else cls(data_model)
