"""Functional surrogates on the device — mirrors bofire/surrogates/{single_task_gp,botorch,
surrogate,trainable,botorch_surrogates}.py for ``SingleTaskGPSurrogate``.

The fitted model (transformed training inputs, targets, hyperparameters, Normalize bounds,
kernel family) is the wire format of ``dumps()/loads()`` — a versioned JSON + base64(npz)
blob instead of the reference's base64 BoTorch pickle (bofire/surrogates/botorch.py:66-77),
which cannot be produced without BoTorch.
"""
from __future__ import annotations

import base64
import io
import json
import math
from typing import Dict, List, Optional, Tuple

import numpy as np
import pandas as pd
import torch

from . import data_models as dm
from .data_models.models import (CategoricalEncodingEnum, DimensionalityScaledLogNormalPrior, GammaPrior,
                                  LogNormalPrior, MaternKernel, NormalPrior, RBFKernel, ScalerEnum)
from .gp import GPBatch, GPHyper, fit_single, standardize_params

KIND_BY_NU = {0.5: 1, 1.5: 2, 2.5: 3}


def device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("everest_amd surrogates run on the MI355X only (no HIP device visible)")
    return torch.device("cuda", torch.cuda.current_device())


def kernel_kind(kernel) -> int:
    """bofire/kernels/mapper.py:31-69."""
    if isinstance(kernel, RBFKernel):
        return 0
    if isinstance(kernel, MaternKernel):
        return KIND_BY_NU[kernel.nu]
    raise NotImplementedError(f"kernel {type(kernel).__name__} is out of scope for the MI355X build")


def map_prior(prior, d: int) -> Optional[Tuple[str, float, float]]:
    """bofire/priors/mapper.py:9-63 -> (family, p1, p2)."""
    if prior is None:
        return None
    if isinstance(prior, DimensionalityScaledLogNormalPrior):
        return ("lognormal", prior.loc + math.log(d) * prior.loc_scaling,
                (prior.scale ** 2 + math.log(d) * prior.scale_scaling) ** 0.5)
    if isinstance(prior, LogNormalPrior):
        return ("lognormal", float(prior.loc), float(prior.scale))
    if isinstance(prior, GammaPrior):
        return ("gamma", float(prior.concentration), float(prior.rate))
    if isinstance(prior, NormalPrior):
        return ("normal", float(prior.loc), float(prior.scale))
    raise NotImplementedError(type(prior).__name__)


class SingleTaskGPSurrogate:
    """Exact GP surrogate for one output (bofire/surrogates/single_task_gp.py:23-71)."""

    def __init__(self, data_model: dm.SingleTaskGPSurrogate):
        self.data_model = data_model
        self.inputs = data_model.inputs
        self.outputs = data_model.outputs
        self.kernel = data_model.kernel
        self.noise_prior = data_model.noise_prior
        self.scaler = data_model.scaler
        self.output_scaler = data_model.output_scaler
        self.input_preprocessing_specs = {k: v.value if hasattr(v, "value") else v
                                          for k, v in data_model.input_preprocessing_specs.items()}
        self.state: Optional[dict] = None
        self.gp: Optional[GPBatch] = None
        if data_model.dump is not None:
            self.loads(data_model.dump)

    @property
    def is_fitted(self) -> bool:
        return self.state is not None

    @property
    def output_key(self) -> str:
        return self.outputs.get_keys()[0]

    # ---- transforms ----------------------------------------------------------------
    def _bounds(self, X: pd.DataFrame) -> Tuple[np.ndarray, np.ndarray]:
        """Normalize bounds on the continuous columns (get_scaler, bofire/surrogates/utils.py:103-164);
        one-hot columns keep [0, 1] (identity)."""
        f2i, _ = self.inputs._transform_info(self.input_preprocessing_specs)
        d = sum(len(v) for v in f2i.values())
        lo, hi = np.zeros(d), np.ones(d)
        if self.scaler == ScalerEnum.NORMALIZE:
            for feat in self.inputs.get(dm.ContinuousInput).features:
                (l,), (u,) = feat.get_bounds(values=X[feat.key])
                j = f2i[feat.key][0]
                lo[j], hi[j] = l, (u if u > l else l + 1.0)
        elif self.scaler != ScalerEnum.IDENTITY:
            raise NotImplementedError("InputStandardize is out of scope for the MI355X build")
        return lo, hi

    def transform_inputs(self, X: pd.DataFrame) -> np.ndarray:
        return self.inputs.transform(X, self.input_preprocessing_specs).values.astype(np.float64)

    # ---- fit -------------------------------------------------------------------------
    def fit(self, experiments: pd.DataFrame, options: Optional[dict] = None):
        """TrainableSurrogate.fit (bofire/surrogates/trainable.py:24-42): valid rows of this output."""
        X, Y = self._fit_data(experiments)
        self._fit(X, Y, options)

    def _fit_data(self, experiments: pd.DataFrame):
        key = self.output_key
        df = experiments
        if f"valid_{key}" in df:
            df = df[df[f"valid_{key}"] > 0]
        df = df.dropna(subset=[key])
        return df[self.inputs.get_keys()], df[[key]]

    def _fit_problem(self, X: pd.DataFrame, Y: pd.DataFrame) -> dict:
        """Everything the MLL fit needs: transformed inputs, bounds, targets, kernel, priors."""
        Xt = self.transform_inputs(X)
        lo, hi = self._bounds(X)
        return dict(Xt=Xt, lo=lo, hi=hi, y=Y.values[:, 0].astype(np.float64), kind=kernel_kind(self.kernel),
                    ls_prior=map_prior(getattr(self.kernel, "lengthscale_prior", None), Xt.shape[1]),
                    noise_prior=map_prior(self.noise_prior, 1),
                    standardize=self.output_scaler == ScalerEnum.STANDARDIZE)

    def _fit(self, X: pd.DataFrame, Y: pd.DataFrame, options: Optional[dict] = None):
        pb = self._fit_problem(X, Y)
        Xn = torch.as_tensor((pb["Xt"] - pb["lo"]) / (pb["hi"] - pb["lo"]), dtype=torch.float64, device=device())
        hyp = fit_single(Xn, pb["y"], pb["kind"], pb["ls_prior"], pb["noise_prior"], standardize=pb["standardize"],
                         options=options)
        self._set_state(pb["Xt"], pb["y"], pb["lo"], pb["hi"], pb["kind"], hyp)

    def _set_state(self, Xt, y, lo, hi, kind, hyp: GPHyper):
        self.state = dict(X=np.asarray(Xt), y=np.asarray(y), lo=np.asarray(lo), hi=np.asarray(hi), kind=int(kind),
                          lengthscale=np.asarray(hyp.lengthscale), noise=float(hyp.noise),
                          constant=float(hyp.constant), y_mean=float(hyp.y_mean), y_std=float(hyp.y_std))
        self.gp = self._build_gp()

    def hyper(self) -> GPHyper:
        s = self.state
        return GPHyper(lengthscale=s["lengthscale"], noise=s["noise"], constant=s["constant"], y_mean=s["y_mean"],
                       y_std=s["y_std"])

    def _build_gp(self) -> GPBatch:
        s = self.state
        dev = device()
        t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=dev)  # noqa: E731
        Xn = t((s["X"] - s["lo"]) / (s["hi"] - s["lo"]))
        return GPBatch(Xn, t(s["y"][:, None]), [self.hyper()], s["kind"], t(s["lo"]), t(s["hi"]))

    # ---- predict ----------------------------------------------------------------------
    def predict(self, experiments: pd.DataFrame) -> pd.DataFrame:
        """Surrogate.predict (bofire/surrogates/surrogate.py:39-67): posterior(observation_noise=True)."""
        if not self.is_fitted:
            raise ValueError("Model is not fitted/available yet.")
        Xt = self.transform_inputs(experiments[self.inputs.get_keys()])
        mean, var = self.gp.posterior(torch.as_tensor(Xt, dtype=torch.float64, device=self.gp.device),
                                      observation_noise=True)
        key = self.output_key
        return pd.DataFrame({f"{key}_pred": mean[0].cpu().numpy(), f"{key}_sd": np.sqrt(var[0].cpu().numpy())},
                            index=experiments.index)

    # ---- dump / load ------------------------------------------------------------------
    def dumps(self) -> str:
        if not self.is_fitted:
            raise ValueError("Model is not fitted/available yet.")
        buf = io.BytesIO()
        s = self.state
        np.savez(buf, X=s["X"], y=s["y"], lo=s["lo"], hi=s["hi"], lengthscale=s["lengthscale"])
        meta = {"format": "everest_amd.SingleTaskGP/1", "kind": s["kind"], "noise": s["noise"],
                "constant": s["constant"], "y_mean": s["y_mean"], "y_std": s["y_std"],
                "arrays": base64.b64encode(buf.getvalue()).decode()}
        return base64.b64encode(json.dumps(meta).encode()).decode()

    def loads(self, data: str):
        meta = json.loads(base64.b64decode(data.encode()).decode())
        if meta.get("format") != "everest_amd.SingleTaskGP/1":
            raise ValueError("unknown surrogate dump format (BoTorch pickles cannot be loaded without BoTorch)")
        arr = np.load(io.BytesIO(base64.b64decode(meta["arrays"])), allow_pickle=False)
        hyp = GPHyper(lengthscale=arr["lengthscale"], noise=meta["noise"], constant=meta["constant"],
                      y_mean=meta["y_mean"], y_std=meta["y_std"])
        self._set_state(arr["X"], arr["y"], arr["lo"], arr["hi"], meta["kind"], hyp)


class BotorchSurrogates:
    """bofire/surrogates/botorch_surrogates.py:19-128."""

    def __init__(self, data_model: dm.BotorchSurrogates):
        self.surrogates = [SingleTaskGPSurrogate(s) for s in data_model.surrogates]

    def fit(self, experiments: pd.DataFrame):
        """Fits the per-output GPs (independent problems, as in the reference's sequential
        loop, bofire/surrogates/botorch_surrogates.py).  Outputs observed on the same rows with
        the same kernel, priors and scalers (the usual case) are fitted in lock-step by
        gp.fit_batch: one L-BFGS-B per output, one batched MLL launch chain per round.  Others
        run concurrently, one host thread and one HIP stream per output (EVR_FIT_THREADS=1:
        sequentially); EVR_FIT_BATCH=0 disables the lock-step fit."""
        import os
        from concurrent.futures import ThreadPoolExecutor

        from .gp import fit_batch

        rest = list(self.surrogates)
        if os.environ.get("EVR_FIT_BATCH", "1") != "0" and len(rest) > 1 and torch.cuda.is_available():
            probs = [(s, s._fit_problem(*s._fit_data(experiments))) for s in rest]
            groups = {}
            for s, pb in probs:
                key = (pb["Xt"].shape, pb["Xt"].tobytes(), pb["lo"].tobytes(), pb["hi"].tobytes(), pb["kind"],
                       pb["ls_prior"], pb["noise_prior"], pb["standardize"])
                groups.setdefault(key, []).append((s, pb))
            rest = []
            for members in groups.values():
                if len(members) == 1:
                    rest.append(members[0][0])
                    continue
                pb0 = members[0][1]
                Xn = torch.as_tensor((pb0["Xt"] - pb0["lo"]) / (pb0["hi"] - pb0["lo"]), dtype=torch.float64,
                                     device=device())
                hyps = fit_batch(Xn, np.stack([pb["y"] for _, pb in members], 1), pb0["kind"], pb0["ls_prior"],
                                 pb0["noise_prior"], standardize=pb0["standardize"])
                for (s, pb), h in zip(members, hyps):
                    s._set_state(pb["Xt"], pb["y"], pb["lo"], pb["hi"], pb["kind"], h)
            if not rest:
                return

        workers = int(os.environ.get("EVR_FIT_THREADS", "0") or 0) or len(rest)
        if workers <= 1 or len(rest) <= 1 or not torch.cuda.is_available():
            for s in rest:
                s.fit(experiments)
            return
        dev = device()

        def run(s):
            stream = torch.cuda.Stream(device=dev)
            with torch.cuda.stream(stream):
                s.fit(experiments)
            stream.synchronize()

        with ThreadPoolExecutor(max_workers=min(workers, len(rest))) as ex:
            for f in [ex.submit(run, s) for s in rest]:
                f.result()

    def compatibilize(self, inputs, outputs) -> GPBatch:
        """One batched device model over the outputs in domain order — the ModelListGP of
        bofire/surrogates/botorch_surrogates.py:79-128.  Outputs may be fitted on different
        rows (each surrogate trains on the rows where its output is valid,
        bofire/surrogates/trainable.py:44-66) and with different kernel families: the batch
        holds the union of the training rows with a per-output row mask and a per-output
        family (gp.GPBatch), and each output's Normalize bounds are folded into its
        lengthscales (the stationary kernels see (x - x') / ((hi - lo) ls) only), so every
        member is exactly its own GP."""
        by_key = {s.output_key: s for s in self.surrogates}
        order = [k for k in outputs.get_keys() if k in by_key]
        ss = [by_key[k] for k in order]
        for k, s in zip(order, ss):
            if not s.is_fitted:
                raise ValueError(f"Surrogate for output feature {k} not fitted.")
        d = ss[0].state["X"].shape[1]
        if any(s.state["X"].shape[1] != d for s in ss):
            raise NotImplementedError("surrogates over different input subsets are out of scope for the MI355X build")
        X_all, rows = union_rows([s.state["X"] for s in ss])
        n, B = X_all.shape[0], len(ss)
        mask = np.zeros((B, n), dtype=bool)
        Y = np.zeros((n, B))
        for j, (s, r) in enumerate(zip(ss, rows)):
            mask[j, r] = True
            Y[r, j] = s.state["y"]
        s0 = ss[0].state
        lo, hi = np.asarray(s0["lo"], dtype=np.float64), np.asarray(s0["hi"], dtype=np.float64)
        hypers = []
        for s in ss:
            h = s.hyper()
            st = s.state
            if not (np.array_equal(st["lo"], lo) and np.array_equal(st["hi"], hi)):
                h.lengthscale = np.asarray(h.lengthscale) * ((st["hi"] - st["lo"]) / (hi - lo))
            hypers.append(h)
        dev = device()
        t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=dev)  # noqa: E731
        gp = GPBatch(t((X_all - lo) / (hi - lo)), t(Y), hypers, [s.state["kind"] for s in ss], t(lo), t(hi),
                     mask=mask)
        gp.output_keys = order
        gp.X_raw = X_all
        gp.rows = rows
        return gp


def union_rows(Xs):
    """Union of the training-row multisets of several outputs, first output's rows first in
    their order, then each later output's rows that no earlier row of equal value (unused by
    that output) covers.  Returns (X_union, [row indices of output j's rows])."""
    out, index, per = [], {}, []
    for X in Xs:
        X = np.asarray(X, dtype=np.float64)
        used = {}
        ids = np.empty(X.shape[0], dtype=np.int64)
        for i, row in enumerate(X):
            key = row.tobytes()
            lst = index.setdefault(key, [])
            k = used.get(key, 0)
            if k == len(lst):
                lst.append(len(out))
                out.append(row)
            ids[i] = lst[k]
            used[key] = k + 1
        per.append(ids)
    return np.asarray(out, dtype=np.float64).reshape(-1, Xs[0].shape[1]), per


def map(data_model):
    """bofire/surrogates/mapper.py:21-44 (SingleTaskGPSurrogate only)."""
    if isinstance(data_model, dm.SingleTaskGPSurrogate):
        return SingleTaskGPSurrogate(data_model)
    if isinstance(data_model, dm.BotorchSurrogates):
        return BotorchSurrogates(data_model)
    raise NotImplementedError(f"{type(data_model).__name__} is out of scope for the MI355X build")
