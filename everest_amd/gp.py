"""Exact GPs resident in HBM: batched posterior and MLL (value + gradient) on the HIP kernels.

Mirrors BoFire's ``SingleTaskGPSurrogate`` model (bofire/surrogates/single_task_gp.py:39-71)
on top of [upstream] BoTorch ``SingleTaskGP``: Normalize(bounds) inputs, Standardize outputs,
ConstantMean, RBF/Matérn ARD kernel (no outputscale by default), Gaussian likelihood with
noise >= 1e-4 and hyperpriors; fit = scipy L-BFGS-B on the raw parameters
(``fit_gpytorch_mll``, max_attempts=10), every loss/gradient evaluated on the device.

``GPBatch`` holds B exact GPs over one set of normalized training rows (the ModelListGP of
BotorchSurrogates.compatibilize, bofire/surrogates/botorch_surrogates.py:79-128) so that
posteriors for all outputs are one batched launch.  The members may differ in kernel family
(one per output, EVR_KERNEL_MIXED) and in training rows: with a row mask, output j's GP is
exact over its own rows V_j only — K_j is padded to the union with identity rows / columns
outside V_j, so chol(K_pad) is L_j interleaved with identity rows, and L^-1's rows outside V_j
(and with them alpha's entries) are zeroed: L^-T L^-1 = K_j^-1 embedded, and every posterior,
root and projection formula runs unchanged over the union rows.
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _native, ops

MIN_INFERRED_NOISE_LEVEL = 1e-4
KIND_MIXED, KIND_MAX_MIXED = 16, 13     # include/everest_amd.h EVR_KERNEL_MIXED


def kind_code(kinds: Sequence[int]) -> int:
    """Kernel family code of a batch of outputs: the family itself when all agree, else
    EVR_KERNEL_MIXED with 2 bits per output (kind_j << (5 + 2 j))."""
    kinds = [int(k) for k in kinds]
    if any(k < 0 or k > 3 for k in kinds):
        raise ValueError(f"kernel kinds must be in 0..3, got {kinds}")
    if len(set(kinds)) <= 1:
        return kinds[0] if kinds else 0
    if len(kinds) > KIND_MAX_MIXED:
        raise NotImplementedError(f"mixed kernel families are supported for at most {KIND_MAX_MIXED} outputs")
    code = KIND_MIXED
    for j, k in enumerate(kinds):
        code |= k << (5 + 2 * j)
    return code


def kinds_of(code: int, B: int) -> List[int]:
    code = int(code)
    return [code] * B if code < KIND_MIXED else [(code >> (5 + 2 * j)) & 3 for j in range(B)]


def softplus_np(x):
    return np.logaddexp(0.0, x)


def _softplus_libm(v: float) -> float:
    """numpy.logaddexp(0, v) with the C library's scalar exp / log1p (CPython's math module):
    the arithmetic of the native fit driver's softplus (mll_plan.hip)."""
    v = float(v)
    if v == 0.0:
        return 0.6931471805599453
    return v + math.log1p(math.exp(-v)) if v > 0.0 else math.log1p(math.exp(v))


def sigmoid_np(x):
    return 1.0 / (1.0 + np.exp(-x))


def _prior(p):
    """Normalise a prior spec: None, (loc, scale) [LogNormal] or (family, p1, p2)."""
    if p is None:
        return None
    if len(p) == 2:
        return ("lognormal", float(p[0]), float(p[1]))
    return (p[0], float(p[1]), float(p[2]))


def prior_logpdf_np(p, x):
    """gpytorch LogNormalPrior / GammaPrior / NormalPrior log densities (elementwise)."""
    fam, a, b = p
    x = np.asarray(x, dtype=np.float64)
    if fam == "lognormal":
        lx = np.log(x)
        return -lx - math.log(b) - 0.5 * math.log(2 * math.pi) - 0.5 * ((lx - a) / b) ** 2
    if fam == "gamma":
        return a * math.log(b) - math.lgamma(a) + (a - 1) * np.log(x) - b * x
    if fam == "normal":
        return -0.5 * math.log(2 * math.pi * b * b) - 0.5 * ((x - a) / b) ** 2
    raise ValueError(fam)


def prior_dlogpdf_np(p, x):
    fam, a, b = p
    x = np.asarray(x, dtype=np.float64)
    if fam == "lognormal":
        return (-1.0 - (np.log(x) - a) / b ** 2) / x
    if fam == "gamma":
        return (a - 1) / x - b
    if fam == "normal":
        return -(x - a) / (b * b)
    raise ValueError(fam)


def prior_sample_np(p, rng, size):
    fam, a, b = p
    if fam == "lognormal":
        return np.exp(rng.normal(a, b, size))
    if fam == "gamma":
        return rng.gamma(a, 1.0 / b, size)
    if fam == "normal":
        return np.abs(rng.normal(a, b, size))
    raise ValueError(fam)


def standardize_params(y: np.ndarray) -> Tuple[float, float]:
    """[upstream] Standardize(m=1): mean, unbiased std, std < 1e-8 -> 1, n == 1 -> 1."""
    mean = float(np.mean(y))
    if y.shape[0] == 1:
        return mean, 1.0
    std = float(np.std(y, ddof=1))
    return mean, (std if std >= 1e-8 else 1.0)


@dataclass
class GPHyper:
    lengthscale: np.ndarray   # d
    noise: float
    constant: float
    y_mean: float
    y_std: float


class GPBatch:
    """B exact GPs on shared normalized inputs Xn (n x d, device).  ``kind``: one family, a
    per-output list, or a kind code; ``mask`` (B x n, optional): the rows each output is
    trained on (Y's entries outside them are ignored)."""

    def __init__(self, Xn: torch.Tensor, Y: torch.Tensor, hypers: Sequence[GPHyper], kind,
                 lo: torch.Tensor, hi: torch.Tensor, mask: Optional[np.ndarray] = None):
        self.Xn = Xn.contiguous()
        B_ = len(hypers)
        if isinstance(kind, (list, tuple, np.ndarray)):
            if len(kind) != B_:
                raise ValueError(f"{len(kind)} kernel kinds for {B_} outputs")
            kind = kind_code(kind)
        self.kind = int(kind)
        self.kinds = kinds_of(self.kind, B_)
        self.lo = lo
        self.hi = hi
        self.inv_range = 1.0 / (hi - lo)
        self.hypers = list(hypers)
        dev = Xn.device
        self.device = dev
        self.B = len(hypers)
        self.n, self.d = Xn.shape
        t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=dev)  # noqa: E731
        self.ls = t(np.stack([h.lengthscale for h in hypers]))
        self.noise = t([h.noise for h in hypers])
        self.const = t([h.constant for h in hypers])
        self.ym = t([h.y_mean for h in hypers])
        self.ys = t([h.y_std for h in hypers])
        self.kxx = torch.ones(self.B, dtype=torch.float64, device=dev)
        self.mask = None
        if mask is not None:
            mk = np.asarray(mask, dtype=bool).reshape(self.B, self.n)
            if not mk.any(axis=1).all():
                raise ValueError("every output needs at least one training row")
            if not mk.all():
                self.mask = torch.as_tensor(mk.astype(np.float64), device=dev)
        # standardized targets (B x n); zero (the prior mean's residual is masked) outside each
        # output's own rows
        Yc = Y.to(device=dev, dtype=torch.float64).reshape(self.n, self.B).T.contiguous()
        self.y = ((Yc - self.ym[:, None]) / self.ys[:, None]).contiguous()
        if self.mask is not None:
            self.y = torch.where(self.mask > 0, self.y, torch.zeros_like(self.y)).contiguous()
        self.refresh()

    def valid_all_rows(self) -> np.ndarray:
        """Rows every output is trained on (n bools)."""
        if self.mask is None:
            return np.ones(self.n, dtype=bool)
        return (self.mask.min(0).values > 0).cpu().numpy()

    # -- caches: L = chol(K + s2 I), Linv, alpha, M = [Linv; alpha^T] ----------------------
    def refresh(self):
        Ky = ops.kernel_matrix(self.Xn, self.Xn, self.ls, self.kind, diag_add=self.noise)
        if self.mask is not None:
            # K_j padded: identity rows / columns outside output j's rows
            mk = self.mask
            Ky.mul_(mk[:, :, None] * mk[:, None, :])
            Ky.diagonal(dim1=-2, dim2=-1).add_(1.0 - mk)
        self.L, self.Linv, _, _ = ops.cholesky_inverse(Ky, 1e-8, 3)
        if self.mask is not None:
            self.Linv.mul_(self.mask[:, :, None])                               # K_j^-1 embedded
        r = (self.y - self.const[:, None]).unsqueeze(-1)                        # B x n x 1
        if self.mask is not None:
            r = r * self.mask[:, :, None]
        r = r.contiguous()
        v = ops.gemm(self.Linv, r)
        self.alpha = ops.gemm(self.Linv, v, transA=True)[..., 0].contiguous()  # B x n
        self.M = torch.cat([self.Linv, self.alpha.unsqueeze(1)], dim=1).contiguous()  # B x (n+1) x n

    def kernel_train(self, noise: bool = False) -> torch.Tensor:
        return ops.kernel_matrix(self.Xn, self.Xn, self.ls, self.kind, diag_add=self.noise if noise else None)

    def cross(self, Xraw: torch.Tensor) -> torch.Tensor:
        """K(Xtr, normalize(Xraw)) : B x n x nt."""
        return ops.kernel_matrix(self.Xn, Xraw, self.ls, self.kind, shift2=self.lo, scale2=self.inv_range)

    def posterior(self, Xraw: torch.Tensor, observation_noise: bool = False):
        """Mean and variance (B x nt) at raw (transformed, unnormalized) inputs."""
        from . import torch_ops

        Xraw = Xraw.to(device=self.device, dtype=torch.float64).contiguous()
        # the registered operator torch.ops.everest_amd.gp_posterior (evr_gp_posterior)
        return torch_ops.load().gp_posterior(self.Xn, Xraw, self.lo, self.inv_range, self.ls, self.M, self.kind,
                                             self.const, self.ym, self.ys, self.kxx,
                                             self.noise if observation_noise else None)


# ---------------------------------------------------------------------------------------
# device MLL value + gradient (one output)
# ---------------------------------------------------------------------------------------
class MLLEvaluator:
    """Exact MLL / n with hyperpriors for one GP on device; raw parameter vector
    x = [noise, constant, raw_lengthscale(d)] (BoTorch bounds: noise >= 1e-4)."""

    def __init__(self, Xn: torch.Tensor, y_std_space: np.ndarray, kind: int,
                 ls_prior: Optional[Tuple[float, float]], noise_prior: Optional[Tuple[float, float]]):
        self.Xn = Xn.contiguous()
        self.n, self.d = Xn.shape
        self.kind = kind
        self.y = np.asarray(y_std_space, dtype=np.float64)
        self.ls_prior = _prior(ls_prior)
        self.noise_prior = _prior(noise_prior)
        self.dev = Xn.device

    def __call__(self, x: np.ndarray):
        n, d = self.n, self.d
        noise, const, raw = float(x[0]), float(x[1]), np.asarray(x[2:], dtype=np.float64)
        ls = softplus_np(raw)
        dev = self.dev
        ls_t = torch.as_tensor(ls[None, :], device=dev)
        Ky = ops.kernel_matrix(self.Xn, self.Xn, ls_t, self.kind,
                               diag_add=torch.tensor([noise], dtype=torch.float64, device=dev))
        L, Linv, _, _ = ops.cholesky_inverse(Ky, 1e-8, 3)
        r = torch.as_tensor((self.y - const)[None, :, None], device=dev)
        v = ops.gemm(Linv, r)
        alpha = ops.gemm(Linv, v, transA=True)                       # 1 x n x 1
        W = ops.gemm(alpha, alpha, transB=True)                      # alpha alpha^T
        ops.gemm(Linv, Linv, transA=True, alpha=-1.0, beta=1.0, out=W)   # - K^-1
        gls = ops.kernel_lengthscale_grad(self.Xn, ls_t, W, self.kind)  # 1 x d
        terms = ops.mll_terms(L, Linv, r[..., 0].contiguous(), alpha[..., 0].contiguous())
        terms = terms.cpu().numpy()[0]
        gls = gls.cpu().numpy()[0]
        logdet, quad, trKinv, sum_a, sum_a2 = terms
        ll = -0.5 * quad - 0.5 * logdet - 0.5 * n * math.log(2 * math.pi)
        d_noise = 0.5 * (sum_a2 - trKinv)
        d_const = sum_a
        d_ls = 0.5 * gls
        if self.ls_prior is not None:
            ll += float(np.sum(prior_logpdf_np(self.ls_prior, ls)))
            d_ls = d_ls + prior_dlogpdf_np(self.ls_prior, ls)
        if self.noise_prior is not None:
            ll += float(prior_logpdf_np(self.noise_prior, noise))
            d_noise += float(prior_dlogpdf_np(self.noise_prior, noise))
        d_raw = d_ls * sigmoid_np(raw)
        g = np.concatenate([[d_noise, d_const], d_raw]) / n
        return ll / n, g


def fit_single(Xn: torch.Tensor, y_raw: np.ndarray, kind: int, ls_prior, noise_prior=(-4.0, 1.0),
               max_attempts: int = 10, seed: int = 0, options: Optional[dict] = None,
               standardize: bool = True) -> GPHyper:
    """fit_gpytorch_mll restated on device kernels: minimise -mll with scipy L-BFGS-B over
    (noise >= 1e-4, constant, raw lengthscale) starting from noise = prior mode (LogNormal
    noise prior: exp(loc - scale^2)), constant 0, lengthscale softplus(0) = ln 2; on
    NotPSDError resample the hyperparameters from their priors and retry (max_attempts=10,
    bofire/surrogates/single_task_gp.py:71)."""
    from scipy.optimize import minimize

    if standardize:
        y_mean, y_std = standardize_params(y_raw)
    else:
        y_mean, y_std = 0.0, 1.0
    y = (y_raw - y_mean) / y_std
    d = Xn.shape[1]
    lsp, nzp = _prior(ls_prior), _prior(noise_prior)
    ev = MLLEvaluator(Xn, y, kind, lsp, nzp)
    if nzp is not None and nzp[0] == "lognormal":
        noise0 = math.exp(nzp[1] - nzp[2] ** 2)
    elif nzp is not None and nzp[0] == "gamma" and nzp[1] > 1:
        noise0 = (nzp[1] - 1) / nzp[2]
    else:
        noise0 = 2 * MIN_INFERRED_NOISE_LEVEL
    noise0 = max(noise0, MIN_INFERRED_NOISE_LEVEL)
    x0 = np.concatenate([[noise0, 0.0], np.zeros(d)])
    bounds = [(MIN_INFERRED_NOISE_LEVEL, None), (None, None)] + [(None, None)] * d
    rng = np.random.default_rng(seed)
    last_err = None
    for attempt in range(max_attempts):
        try:
            res = minimize(lambda x: tuple(-v for v in ev(x)), x0, jac=True, method="L-BFGS-B", bounds=bounds,
                           options=options or {})
            xv = res.x
            return GPHyper(lengthscale=softplus_np(xv[2:]), noise=float(xv[0]), constant=float(xv[1]),
                           y_mean=y_mean, y_std=y_std)
        except ops.NotPSDError as e:  # sample_all_priors, then retry
            last_err = e
            ls = prior_sample_np(lsp, rng, d) if lsp else np.full(d, math.log(2.0))
            nz = max(float(prior_sample_np(nzp, rng, 1)[0]) if nzp else 1e-3, MIN_INFERRED_NOISE_LEVEL)
            x0 = np.concatenate([[nz, 0.0], np.log(np.expm1(ls))])
    raise RuntimeError(f"GP fit failed after {max_attempts} attempts: {last_err}")


# ---------------------------------------------------------------------------------------
# lock-step fit of several outputs on shared inputs: one batched MLL launch chain per round
# ---------------------------------------------------------------------------------------
class MLLBatch:
    """MLL / n (+ hyperpriors) value and gradient of B GPs sharing Xn (one per output),
    evaluated for any subset of the outputs in one batched launch chain (kernel matrices,
    psd_safe Cholesky + inverse, alpha, W = alpha alpha^T - K^-1, lengthscale gradients, the
    scalar terms) and one device->host copy.  Returns None for a member whose Cholesky stays
    not p.d. after the jitter ladder (NotPSDError of that fit)."""

    def __init__(self, Xn: torch.Tensor, Ys: np.ndarray, kind: int, ls_prior, noise_prior):
        self.Xn = Xn.contiguous()
        self.n, self.d = Xn.shape
        self.kind = kind
        self.Y = torch.as_tensor(np.asarray(Ys, dtype=np.float64), device=Xn.device)   # B x n (standardized)
        self.ls_prior = _prior(ls_prior)
        self.noise_prior = _prior(noise_prior)
        self.use_plan = os.environ.get("EVR_MLL_PLAN", "1") != "0"
        self._plan = None

    def _eval_ops(self, idx, ls, noise, const):
        """The op-by-op chain with the psd_safe_cholesky jitter ladder (host arrays)."""
        dev = self.Xn.device
        ls_t = torch.as_tensor(ls, device=dev)
        Ky = ops.kernel_matrix(self.Xn, self.Xn, ls_t, self.kind, diag_add=torch.as_tensor(noise, device=dev))
        L, Linv, _, info = ops.cholesky_inverse(Ky, 1e-8, 3, raise_on_fail=False)
        it = torch.as_tensor(np.asarray(idx, dtype=np.int64), device=dev)
        r = (self.Y[it] - torch.as_tensor(const, device=dev)[:, None]).unsqueeze(-1).contiguous()   # B x n x 1
        v = ops.gemm(Linv, r)
        alpha = ops.gemm(Linv, v, transA=True)
        W = ops.gemm(alpha, alpha, transB=True)
        ops.gemm(Linv, Linv, transA=True, alpha=-1.0, beta=1.0, out=W)
        gls = ops.kernel_lengthscale_grad(self.Xn, ls_t, W, self.kind)
        terms = ops.mll_terms(L, Linv, r[..., 0].contiguous(), alpha[..., 0].contiguous())
        return torch.cat([terms.reshape(-1), gls.reshape(-1), info.to(torch.float64)]).cpu().numpy()

    def plan_handle(self):
        """The native MLL plan (evr_mll_plan_create), built on first use."""
        if self._plan is None:
            Bt, d = self.Y.shape[0], self.d
            h = ctypes.c_void_p()
            ops.call("evr_mll_plan_create", ops._stream(), int(self.kind), Bt, self.n, d, self.Xn.data_ptr(),
                     self.Y.data_ptr(), ctypes.byref(h))
            self._plan = h
            self._lib = _native.load()
            self._params = None
            self._pout = np.empty(Bt * (5 + d + 1))
        return self._plan

    def prior_spec(self) -> np.ndarray:
        """[ls family, a, b, noise family, a, b] for evr_mll_fit_rounds (family 0 none,
        1 LogNormal, 2 Gamma, 3 Normal)."""
        fam = {"lognormal": 1, "gamma": 2, "normal": 3}
        out = np.zeros(6)
        for k, p in enumerate((self.ls_prior, self.noise_prior)):
            if p is not None:
                out[3 * k:3 * k + 3] = (fam[p[0]], p[1], p[2])
        return out

    def _eval_plan(self, idx, ls, noise, const):
        """All members through the native MLL plan (evr_mll_plan_eval: one graph launch);
        members outside idx keep their last parameters.  None when an active member's
        attempt-0 factor fails (the caller takes the ladder path)."""
        Bt, d = self.Y.shape[0], self.d
        self.plan_handle()
        if self._params is None:
            self._params = np.empty((Bt, d + 2))
            self._params[:, :d] = ls[0]
            self._params[:, d] = noise[0]
            self._params[:, d + 1] = const[0]
        P = self._params
        for k, b in enumerate(idx):
            P[b, :d], P[b, d], P[b, d + 1] = ls[k], noise[k], const[k]
        flat = np.concatenate([P[:, :d].reshape(-1), P[:, d], P[:, d + 1]])
        _native.check(self._lib.evr_mll_plan_eval(ops._stream(), self._plan, flat.ctypes.data, self._pout.ctypes.data),
                      "evr_mll_plan_eval")
        o = self._pout
        terms, gls, info = o[:5 * Bt].reshape(Bt, 5), o[5 * Bt:5 * Bt + Bt * d].reshape(Bt, d), o[5 * Bt + Bt * d:]
        ii = np.asarray(idx, dtype=np.int64)
        if np.any(info[ii] != 0):
            return None
        return np.concatenate([terms[ii].reshape(-1), gls[ii].reshape(-1), info[ii]])

    def __del__(self):
        h = getattr(self, "_plan", None)
        if h is not None and getattr(self, "_lib", None) is not None:
            try:
                self._lib.evr_mll_plan_destroy(h)
            except Exception:
                pass
            self._plan = None

    def __call__(self, idx: Sequence[int], xs: Sequence[np.ndarray]):
        n, d = self.n, self.d
        xs = np.ascontiguousarray(np.stack([np.asarray(x, dtype=np.float64) for x in xs]))
        noise, const, raw = xs[:, 0], xs[:, 1], xs[:, 2:]
        # softplus with libm's scalar exp / log1p: the native round driver's arithmetic
        ls = np.array([[_softplus_libm(v) for v in row] for row in raw]).reshape(raw.shape)
        host = self._eval_plan(idx, ls, noise, const) if self.use_plan else None
        if host is None:
            host = self._eval_ops(idx, ls, noise, const)
        B = len(idx)
        terms_h = np.ascontiguousarray(host[:5 * B].reshape(B, 5))
        gls_h = np.ascontiguousarray(host[5 * B:5 * B + B * d].reshape(B, d))
        info_h = host[5 * B + B * d:]
        # ll / n and its gradient with the priors: evr_mll_assemble, the code the native driver
        # (evr_mll_fit_rounds) runs, so both drivers take bitwise the same L-BFGS-B steps
        ll = np.empty(B)
        g = np.empty((B, d + 2))
        lib = _native.load()
        _native.check(lib.evr_mll_assemble(B, n, d, self.prior_spec().ctypes.data, xs.ctypes.data, terms_h.ctypes.data,
                                           gls_h.ctypes.data, ll.ctypes.data, g.ctypes.data), "evr_mll_assemble")
        return [None if info_h[k] != 0 or not np.all(np.isfinite(terms_h[k])) else (float(ll[k]), g[k].copy())
                for k in range(B)]


# the last fit_batch's per-output L-BFGS-B evaluation / iteration counts (tools/fit_probe.py)
LAST_FIT_STATS: dict = {}


def _fit_rounds_native(ev: "MLLBatch", B: int, d: int, x0: np.ndarray, lb: np.ndarray, ub: np.ndarray, maxiter: int,
                       maxfun: int, restart_x) -> List[np.ndarray]:
    """fit_batch's lock-step loop in native code (evr_mll_fit_rounds: per round one MLL plan
    evaluation, the -MLL / n value and gradient with the priors, and every member's L-BFGS-B
    steps, with no Python between rounds).  A round in which a member's attempt-0 factor
    fails comes back here: it is evaluated through MLLBatch (the jitter ladder), members that
    stay not p.d. restart from a prior sample, and the others advance (evr_lbfgsb_advance).
    Same algorithm and state machine as the generator loop (lbfgsb_steps)."""
    from .optim import _EPS, LBFGSB_FG

    lib = _native.load()
    nx = d + 2
    lo = np.ascontiguousarray(lb, dtype=np.float64)
    hi = np.ascontiguousarray(ub, dtype=np.float64)
    runs = (ctypes.c_void_p * B)()
    task = np.zeros(B, dtype=np.int32)
    nit = np.zeros(B, dtype=np.int32)
    nfev = np.zeros(B, dtype=np.int32)
    status = np.zeros(B, dtype=np.int32)
    X = np.zeros((B, nx))
    F = np.zeros(B)
    G = np.zeros((B, nx))
    params = np.zeros(B * nx)
    prior = ev.prior_spec()
    plan = ev.plan_handle()
    i32 = lambda a, k=0: a.ctypes.data + 4 * k  # noqa: E731

    def start(b, xb0):
        if runs[b]:
            lib.evr_lbfgsb_destroy(runs[b])
            runs[b] = None
        h = ctypes.c_void_p()
        _native.check(lib.evr_lbfgsb_create(nx, 10, lo.ctypes.data, hi.ctypes.data, 2.220446049250313e-09 / _EPS,
                                            1e-5, 20, ctypes.byref(h)), "evr_lbfgsb_create")
        runs[b] = h.value
        x0c = np.ascontiguousarray(xb0, dtype=np.float64)
        task[b] = lib.evr_lbfgsb_start(runs[b], x0c.ctypes.data, X[b].ctypes.data)
        nit[b] = nfev[b] = status[b] = 0

    try:
        for b in range(B):
            start(b, x0)
        pending = ctypes.c_int(0)
        while True:
            _native.check(lib.evr_mll_fit_rounds(ops._stream(), plan, ctypes.addressof(runs), task.ctypes.data,
                                                 X.ctypes.data,
                                                 F.ctypes.data, G.ctypes.data, nit.ctypes.data, nfev.ctypes.data,
                                                 status.ctypes.data, int(maxiter), int(maxfun), prior.ctypes.data,
                                                 params.ctypes.data, ctypes.byref(pending)), "evr_mll_fit_rounds")
            if not pending.value:
                break
            idx = [b for b in range(B) if task[b] == LBFGSB_FG]
            vals = ev(idx, [X[b].copy() for b in idx])
            for b, v in zip(idx, vals):
                if v is None:
                    start(b, restart_x(b))
                    continue
                f, g = v
                F[b] = -f
                G[b] = -np.asarray(g, dtype=np.float64)
                _native.check(lib.evr_lbfgsb_advance(runs[b], float(F[b]), G[b].ctypes.data, X[b].ctypes.data,
                                                     i32(task, b), i32(nit, b), i32(nfev, b), i32(status, b),
                                                     int(maxiter), int(maxfun)), "evr_lbfgsb_advance")
        # per-member evaluation / iteration counts (tools/fit_probe.py): max nfev is the number
        # of lock-step rounds since the last restart
        ev.native_stats = {"nfev": nfev.tolist(), "nit": nit.tolist(), "status": status.tolist()}
        LAST_FIT_STATS.update(driver="native", nfev=nfev.tolist(), nit=nit.tolist())
        return [X[b].copy() for b in range(B)]
    finally:
        for b in range(B):
            if runs[b]:
                lib.evr_lbfgsb_destroy(runs[b])


def fit_batch(Xn: torch.Tensor, Y_raw: np.ndarray, kind: int, ls_prior, noise_prior=(-4.0, 1.0),
              max_attempts: int = 10, seed: int = 0, options: Optional[dict] = None,
              standardize: bool = True) -> List[GPHyper]:
    """fit_single for the B columns of ``Y_raw`` (n x B) on shared inputs, in lock-step: each
    output runs its own L-BFGS-B (the native restatement of scipy's, csrc/lbfgsb.cpp; same
    start, bounds and NotPSDError retries with prior samples as fit_single), and every round
    evaluates the outputs that asked for a function value in ONE batched MLL launch chain.
    The fits stay independent problems, as in the reference's per-surrogate
    fit_gpytorch_mll (bofire/surrogates/single_task_gp.py:70-71)."""
    from .optim import lbfgsb_steps

    Y_raw = np.asarray(Y_raw, dtype=np.float64).reshape(Xn.shape[0], -1)
    B, d = Y_raw.shape[1], Xn.shape[1]
    opts = dict(options or {})
    maxiter, maxfun = int(opts.get("maxiter", 15000)), int(opts.get("maxfun", 15000))
    stats, Ys = [], []
    for b in range(B):
        ym, ys = standardize_params(Y_raw[:, b]) if standardize else (0.0, 1.0)
        stats.append((ym, ys))
        Ys.append((Y_raw[:, b] - ym) / ys)
    lsp, nzp = _prior(ls_prior), _prior(noise_prior)
    ev = MLLBatch(Xn, np.stack(Ys), kind, lsp, nzp)
    if nzp is not None and nzp[0] == "lognormal":
        noise0 = math.exp(nzp[1] - nzp[2] ** 2)
    elif nzp is not None and nzp[0] == "gamma" and nzp[1] > 1:
        noise0 = (nzp[1] - 1) / nzp[2]
    else:
        noise0 = 2 * MIN_INFERRED_NOISE_LEVEL
    noise0 = max(noise0, MIN_INFERRED_NOISE_LEVEL)
    lb = np.r_[MIN_INFERRED_NOISE_LEVEL, -np.inf, np.full(d, -np.inf)]
    ub = np.full(d + 2, np.inf)
    rngs = [np.random.default_rng(seed) for _ in range(B)]
    attempts = [0] * B

    def restart_x(b):   # NotPSDError: sample_all_priors, then retry (max_attempts)
        attempts[b] += 1
        if attempts[b] >= max_attempts:
            raise RuntimeError(f"GP fit of output {b} failed after {max_attempts} attempts (NotPSDError)")
        ls = prior_sample_np(lsp, rngs[b], d) if lsp else np.full(d, math.log(2.0))
        nz = max(float(prior_sample_np(nzp, rngs[b], 1)[0]) if nzp else 1e-3, MIN_INFERRED_NOISE_LEVEL)
        return np.concatenate([[nz, 0.0], np.log(np.expm1(ls))])

    if ev.use_plan and os.environ.get("EVR_FIT_NATIVE", "1") != "0":
        xs = _fit_rounds_native(ev, B, d, np.concatenate([[noise0, 0.0], np.zeros(d)]), lb, ub, maxiter, maxfun,
                                restart_x)
        return [GPHyper(lengthscale=softplus_np(xs[b][2:]), noise=float(xs[b][0]), constant=float(xs[b][1]),
                        y_mean=stats[b][0], y_std=stats[b][1]) for b in range(B)]

    def start(x0):
        gen = lbfgsb_steps(x0, lb, ub, maxiter, maxfun)
        return gen, next(gen)

    runs = {b: start(np.concatenate([[noise0, 0.0], np.zeros(d)])) for b in range(B)}
    result, counts = {}, {}
    while runs:
        idx = sorted(runs)
        vals = ev(idx, [runs[b][1] for b in idx])
        for b, v in zip(idx, vals):
            gen, _ = runs[b]
            if v is None:        # NotPSDError: sample_all_priors, then retry (max_attempts)
                gen.close()
                runs[b] = start(restart_x(b))
                continue
            f, g = v
            try:
                runs[b] = (gen, gen.send((-f, -g)))
            except StopIteration as stop:
                result[b] = stop.value.x
                counts[b] = (stop.value.nfev, stop.value.nit)
                del runs[b]
    LAST_FIT_STATS.update(driver="python", nfev=[counts[b][0] for b in range(B)], nit=[counts[b][1] for b in range(B)])
    return [GPHyper(lengthscale=softplus_np(result[b][2:]), noise=float(result[b][0]), constant=float(result[b][1]),
                    y_mean=stats[b][0], y_std=stats[b][1]) for b in range(B)]
