"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Exact-GP restatement in torch-CPU float64 of BoFire's ``SingleTaskGPSurrogate``
(bofire/surrogates/single_task_gp.py:39-71) on top of [upstream] BoTorch ``SingleTaskGP`` /
GPyTorch ``ExactGP``:

* Normalize input transform with fixed bounds (bofire/surrogates/utils.py:144-154).
* Standardize outcome transform (bofire/surrogates/single_task_gp.py:60-64).
* ConstantMean, RBF / Matérn-ν ARD kernel without outputscale
  (bofire/kernels/mapper.py:31-69; default kernel bofire/data_models/surrogates/single_task_gp.py:109-114).
* Gaussian likelihood, noise ≥ 1e-4 and LogNormal(−4, 1) noise prior
  (bofire/surrogates/single_task_gp.py:68; bofire/data_models/priors/api.py:50).
* ``psd_safe_cholesky`` jitter ladder.
* Exact marginal log likelihood + hyperpriors / n, minimised by scipy L-BFGS-B over the raw
  parameters (bofire/surrogates/single_task_gp.py:70-71).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np
import torch

TK = dict(dtype=torch.float64, device="cpu")

RBF, MATERN05, MATERN15, MATERN25 = 0, 1, 2, 3
KIND_BY_NU = {0.5: MATERN05, 1.5: MATERN15, 2.5: MATERN25}

MIN_INFERRED_NOISE_LEVEL = 1e-4  # [upstream] botorch.models.utils.gpytorch_modules


class NotPSDError(RuntimeError):
    pass


def require_f64(t, what):
    """The oracle computes in f64 only; a float32 input (e.g. torch.tensor of a JSON list) is an
    error of the caller, not something to promote silently."""
    if isinstance(t, torch.Tensor) and t.is_floating_point() and t.dtype != torch.float64:
        raise TypeError(f"{what}: oracle inputs must be float64, got {t.dtype}")


# ---------------------------------------------------------------------------------------
# kernels
# ---------------------------------------------------------------------------------------
def sq_dist(x1: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    """Squared distances by explicit differences (more accurate than GPyTorch's quadratic
    expansion in gpytorch.functions._dist; they agree to ~1e-15 relative)."""
    diff = x1.unsqueeze(-2) - x2.unsqueeze(-3)
    return (diff * diff).sum(-1)


def kernel_from_sqdist(d2: torch.Tensor, kind: int) -> torch.Tensor:
    if kind == RBF:  # gpytorch RBFKernel: exp(-d^2/2)
        return torch.exp(-0.5 * d2)
    # gpytorch MaternKernel: dist = sqrt(clamp_min(d2, 1e-30))
    d = d2.clamp_min(1e-30).sqrt()
    if kind == MATERN05:
        return torch.exp(-d)
    if kind == MATERN15:
        return (1.0 + math.sqrt(3.0) * d) * torch.exp(-math.sqrt(3.0) * d)
    if kind == MATERN25:
        return (1.0 + math.sqrt(5.0) * d + (5.0 / 3.0) * d2) * torch.exp(-math.sqrt(5.0) * d)
    raise ValueError(f"unknown kernel kind {kind}")


def kernel_matrix(x1, x2, lengthscale, kind=RBF, outputscale=1.0):
    """k(x1, x2) with ARD lengthscales; x1: ... x n1 x d, x2: ... x n2 x d."""
    ls = lengthscale
    return outputscale * kernel_from_sqdist(sq_dist(x1 / ls, x2 / ls), kind)


# ---------------------------------------------------------------------------------------
# psd_safe_cholesky  [upstream] linear_operator.utils.cholesky
# ---------------------------------------------------------------------------------------
def psd_safe_cholesky(A: torch.Tensor, jitter: Optional[float] = None, max_tries: int = 3):
    """Plain Cholesky; on failure add jitter*10**i (cumulative total, only to the failing
    batch members) for i < max_tries, else NotPSDError.  Returns (L, jitter_used)."""
    L, info = torch.linalg.cholesky_ex(A)
    used = torch.zeros(A.shape[:-2], **TK)
    if not torch.any(info):
        return L, used
    if torch.isnan(A).any():
        raise NotPSDError("NaN in matrix")
    if jitter is None:
        jitter = 1e-8 if A.dtype == torch.float64 else 1e-6
    Aprime = A.clone()
    jitter_prev = 0.0
    for i in range(max_tries):
        jitter_new = jitter * (10 ** i)
        add = (info > 0).to(A.dtype) * (jitter_new - jitter_prev)
        used = used + add
        Aprime.diagonal(dim1=-2, dim2=-1).add_(add.unsqueeze(-1))
        jitter_prev = jitter_new
        L, info = torch.linalg.cholesky_ex(Aprime)
        if not torch.any(info):
            return L, used
    raise NotPSDError(f"not p.d. after jitter up to {jitter_new:.1e}")


# ---------------------------------------------------------------------------------------
# transforms
# ---------------------------------------------------------------------------------------
def standardize_params(y: torch.Tensor):
    """[upstream] botorch Standardize: mean, unbiased std; std < 1e-8 -> 1; n==1 -> 1."""
    mean = y.mean(0)
    if y.shape[0] == 1:
        std = torch.ones_like(mean)
    else:
        std = y.std(0)
        std = torch.where(std >= 1e-8, std, torch.ones_like(std))
    return mean, std


# ---------------------------------------------------------------------------------------
# GP state (one output)
# ---------------------------------------------------------------------------------------
@dataclass
class GPState:
    X: torch.Tensor            # n x d normalized training inputs
    y: torch.Tensor            # n standardized targets
    lengthscale: torch.Tensor  # d
    noise: float               # sigma^2 (standardized space)
    constant: float            # constant mean (standardized space)
    y_mean: float
    y_std: float
    kind: int = RBF
    lo: Optional[torch.Tensor] = None   # Normalize bounds (raw input space)
    hi: Optional[torch.Tensor] = None
    # caches
    L: torch.Tensor = field(default=None)
    alpha: torch.Tensor = field(default=None)

    def __post_init__(self):
        # torch.tensor(<python list>) is float32: a state built from JSON lists would silently
        # round its inputs / lengthscales to f32 (~6e-8 relative) and move the posterior
        for name in ("X", "y", "lengthscale", "lo", "hi"):
            require_f64(getattr(self, name), f"GPState.{name}")
        self.refresh()

    def refresh(self):
        K = kernel_matrix(self.X, self.X, self.lengthscale, self.kind)
        K = K + self.noise * torch.eye(K.shape[0], **TK)
        self.L, _ = psd_safe_cholesky(K)
        r = (self.y - self.constant).unsqueeze(-1)
        self.alpha = torch.cholesky_solve(r, self.L).squeeze(-1)

    def normalize(self, Xraw: torch.Tensor) -> torch.Tensor:
        if self.lo is None:
            return Xraw
        return (Xraw - self.lo) / (self.hi - self.lo)


def posterior(state: GPState, Xn: torch.Tensor, observation_noise: bool = False, full_cov=False):
    """Exact prediction: mu = c + K*·alpha; cov = K** - (K* L^-T)(K* L^-T)^T,
    un-standardized (mu·s + m, cov·s²); observation_noise adds sigma² before un-standardizing."""
    require_f64(Xn, "posterior Xn")
    Ks = kernel_matrix(Xn, state.X, state.lengthscale, state.kind)          # nt x n
    mean = state.constant + Ks @ state.alpha
    Linv = torch.linalg.solve_triangular(state.L, torch.eye(state.L.shape[0], **TK), upper=False)
    R = Ks @ Linv.T
    if full_cov:
        cov = kernel_matrix(Xn, Xn, state.lengthscale, state.kind) - R @ R.T
        if observation_noise:
            cov = cov + state.noise * torch.eye(cov.shape[0], **TK)
        return mean * state.y_std + state.y_mean, cov * state.y_std ** 2
    var = 1.0 - (R * R).sum(-1)
    if observation_noise:
        var = var + state.noise
    return mean * state.y_std + state.y_mean, var * state.y_std ** 2


def posterior_scipy(state: GPState, Xn: torch.Tensor, observation_noise=False):
    """Independent cross-check of ``posterior`` via scipy cho_factor/cho_solve."""
    import scipy.linalg as sla

    X = state.X.numpy()
    K = kernel_matrix(state.X, state.X, state.lengthscale, state.kind).numpy()
    K = K + state.noise * np.eye(K.shape[0])
    cf = sla.cho_factor(K, lower=True)
    Ks = kernel_matrix(Xn, state.X, state.lengthscale, state.kind).numpy()
    mean = state.constant + Ks @ sla.cho_solve(cf, state.y.numpy() - state.constant)
    var = 1.0 - np.einsum("ij,ji->i", Ks, sla.cho_solve(cf, Ks.T))
    if observation_noise:
        var = var + state.noise
    return mean * state.y_std + state.y_mean, var * state.y_std ** 2


# ---------------------------------------------------------------------------------------
# priors  (bofire/priors/mapper.py:37-50; gpytorch LogNormalPrior)
# ---------------------------------------------------------------------------------------
def lognormal_logpdf(x, loc, scale):
    lx = torch.log(x)
    return -lx - math.log(scale) - 0.5 * math.log(2 * math.pi) - 0.5 * ((lx - loc) / scale) ** 2


def dim_scaled_lognormal(d: int, loc=math.sqrt(2), loc_scaling=0.5, scale=math.sqrt(3), scale_scaling=0.0):
    """bofire/priors/mapper.py:43-50."""
    return loc + math.log(d) * loc_scaling, (scale ** 2 + math.log(d) * scale_scaling) ** 0.5


# ---------------------------------------------------------------------------------------
# MLL (ExactMarginalLogLikelihood + priors) / n
# ---------------------------------------------------------------------------------------
def softplus(x):
    return torch.nn.functional.softplus(x)


def inv_softplus(y):
    return y + torch.log(-torch.expm1(-y))


def mll_value(X, y, raw_ls, noise, constant, kind, ls_prior, noise_prior=(-4.0, 1.0)):
    """Returns the BoTorch fit loss' negative: mll = [log N(y | c, K + s2 I) + log p(ls) +
    log p(s2)] / n as a differentiable torch scalar."""
    ls = softplus(raw_ls)
    n = X.shape[0]
    K = kernel_matrix(X, X, ls, kind) + noise * torch.eye(n, **TK)
    L = torch.linalg.cholesky(K)
    r = (y - constant).unsqueeze(-1)
    a = torch.cholesky_solve(r, L)
    quad = (r * a).sum()
    logdet = 2.0 * torch.log(torch.diagonal(L)).sum()
    ll = -0.5 * quad - 0.5 * logdet - 0.5 * n * math.log(2 * math.pi)
    if ls_prior is not None:
        ll = ll + lognormal_logpdf(ls, *ls_prior).sum()
    if noise_prior is not None:
        ll = ll + lognormal_logpdf(noise, *noise_prior)
    return ll / n


def fit_gp(X, y_raw, kind=RBF, ls_prior=None, noise_prior=(-4.0, 1.0), lo=None, hi=None,
           init=None, maxiter=15000):
    """fit_gpytorch_mll restated: L-BFGS-B over (raw_noise [>=1e-4], constant,
    raw_lengthscale [softplus]) starting from noise = prior mode exp(-5), constant 0,
    lengthscale = softplus(0) = ln 2.  X must already be normalized."""
    from scipy.optimize import minimize

    y_mean, y_std = standardize_params(y_raw.unsqueeze(-1))
    y = (y_raw - y_mean) / y_std
    d = X.shape[1]
    if init is None:
        noise0 = math.exp(noise_prior[0] - noise_prior[1] ** 2) if noise_prior else 1e-4 * 1.1
        x0 = np.concatenate([[noise0, 0.0], np.zeros(d)])
    else:
        x0 = np.asarray(init, dtype=np.float64)

    def f(xv):
        t = torch.tensor(xv, **TK, requires_grad=True)
        v = -mll_value(X, y, t[2:], t[0], t[1], kind, ls_prior, noise_prior)
        v.backward()
        return v.item(), t.grad.numpy().copy()

    bounds = [(MIN_INFERRED_NOISE_LEVEL, None), (None, None)] + [(None, None)] * d
    res = minimize(f, x0, jac=True, method="L-BFGS-B", bounds=bounds, options={"maxiter": maxiter})
    xv = res.x
    st = GPState(X=X, y=y, lengthscale=softplus(torch.tensor(xv[2:], **TK)), noise=float(xv[0]),
                 constant=float(xv[1]), y_mean=float(y_mean), y_std=float(y_std), kind=kind, lo=lo, hi=hi)
    return st, res
