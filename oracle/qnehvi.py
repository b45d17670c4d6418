"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Reference-structure restatement (torch-CPU float64, autograd-capable) of
``qNoisyExpectedHypervolumeImprovement`` as BoFire builds it
(bofire/strategies/predictives/qnehvi.py:23-53: prune_baseline=True, cache_root=True,
alpha=0, output constraints / eta from get_output_constraints), of qEHVI (QehviStrategy / MoboStrategy) and of qEI
(bofire/strategies/predictives/sobo.py:51-90).

It deliberately keeps BoTorch's computation *shape*  so that it doubles as
the CPU baseline timed by bench.py: the joint posterior over [X_baseline; X] is formed per
candidate with the K(X_full, X_train)·L^-T root GEMM, samples come from
``sample_cached_cholesky`` and the HVI is the per-cell scan of ``_compute_qehvi``.

Semantics restated ([upstream] BoTorch >= 0.13):
  * base samples: scrambled Sobol -> inverse normal CDF (``draw_sobol_normal_samples``),
    laid out S x n_points x m (Sobol dim index = point*m + output), baseline rows fixed,
    new rows from a (n_base+q)*m-dim draw of the same seed (``_update_base_samples``).
  * prune: P(point is Pareto-optimal and better than ref) > 0 over 2048 samples of the
    joint posterior at X_baseline (``prune_inferior_points_multi_objective``).
  * cached-Cholesky sampling with ``psd_safe_cholesky(max_tries=6)`` on the new block.
  * HVI with inclusion–exclusion over q-subsets, mean over samples.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch

from .gp import GPState, TK, kernel_matrix, psd_safe_cholesky, require_f64
from .multiobjective import approximate_cells, is_non_dominated, nondominated_cells, pareto_above_ref


def draw_sobol_normal_samples(d: int, n: int, seed: int) -> torch.Tensor:
    """[upstream] botorch.utils.sampling.draw_sobol_normal_samples (inv_transform=True)."""
    eng = torch.quasirandom.SobolEngine(dimension=d, scramble=True, seed=seed)
    u = eng.draw(n, dtype=torch.float64)
    v = 0.5 + (1 - torch.finfo(u.dtype).eps) * (u - 0.5)
    return torch.erfinv(2 * v - 1) * math.sqrt(2)


def base_samples(S: int, n_points: int, m: int, seed: int) -> torch.Tensor:
    return draw_sobol_normal_samples(n_points * m, S, seed).view(S, n_points, m)


def base_samples_pending(S: int, nb: int, npend: int, q: int, m: int, seed: int):
    """Base samples once ``npend`` pending points join a baseline of ``nb`` pruned points
    ([upstream] ``set_X_pending`` with cache_pending=True, max_iep=0: the points are appended
    to X_baseline and the base sampler is extended by ``_update_base_samples``, which keeps
    the existing rows and takes the new rows from a draw of the enlarged dimension with the
    same seed).  Returns (z_base S x (nb+npend) x m, z_new S x q x m)."""
    zb = base_samples(S, nb, m, seed)
    if npend:
        zb = torch.cat([zb, base_samples(S, nb + npend, m, seed)[:, nb:]], 1)
    zn = base_samples(S, nb + npend + q, m, seed)[:, nb + npend:]
    return zb, zn


@dataclass
class Objective:
    """Affine objective g_j(y) = a_j*y_j + b_j (Maximize/Minimize with bounds,
    bofire/utils/torch_tools.py:389-398)."""
    a: torch.Tensor
    b: torch.Tensor

    def __call__(self, y):
        return y * self.a + self.b


@dataclass
class GeneralObjective:
    """Objectives over selected outputs (get_multiobjective_objective,
    bofire/utils/torch_tools.py:699-727): kind 0 = affine p0*y + p1 (Maximize / Minimize,
    :389-398), kind 1 = CloseToTarget -|y - p0|^p1 (:399-402)."""
    out: Sequence[int]
    kind: Sequence[int]
    p0: Sequence[float]
    p1: Sequence[float]

    def __call__(self, y):
        cols = []
        for o, k, a, b in zip(self.out, self.kind, self.p0, self.p1):
            v = y[..., o]
            cols.append(v * a + b if k == 0 else -(torch.abs(v - a) ** b))
        return torch.stack(cols, -1)


@dataclass
class OutputConstraints:
    """Output-constraint callables c(Z) = sign*(Z[..., out] - thr) with their eta
    (constrained_objective2botorch, bofire/utils/torch_tools.py:284-315: Maximize/Minimize
    sigmoid and Target objectives), feasible where c <= 0."""
    out: Sequence[int]
    sign: Sequence[float]
    thr: Sequence[float]
    eta: Sequence[float]

    def values(self, y):
        return torch.stack([s * (y[..., o] - t) for o, s, t in zip(self.out, self.sign, self.thr)], -1)

    def feasible(self, y):
        return (self.values(y) <= 0).all(-1)

    def weight(self, y):
        """[upstream] compute_smoothed_feasibility_indicator(log=False, fat=False): exp of the
        sum of logsigmoid(-c / eta) over the constraints."""
        c = self.values(y)
        eta = torch.as_tensor(list(self.eta), dtype=c.dtype)
        return torch.nn.functional.logsigmoid(-c / eta).sum(-1).exp()


def joint_posterior(models: Sequence[GPState], Xn: torch.Tensor, raw: bool = False):
    """Per-output joint posterior at Xn (... x p x d, normalized).  Returns mean (... x p x m)
    and cov (... x m x p x p), computed the GPyTorch way: R = K(X, Xtr) L^-T.  ``raw``: Xn
    holds raw inputs and each model applies its own Normalize bounds (a ModelListGP whose
    members were fitted on different rows, bofire/surrogates/botorch_surrogates.py:79-128)."""
    require_f64(Xn, "joint_posterior Xn")
    means, covs = [], []
    X_in = Xn
    for st in models:
        Xn = st.normalize(X_in) if raw else X_in
        Ks = kernel_matrix(Xn, st.X, st.lengthscale, st.kind)
        Linv = torch.linalg.solve_triangular(st.L, torch.eye(st.L.shape[0], **TK), upper=False)
        R = Ks @ Linv.T
        mean = st.constant + Ks @ st.alpha
        cov = kernel_matrix(Xn, Xn, st.lengthscale, st.kind) - R @ R.transpose(-1, -2)
        means.append(mean * st.y_std + st.y_mean)
        covs.append(cov * st.y_std ** 2)
    return torch.stack(means, -1), torch.stack(covs, -3)


def prune_baseline(models, Xn, objective, ref, z_prune: torch.Tensor, max_frac: float = 1.0, chunk: int = 0,
                   constraints: Optional[OutputConstraints] = None, raw: bool = False):
    """prune_inferior_points_multi_objective restated.  z_prune: S' x n x m.  Returns the
    kept row indices (sorted, unique) into Xn.  ``chunk`` > 0 walks the S' draws in chunks
    (same counts; bounds the n x n dominance tensors at BASELINE sizes).  Infeasible samples
    (any output constraint > 0) are set to the reference point."""
    mean, cov = joint_posterior(models, Xn, raw)               # n x m, m x n x n
    L, _ = psd_safe_cholesky(cov)                              # m x n x n
    Sp = z_prune.shape[0]
    step = chunk if chunk > 0 else Sp
    counts = torch.zeros(Xn.shape[0], dtype=torch.float64)
    for s0 in range(0, Sp, step):
        Y = mean.unsqueeze(0) + torch.einsum("jik,skj->sij", L, z_prune[s0:s0 + step])
        obj = objective(Y)
        if constraints is not None:
            obj = torch.where(constraints.feasible(Y).unsqueeze(-1), obj, ref)
        pareto = is_non_dominated(obj, deduplicate=False) & (obj > ref).all(-1)
        counts += pareto.to(torch.float64).sum(0)
    probs = counts / Sp
    idx = probs.nonzero().view(-1)
    max_points = math.ceil(max_frac * Xn.shape[0])
    if idx.shape[0] > max_points:
        _, order = torch.sort(probs, stable=True, descending=True)
        idx = order[:max_points]
    return idx.unique(), probs


class QNEHVI:
    """Reference-structure qNEHVI.  models: one GPState per output (shared inputs).
    Xb_n: baseline (already pruned), normalized.  z_base: S x n_b x m; z_new: S x q x m."""

    def __init__(self, models: List[GPState], Xb_n: torch.Tensor, objective: Objective,
                 ref: torch.Tensor, z_base: torch.Tensor, z_new: torch.Tensor, cells=None,
                 constraints: Optional[OutputConstraints] = None, alpha: float = 0.0, raw: bool = False):
        """``raw``: Xb_n and the candidates are raw inputs, normalised per model (joint_posterior).
        ``cells`` (list of 2 x C x m per sample) may be injected to time the forward
        pass alone (bench.py cpu_baseline); parity tests always build their own.
        ``constraints``: baseline samples infeasible under them leave the Pareto sets (set to
        ref), candidate areas are weighted by the smoothed feasibility.
        ``alpha`` > 0 (m > 2): [upstream] NondominatedPartitioning(alpha)'s approximate cells
        (bofire/strategies/predictives/qnehvi.py:50)."""
        self.models = models
        self.Xb = Xb_n
        self.obj = objective
        self.ref = ref
        self.z_base = z_base
        self.z_new = z_new
        self.constraints = constraints
        self.raw = raw
        mean_b, cov_b = joint_posterior(models, Xb_n, raw)     # nb x m, m x nb x nb
        self.L_base, self.base_jitter = psd_safe_cholesky(cov_b)
        Yb = mean_b.unsqueeze(0) + torch.einsum("jik,skj->sij", self.L_base, z_base)
        self.base_obj = objective(Yb)                          # S x nb x m_obj
        if constraints is not None:
            self.base_obj = torch.where(constraints.feasible(Yb).unsqueeze(-1), self.base_obj, ref)
        if cells is not None:
            self.cells = cells
        else:
            part = ((lambda P: approximate_cells(P, ref, alpha)) if alpha > 0 and ref.shape[0] > 2
                    else (lambda P: nondominated_cells(P, ref)))
            self.cells = [part(pareto_above_ref(self.base_obj[s], ref)) for s in range(z_base.shape[0])]

    def samples(self, Xn: torch.Tensor) -> torch.Tensor:
        """Xn: b x q x d normalized -> samples S x b x q x m (sample_cached_cholesky)."""
        b, q, _ = Xn.shape
        nb = self.Xb.shape[0]
        Xfull = torch.cat([self.Xb.expand(b, nb, self.Xb.shape[-1]), Xn], dim=-2)
        mean, cov = joint_posterior(self.models, Xfull, self.raw)   # b x (nb+q) x m, b x m x P x P
        bottom = cov[..., -q:, :]
        bl, br = bottom[..., :nb], bottom[..., nb:]
        bl_chol = torch.linalg.solve_triangular(self.L_base, bl.transpose(-1, -2), upper=False).transpose(-1, -2)
        br_to_chol = br - bl_chol @ bl_chol.transpose(-1, -2)
        br_chol, _ = psd_safe_cholesky(br_to_chol, max_tries=6)
        newL = torch.cat([bl_chol, br_chol], -1)                 # b x m x q x (nb+q)
        z = torch.cat([self.z_base, self.z_new], dim=1)          # S x (nb+q) x m
        s = torch.einsum("bjqk,skj->sbqj", newL, z)
        return mean[..., -q:, :].unsqueeze(0) + s

    def hvi_per_sample(self, obj: torch.Tensor, weights: Optional[torch.Tensor] = None) -> torch.Tensor:
        """obj: S x b x q x m -> S x b (inclusion–exclusion over q-subsets); ``weights``
        (S x b x q feasibility) multiply each subset's areas by their product over the subset
        ([upstream] _compute_qehvi with constraints)."""
        import itertools
        S, b, q, m = obj.shape
        out = torch.zeros(S, b, **TK)
        for s in range(S):
            lo, hi = self.cells[s][0], self.cells[s][1]           # C x m
            for i in range(1, q + 1):
                for sub in itertools.combinations(range(q), i):
                    ov = obj[s][:, list(sub), :].min(dim=-2).values            # b x m
                    ln = (torch.minimum(ov.unsqueeze(-2), hi) - lo).clamp_min(0.0)
                    area = ln.prod(-1).sum(-1)
                    if weights is not None:
                        area = area * weights[s][:, list(sub)].prod(-1)
                    out[s] = out[s] + ((-1) ** (i + 1)) * area
        return out

    def forward(self, Xn: torch.Tensor) -> torch.Tensor:
        Y = self.samples(Xn)
        w = None if self.constraints is None else self.constraints.weight(Y)
        return self.hvi_per_sample(self.obj(Y), w).mean(0)


class QEHVI:
    """Reference-structure qEHVI ([upstream] qExpectedHypervolumeImprovement) as built by
    QehviStrategy._get_acqfs (bofire/strategies/predictives/qehvi.py:37-79) and by
    get_acquisition_function("qEHVI") in MoboStrategy._get_acqfs
    (bofire/strategies/predictives/mobo.py:44-90): one exact partition of the non-dominated
    region of ``Y_part`` above ``ref`` shared by all samples, samples of the independent
    per-output posterior at the candidates only (no baseline), HVI by inclusion–exclusion
    over q-subsets, mean over samples.  z: S x q x m (Sobol dim = point*m + output)."""

    def __init__(self, models: List[GPState], Y_part: torch.Tensor, objective: Objective, ref: torch.Tensor,
                 z: torch.Tensor, constraints: Optional[OutputConstraints] = None,
                 X_pending: Optional[torch.Tensor] = None):
        """``X_pending`` (normalized) joins every candidate's joint batch ([upstream]
        concatenate_pending_points); z then covers q + n_pending points."""
        self.models, self.obj, self.ref, self.z = models, objective, ref, z
        self.constraints, self.X_pending = constraints, X_pending
        self.cell = nondominated_cells(pareto_above_ref(Y_part, ref), ref)

    def samples(self, Xn: torch.Tensor) -> torch.Tensor:
        mean, cov = joint_posterior(self.models, Xn)               # b x q x m, b x m x q x q
        L, _ = psd_safe_cholesky(cov, max_tries=6)
        return mean.unsqueeze(0) + torch.einsum("bjqk,skj->sbqj", L, self.z)

    def forward(self, Xn: torch.Tensor) -> torch.Tensor:
        import itertools
        if self.X_pending is not None:
            Xn = torch.cat([Xn, self.X_pending.unsqueeze(0).expand(Xn.shape[0], *self.X_pending.shape)], -2)
        Y = self.samples(Xn)
        obj = self.obj(Y)                                          # S x b x q x m
        w = None if self.constraints is None else self.constraints.weight(Y)
        S, b, q, m = obj.shape
        lo, hi = self.cell[0], self.cell[1]
        out = torch.zeros(S, b, **TK)
        for i in range(1, q + 1):
            for sub in itertools.combinations(range(q), i):
                ov = obj[:, :, list(sub), :].min(dim=-2).values                   # S x b x m
                ln = (torch.minimum(ov.unsqueeze(-2), hi) - lo).clamp_min(0.0)    # S x b x C x m
                area = ln.prod(-1).sum(-1)
                if w is not None:
                    area = area * w[:, :, list(sub)].prod(-1)
                out = out + ((-1) ** (i + 1)) * area
        return out.mean(0)


# ---------------------------------------------------------------------------------------
# log-space variants (MoboStrategy's default qLogNEHVI, and qLogEHVI)
# [upstream] botorch.acquisition.multi_objective.logei._compute_log_qehvi with fat=True and
# botorch.utils.safe_math (fatplus, fatmax/_pareto, logmeanexp), restated: BoTorch is not
# available offline, so these constants and forms are parity-unpinned against it.
# ---------------------------------------------------------------------------------------
TAU_RELU = 1e-6      # botorch.acquisition.logei.TAU_RELU
TAU_MAX_MO = 1e-3    # qLogEHVI / qLogNEHVI default tau_max
FAT_ALPHA = 2.0      # safe_math ALPHA (power decay of the fat max)
UPPER_CLAMP = 1e10   # cell upper bounds clamp_max (float64)


def fatplus(x: torch.Tensor, tau: float) -> torch.Tensor:
    """tau * (softplus(x/tau) + 0.1 * cauchy(x/tau)), cauchy(x) = 1 / (1 + x^2)."""
    xt = x / tau
    return tau * (torch.nn.functional.softplus(xt) + 0.1 / (1 + xt.square()))


def _pareto(x: torch.Tensor, alpha: float = FAT_ALPHA) -> torch.Tensor:
    a = alpha / 2
    b1 = 2 * a
    b0 = a * b1
    return b0 / (b0 + b1 * x + x.square()).pow(a)


def fatmax(x: torch.Tensor, dim: int, tau: float, alpha: float = FAT_ALPHA) -> torch.Tensor:
    """Fat-tailed smooth max with the +inf handling of safe_math._inf_max_helper."""
    M = x.amax(dim=dim, keepdim=True)
    is_inf_max = torch.isinf(M) & (M > 0)
    y_inf = x.masked_fill(~is_inf_max, 0.0)
    M_no_inf = M.masked_fill(is_inf_max, 0.0)
    y_no_inf = x.masked_fill(is_inf_max, 0.0) - M_no_inf
    fm = M_no_inf + tau * _pareto(-y_no_inf / tau, alpha).sum(dim=dim, keepdim=True).log()
    return torch.where(is_inf_max, y_inf.sum(dim=dim, keepdim=True), fm).squeeze(dim)


def fatmin(x: torch.Tensor, dim: int, tau: float) -> torch.Tensor:
    return -fatmax(-x, dim=dim, tau=tau)


def log_hvi_cells(obj: torch.Tensor, lo: torch.Tensor, hi: torch.Tensor, tau_relu: float, tau_max: float):
    """obj: b x m (one sample, q = 1), cells lo/hi: C x m -> logsumexp over the cells of
    sum_j fatmin(log fatplus(y_j - l_j), log(min(u_j, 1e10) - l_j)) (b)."""
    log_imp = fatplus(obj.unsqueeze(-2) - lo, tau_relu).log()                 # b x C x m
    log_len = (hi.clamp_max(UPPER_CLAMP) - lo).log().expand_as(log_imp)       # b x C x m
    lm = fatmin(torch.stack([log_imp, log_len], -1), dim=-1, tau=tau_max)
    return torch.logsumexp(lm.sum(-1), dim=-1)


def logmeanexp(x: torch.Tensor, dim: int) -> torch.Tensor:
    return torch.logsumexp(x, dim=dim) - math.log(x.shape[dim])


def logdiffexp(log_a: torch.Tensor, log_b: torch.Tensor) -> torch.Tensor:
    """log(exp(a) - exp(b)) for b <= a (safe_math.logdiffexp: a + log1mexp(b - a));
    -inf where the difference is not positive (a cell whose smoothed odd and even subset sums
    cancel contributes nothing instead of a NaN)."""
    d = log_b - log_a
    l1m = torch.where(d > -math.log(2.0), torch.log(-torch.expm1(d)), torch.log1p(-torch.exp(d)))
    out = log_a + l1m
    return torch.where((log_a > log_b) & torch.isfinite(log_a), out, torch.full_like(out, -math.inf))


def log_qehvi_cells(obj: torch.Tensor, lo: torch.Tensor, hi: torch.Tensor, tau_relu: float, tau_max: float,
                    log_feas: Optional[torch.Tensor] = None):
    """[upstream] qLogExpectedHypervolumeImprovement._compute_log_qehvi (fat = True) for one
    MC sample: obj b x q x m, cells lo / hi C x m, log_feas (b x q, log feasibility of each
    point, or None) -> b.  Per cell and q-subset T: the log improvement log fatplus(g_i - l)
    of every point, its fat-min over the points of T, the fat-min with log(min(u, 1e10) - l),
    summed over the objectives (+ sum of log feasibilities over T); logsumexp over the subsets
    of each size, odd sizes added and even sizes subtracted (logdiffexp), logsumexp over
    the cells.  q = 1 equals log_hvi_cells."""
    import itertools
    b, q, m = obj.shape
    log_len = (hi.clamp_max(UPPER_CLAMP) - lo).log()                           # C x m
    pos = torch.full((b, lo.shape[0]), -math.inf, **TK)
    neg = torch.full((b, lo.shape[0]), -math.inf, **TK)
    for i in range(1, q + 1):
        subs = list(itertools.combinations(range(q), i))
        idx = torch.tensor(subs)                                               # n_i x i
        o = obj[:, idx, :]                                                     # b x n_i x i x m
        li = fatplus(o.unsqueeze(1) - lo[None, :, None, None, :], tau_relu).log()   # b x C x n_i x i x m
        li = fatmin(li, dim=-2, tau=tau_max)                                   # b x C x n_i x m
        ll = log_len[None, :, None, :].expand_as(li)
        lens = fatmin(torch.stack([li, ll], -1), dim=-1, tau=tau_max)          # b x C x n_i x m
        area = lens.sum(-1)                                                    # b x C x n_i
        if log_feas is not None:
            area = area + log_feas[:, idx].sum(-1).unsqueeze(1)
        la = torch.logsumexp(area, dim=-1)                                     # b x C
        if i % 2 == 1:
            pos = torch.logaddexp(pos, la)
        else:
            neg = torch.logaddexp(neg, la)
    return torch.logsumexp(logdiffexp(pos, neg), dim=-1)


def log_fatmoid(x: torch.Tensor) -> torch.Tensor:
    """[upstream] botorch.utils.safe_math.log_fatmoid (tau = 1): log of the fat-tailed smooth
    Heaviside fatmoid(x) = 2/3 cauchy(x - m) for x < 0, 1 - 2/3 cauchy(x + m) otherwise, with
    cauchy(x) = 1 / (1 + x^2) and m = sqrt(1/3) (the inflection point; fatmoid(0) = 1/2 on both
    branches).  Its tail is O(1/x^2) as x -> -inf, so infeasible-region gradients decay
    polynomially, not exponentially as the logistic sigmoid's do."""
    m = math.sqrt(1.0 / 3.0)
    neg = math.log(2.0 / 3.0) - torch.log1p((x - m).square())
    pos = torch.log1p(-(2.0 / 3.0) / (1.0 + (x + m).square()))
    return torch.where(x < 0, neg, pos)


def log_feasibility(constraints: Optional[OutputConstraints], Y: torch.Tensor, fat: bool = True):
    """[upstream] compute_smoothed_feasibility_indicator(log=True, fat=fat) as qLogNEHVI /
    qLogEHVI call it (fat = True by default there): the sum over the output constraints of
    log_fatmoid(-c / eta) (fat) or logsigmoid(-c / eta) (not fat); None without constraints."""
    if constraints is None:
        return None
    c = constraints.values(Y)
    eta = torch.as_tensor(list(constraints.eta), dtype=c.dtype)
    x = -c / eta
    return (log_fatmoid(x) if fat else torch.nn.functional.logsigmoid(x)).sum(-1)


class QLogNEHVI(QNEHVI):
    """qLogNEHVI: the qNEHVI samples and per-sample cells, log-space fat-smoothed HVI with
    inclusion–exclusion over q-subsets (log_qehvi_cells), output-constraint log
    feasibilities, logmeanexp over the samples."""

    def __init__(self, *args, tau_relu: float = TAU_RELU, tau_max: float = TAU_MAX_MO, **kw):
        super().__init__(*args, **kw)
        self.tau_relu, self.tau_max = tau_relu, tau_max

    def forward(self, Xn: torch.Tensor) -> torch.Tensor:
        Y = self.samples(Xn)                                                  # S x b x q x m_model
        obj = self.obj(Y)
        lf = log_feasibility(self.constraints, Y)
        lse = torch.stack([log_qehvi_cells(obj[s], self.cells[s][0], self.cells[s][1], self.tau_relu,
                                           self.tau_max, None if lf is None else lf[s])
                           for s in range(obj.shape[0])])
        return logmeanexp(lse, 0)


class QLogEHVI(QEHVI):
    """qLogEHVI: the qEHVI samples (pending points joined) and fixed partition, log-space
    fat-smoothed HVI over q-subsets."""

    def __init__(self, *args, tau_relu: float = TAU_RELU, tau_max: float = TAU_MAX_MO, **kw):
        super().__init__(*args, **kw)
        self.tau_relu, self.tau_max = tau_relu, tau_max

    def forward(self, Xn: torch.Tensor) -> torch.Tensor:
        if self.X_pending is not None:
            Xn = torch.cat([Xn, self.X_pending.unsqueeze(0).expand(Xn.shape[0], *self.X_pending.shape)], -2)
        Y = self.samples(Xn)
        obj = self.obj(Y)
        lf = log_feasibility(self.constraints, Y)
        lse = torch.stack([log_qehvi_cells(obj[s], self.cell[0], self.cell[1], self.tau_relu, self.tau_max,
                                           None if lf is None else lf[s]) for s in range(obj.shape[0])])
        return logmeanexp(lse, 0)


def qei(models, Xn: torch.Tensor, best_f: float, z: torch.Tensor, a: float = 1.0, bconst: float = 0.0):
    """qEI restated (plain MC sampling): mean_S max_q (g(f_s) - best_f)_+.  Xn: b x q x d,
    z: S x q (base samples for the single output)."""
    st = models[0]
    mean, cov = joint_posterior([st], Xn)                          # b x q x 1, b x 1 x q x q
    L, _ = psd_safe_cholesky(cov[..., 0, :, :])
    f = mean[..., 0].unsqueeze(0) + torch.einsum("bqk,sk->sbq", L, z)
    g = a * f + bconst
    return (g - best_f).clamp_min(0.0).max(-1).values.mean(0)
