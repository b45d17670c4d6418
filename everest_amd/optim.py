"""Acquisition optimisation driving the device acquisition functions — restates the
[upstream] BoTorch ``optimize_acqf`` path that BoFire calls at
bofire/strategies/predictives/botorch.py:384-405 (q=1, return_best_only=True):

1. raw samples: scrambled Sobol in the bounds, or hit-and-run on the polytope when linear
   constraints are present (``sample_q_batches_from_polytope``: burn-in 10^4, thinning 32);
2. the whole raw batch is evaluated in ONE device launch sequence (the reference walks it
   in chunks of ``batch_limit``);
3. ``initialize_q_batch_nonneg`` (eta=1, alpha=1e-4) picks ``num_restarts`` starts;
4. ``gen_candidates_scipy``: per chunk of ``batch_limit`` restarts, L-BFGS-B (box) or scipy
   SLSQP (linear constraints) minimises -sum_r acq(x_r) with the analytic device gradient.
   L-BFGS-B is the native restatement of scipy's (csrc/lbfgsb.cpp, same iterates, checked
   against scipy in tests/test_lbfgsb_cpu.py); on a device plan the whole loop runs in C++
   (evr_qnehvi_plan_minimize), otherwise through ``minimize_lbfgsb`` with a Python callback.
   ``options["optimizer"]`` / EVR_OPTIMIZER = "scipy" selects scipy's L-BFGS-B instead;
5. candidates clamped to the bounds, re-evaluated, best restart returned.

With ``dist`` (torch.distributed, one process per GPU) the raw batch is sharded over the
ranks and the per-shard acquisition values are all-gathered (RCCL over xGMI) so that every
rank runs the identical Boltzmann selection.  The restart chunks stay the reference's
problems (batch_limit restarts optimised jointly): with at least as many chunks as ranks
each rank owns whole chunks; with fewer, the ranks form one group per chunk that runs the
chunk's optimiser replicated and evaluates it sharded, all-gathering (value, gradient) once
per evaluation — BoFire's default batch_limit = num_restarts is one joint problem over all
ranks.  The per-rank best (value, x) pairs are all-gathered at the end.
"""
from __future__ import annotations

import ctypes
import math
import os
import warnings
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch
from scipy.optimize import minimize

LinearConstraint = Tuple[np.ndarray, np.ndarray, float]   # (indices, coefficients, rhs): sum c*x[idx] >= rhs


@dataclass
class OptimizeStats:
    raw_evals: int = 0
    opt_evals: int = 0
    opt_iters: int = 0
    t_raw: float = 0.0          # raw candidates: draw + screening
    t_raw_draw: float = 0.0     # of which the draw (Sobol, or hit-and-run under linear constraints)
    t_opt: float = 0.0
    chunks: List[dict] = field(default_factory=list)
    restart_X: Optional[np.ndarray] = None    # the optimised restart candidates of this rank's last chunk
    restart_slice: Optional[slice] = None     # the rows of restart_X this rank evaluates
    init_X: Optional[np.ndarray] = None       # the Boltzmann initial conditions

    @property
    def candidates_evaluated(self) -> int:
        return self.raw_evals + self.opt_evals


LBFGSB_FG, LBFGSB_NEW_X, LBFGSB_CONV_PGTOL, LBFGSB_CONV_FACTR, LBFGSB_ABNORMAL, LBFGSB_ERROR = 1, 2, 3, 4, 5, 6
_EPS = float(np.finfo(float).eps)


@dataclass
class LbfgsbResult:
    x: np.ndarray
    fun: float
    nit: int
    nfev: int
    status: int      # 0 converged, 1 iteration / evaluation limit, 2 abnormal line search
    message: str


_TASK_MSG = {LBFGSB_CONV_PGTOL: "CONVERGENCE: NORM OF PROJECTED GRADIENT <= PGTOL",
             LBFGSB_CONV_FACTR: "CONVERGENCE: RELATIVE REDUCTION OF F <= FACTR*EPSMCH",
             LBFGSB_ABNORMAL: "ABNORMAL: line search failed", LBFGSB_ERROR: "ERROR"}


def minimize_lbfgsb(fun: Callable, x0: np.ndarray, lb: np.ndarray, ub: np.ndarray, maxiter: int = 15000,
                    maxfun: int = 15000, maxcor: int = 10, ftol: float = 2.220446049250313e-09, gtol: float = 1e-5,
                    maxls: int = 20) -> LbfgsbResult:
    """Bound-constrained L-BFGS-B through the native restatement (everest_amd/csrc/lbfgsb.cpp)
    with scipy.optimize.minimize(method="L-BFGS-B", jac=True)'s defaults and driver loop:
    ``fun(x) -> (f, g)``; stop after ``maxiter`` iterations or more than ``maxfun``
    evaluations."""
    gen = lbfgsb_steps(x0, lb, ub, maxiter, maxfun, maxcor, ftol, gtol, maxls)
    x = next(gen)
    try:
        while True:
            x = gen.send(fun(x))
    except StopIteration as stop:
        return stop.value


def lbfgsb_steps(x0: np.ndarray, lb: np.ndarray, ub: np.ndarray, maxiter: int = 15000, maxfun: int = 15000,
                 maxcor: int = 10, ftol: float = 2.220446049250313e-09, gtol: float = 1e-5, maxls: int = 20):
    """minimize_lbfgsb as a generator: yields each x to evaluate and receives ``(f, g)``
    through ``send``; returns the LbfgsbResult (StopIteration.value).  Lets independent
    problems advance in lock-step with one batched device evaluation per round (gp.fit_batch)."""
    from . import _native

    lib = _native.load()
    n = int(np.asarray(x0).size)
    lo = np.ascontiguousarray(np.broadcast_to(np.asarray(lb, dtype=np.float64), (n,)))
    hi = np.ascontiguousarray(np.broadcast_to(np.asarray(ub, dtype=np.float64), (n,)))
    x = np.empty(n, dtype=np.float64)
    x0 = np.ascontiguousarray(np.asarray(x0, dtype=np.float64).reshape(n))
    h = ctypes.c_void_p()
    _native.check(lib.evr_lbfgsb_create(n, int(maxcor), lo.ctypes.data, hi.ctypes.data, ftol / _EPS, float(gtol),
                                        int(maxls), ctypes.byref(h)), "evr_lbfgsb_create")
    try:
        task = lib.evr_lbfgsb_start(h, x0.ctypes.data, x.ctypes.data)
        f, g = 0.0, np.zeros(n)
        nit = nfev = 0
        status = 0
        while True:
            if task == LBFGSB_FG:
                f, g = yield x.copy()
                f = float(f)
                g = np.ascontiguousarray(np.asarray(g, dtype=np.float64).reshape(n))
                nfev += 1
                task = lib.evr_lbfgsb_step(h, f, g.ctypes.data, x.ctypes.data)
            elif task == LBFGSB_NEW_X:
                nit += 1
                if nit >= maxiter or nfev > maxfun:
                    status = 1
                    msg = "STOP: TOTAL NO. OF ITERATIONS REACHED LIMIT" if nit >= maxiter else \
                        "STOP: TOTAL NO. OF F,G EVALUATIONS EXCEEDS LIMIT"
                    break
                task = lib.evr_lbfgsb_step(h, f, g.ctypes.data, x.ctypes.data)
            else:
                status = 2 if task == LBFGSB_ABNORMAL else (3 if task == LBFGSB_ERROR else 0)
                msg = _TASK_MSG.get(task, str(task))
                break
    finally:
        lib.evr_lbfgsb_destroy(h)
    return LbfgsbResult(x=x, fun=f, nit=nit, nfev=nfev, status=status, message=msg)


def draw_sobol_samples(bounds: np.ndarray, n: int, seed: int, q: int = 1) -> np.ndarray:
    """[upstream] botorch.utils.sampling.draw_sobol_samples: one (q*d)-dimensional scrambled
    Sobol draw of n points viewed as n x q x d (q = 1: n x d)."""
    lo, hi = bounds
    d = len(lo)
    eng = torch.quasirandom.SobolEngine(q * d, scramble=True, seed=int(seed))
    u = eng.draw(n, dtype=torch.float64).numpy()
    X = lo + (hi - lo) * u.reshape(n, q, d)
    return X[:, 0] if q == 1 else X


_RAW_POOL = None
_RAW_PREFETCHED: dict = {}


def _raw_key(bounds: np.ndarray, n: int, seed: int, q: int):
    return int(seed), int(n), int(q), np.asarray(bounds, dtype=np.float64).tobytes()


def prefetch_raw_samples(bounds: np.ndarray, n: int, gen: torch.Generator, q: int = 1) -> None:
    """Start optimize_acqf's raw Sobol draw on a worker thread as soon as its seed is known:
    the seed is the generator's next draw once the acquisition has drawn its own seeds, so a
    strategy can peek at it (on a copy of the generator) before the acquisition's construction
    and have the draw ready when raw screening starts.  optimize_acqf takes the future if
    (seed, n, q, bounds) match and draws itself otherwise; the values are the same either way.
    EVR_RAW_PREFETCH=0 disables."""
    global _RAW_POOL
    if os.environ.get("EVR_RAW_PREFETCH", "1") == "0":
        return
    g = torch.Generator()
    g.set_state(gen.get_state())
    seed = int(torch.randint(10_000_000, (1,), generator=g).item())
    b = np.array(bounds, dtype=np.float64)
    key = _raw_key(b, n, seed, q)
    if key in _RAW_PREFETCHED:
        return
    while len(_RAW_PREFETCHED) >= 4:
        _RAW_PREFETCHED.pop(next(iter(_RAW_PREFETCHED)))
    if _RAW_POOL is None:
        from concurrent.futures import ThreadPoolExecutor

        _RAW_POOL = ThreadPoolExecutor(max_workers=1, thread_name_prefix="evr-raw")
    _RAW_PREFETCHED[key] = _RAW_POOL.submit(draw_sobol_samples, b, int(n), seed, int(q))


def _as_Ab(d: int, bounds: np.ndarray, ineq: Sequence[LinearConstraint]):
    """Polytope A x <= b from bounds and BoTorch-form inequality constraints."""
    rows, rhs = [], []
    for j in range(d):
        e = np.zeros(d)
        e[j] = 1.0
        rows.append(e.copy()); rhs.append(bounds[1][j])
        rows.append(-e); rhs.append(-bounds[0][j])
    for idx, coef, r in ineq:
        a = np.zeros(d)
        a[np.asarray(idx, dtype=int)] = -np.asarray(coef, dtype=np.float64)   # sum c x >= r  ->  -c x <= -r
        rows.append(a); rhs.append(-r)
    return np.asarray(rows), np.asarray(rhs)


def hit_and_run(bounds: np.ndarray, ineq: Sequence[LinearConstraint], eq: Sequence[LinearConstraint], n: int,
                seed: int, n_burnin: int = 10000, n_thinning: int = 32) -> np.ndarray:
    """Hit-and-run sampler on {bounds, linear (in)equalities} ([upstream]
    HitAndRunPolytopeSampler as used by sample_q_batches_from_polytope)."""
    from scipy.optimize import linprog

    d = bounds.shape[1]
    A, b = _as_Ab(d, bounds, ineq)
    # equality constraints: sample in the null space around a feasible point
    if eq:
        C = np.zeros((len(eq), d))
        ce = np.zeros(len(eq))
        for k, (idx, coef, r) in enumerate(eq):
            C[k, np.asarray(idx, dtype=int)] = np.asarray(coef, dtype=np.float64)
            ce[k] = r
    else:
        C, ce = np.zeros((0, d)), np.zeros(0)
    # interior point: maximise the common slack t s.t. A x + t <= b
    res = linprog(np.r_[np.zeros(d), -1.0], A_ub=np.c_[A, np.ones(len(b))], b_ub=b,
                  A_eq=np.c_[C, np.zeros(len(ce))] if len(ce) else None, b_eq=ce if len(ce) else None,
                  bounds=[(None, None)] * d + [(0, 1)], method="highs")
    if not res.success or res.x[-1] <= 0:
        raise ValueError("linear constraints define an empty polytope")
    x = res.x[:d]
    if len(ce):
        _, s, Vt = np.linalg.svd(C)
        rank = int((s > 1e-12).sum())
        N = Vt[rank:].T
    else:
        N = np.eye(d)
    if N.shape[1] == 0:      # the equalities fix every dimension: the polytope is one point
        return np.repeat(x[None, :], n, axis=0)
    return hit_and_run_chain(A, b, N, x, n, seed, n_burnin, n_thinning)


def hit_and_run_chain(A: np.ndarray, b: np.ndarray, N: np.ndarray, x0: np.ndarray, n: int, seed: int,
                      n_burnin: int, n_thinning: int) -> np.ndarray:
    """The chain of ``hit_and_run`` from the interior point x0 in x0 + span(N): the native
    sampler (csrc/polytope.cpp, evr_hit_and_run; counter-based SplitMix64 variates)."""
    from ._native import check, load

    A = np.ascontiguousarray(A, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    N = np.ascontiguousarray(N, dtype=np.float64)
    x0 = np.ascontiguousarray(x0, dtype=np.float64)
    d, k = N.shape
    out = np.empty((int(n), d))
    p = lambda a: a.ctypes.data   # noqa: E731
    check(load().evr_hit_and_run(d, A.shape[0], p(A), p(b), k, p(N), p(x0), int(n), int(seed) & (2 ** 64 - 1),
                                 int(n_burnin), int(n_thinning), p(out)), "evr_hit_and_run")
    return out


def initialize_q_batch(X: np.ndarray, acq: np.ndarray, n: int, gen: torch.Generator,
                       eta: float = 1.0) -> Tuple[np.ndarray, np.ndarray]:
    """[upstream] botorch.optim.initializers.initialize_q_batch — Boltzmann sampling with
    weights exp(eta * z-score of acq), for acquisition functions that can be negative (the
    log-space ones); the raw maximiser is always kept."""
    ns = X.shape[0]
    if n > ns:
        raise RuntimeError(f"n ({n}) cannot exceed the number of raw samples ({ns})")
    if n == ns:
        return X, acq
    acq_t = torch.as_tensor(acq)
    Ystd = acq_t.std(dim=0)
    if not bool(torch.isfinite(Ystd)) or float(Ystd) == 0.0:
        warnings.warn("All acquisition values for raw samples points are the same for at least one batch. "
                      "Choosing initial conditions at random.")
        idx = torch.randperm(ns, generator=gen)[:n].numpy()
        return X[idx], acq[idx]
    max_val, max_idx = torch.max(acq_t, dim=0)
    etaZ = eta * (acq_t - acq_t.mean(dim=0)) / Ystd
    weights = torch.exp(etaZ)
    while torch.isinf(weights).any():
        etaZ = etaZ * 0.5
        weights = torch.exp(etaZ)
    idx = torch.multinomial(weights, n, generator=gen)
    if int(max_idx) not in idx.tolist():
        idx[-1] = max_idx
    idx = idx.numpy()
    return X[idx], acq[idx]


def initialize_q_batch_nonneg(X: np.ndarray, acq: np.ndarray, n: int, gen: torch.Generator, eta: float = 1.0,
                              alpha: float = 1e-4) -> Tuple[np.ndarray, np.ndarray]:
    """[upstream] botorch.optim.initializers.initialize_q_batch_nonneg (Boltzmann sampling
    of starting points proportional to exp(eta * acq / max))."""
    ns = X.shape[0]
    if n > ns:
        raise RuntimeError(f"n ({n}) cannot exceed the number of raw samples ({ns})")
    if n == ns:
        return X, acq
    acq_t = torch.as_tensor(acq)
    max_val, max_idx = torch.max(acq_t, dim=0)
    if max_val <= 0:
        warnings.warn("All acquisition values for raw sampled points are nonpositive, so initial conditions are "
                      "being selected randomly.")
        idx = torch.randperm(ns, generator=gen)[:n].numpy()
        return X[idx], acq[idx]
    pos = acq_t > 0
    num_pos = int(pos.sum())
    if num_pos < n:
        rem = (~pos).nonzero().view(-1)
        ri = torch.randperm(rem.shape[0], generator=gen)
        pos[rem[ri[: n - num_pos]]] = True
        idx = pos.nonzero().view(-1).numpy()
        return X[idx], acq[idx]
    alpha_pos = acq_t >= alpha * max_val
    while alpha_pos.sum() < n:
        alpha = 0.1 * alpha
        alpha_pos = acq_t >= alpha * max_val
    cand = torch.arange(ns)[alpha_pos]
    w = torch.exp(eta * (acq_t[alpha_pos] / max_val - 1))
    idx = cand[torch.multinomial(w, n, generator=gen)]
    if max_idx not in idx:
        idx[-1] = max_idx
    idx = idx.numpy()
    return X[idx], acq[idx]


def _scipy_constraints(ineq, eq, nb: int, d: int):
    cons = []
    for kind, group in (("ineq", ineq), ("eq", eq)):
        for idx, coef, rhs in group:
            idx = np.asarray(idx, dtype=int)
            coef = np.asarray(coef, dtype=np.float64)
            for r in range(nb):
                cols = r * d + idx
                jac = np.zeros(nb * d)
                jac[cols] = coef
                cons.append({"type": kind, "fun": (lambda x, c=cols, k=coef, v=rhs: float(x[c] @ k - v)),
                             "jac": (lambda x, j=jac: j)})
    return cons


def host_values(t: torch.Tensor) -> np.ndarray:
    """Device acquisition values -> host; NaN marks a candidate whose posterior block was
    not p.d. after the jitter ladder (QNEHVI.forward) and raises NotPSDError like the
    reference.  Every rank sees the same gathered NaN, so all ranks raise together."""
    v = t.cpu().numpy()
    if np.isnan(v).any():
        from .ops import NotPSDError
        raise NotPSDError("acquisition: posterior covariance block not p.d. after the jitter ladder")
    return v


def _reduce_constraints(cons: Sequence[LinearConstraint], fixed: dict, free: List[int]) -> List[LinearConstraint]:
    """Constraints over the free dims only: fixed terms move to the right-hand side
    ([upstream] botorch _generate_unfixed_lin_constraints)."""
    pos = {j: k for k, j in enumerate(free)}
    out = []
    for idx, coef, rhs in cons:
        idx = np.asarray(idx, dtype=int)
        coef = np.asarray(coef, dtype=np.float64)
        keep = np.array([i in pos for i in idx], dtype=bool)
        r = float(rhs) - float(sum(c * fixed[int(i)] for i, c in zip(idx[~keep], coef[~keep])))
        if keep.any():
            out.append((np.array([pos[int(i)] for i in idx[keep]]), coef[keep], r))
    return out


class _FixedFeatures:
    """Acquisition over the free dims with the fixed ones inserted ([upstream]
    FixedFeatureAcquisitionFunction as used by optimize_acqf(fixed_features=...))."""

    def __init__(self, acqf, d: int, fixed: dict):
        self.acqf, self.d, self.dev = acqf, d, acqf.dev
        self.log_acqf = getattr(acqf, "log_acqf", False)
        self.fixed_idx = np.array(sorted(fixed), dtype=int)
        self.fixed_val = np.array([fixed[j] for j in sorted(fixed)], dtype=np.float64)
        self.free = [j for j in range(d) if j not in fixed]

    def full_np(self, x: np.ndarray) -> np.ndarray:
        X = np.empty(x.shape[:-1] + (self.d,))
        X[..., self.free] = x
        X[..., self.fixed_idx] = self.fixed_val
        return X

    def _full_t(self, X: torch.Tensor) -> torch.Tensor:
        out = torch.empty(X.shape[:-1] + (self.d,), dtype=torch.float64, device=self.dev)
        out[..., self.free] = X.to(device=self.dev, dtype=torch.float64)
        out[..., torch.as_tensor(self.fixed_idx, device=self.dev)] = torch.as_tensor(self.fixed_val, device=self.dev)
        return out

    @property
    def supports_plan(self) -> bool:
        return False

    def forward(self, X):
        return self.acqf.forward(self._full_t(X))

    def forward_backward(self, X):
        a, g = self.acqf.forward_backward(self._full_t(X))
        return a, g[..., self.free]

    def eval_host(self, x: np.ndarray, backward: bool):
        if hasattr(self.acqf, "eval_host"):
            a, g = self.acqf.eval_host(self.full_np(x), backward)
            return a, (g[..., self.free] if backward else None)
        Xt = torch.as_tensor(self.full_np(x), dtype=torch.float64, device=self.dev)
        if backward:
            a, g = self.acqf.forward_backward(Xt)
            return a.cpu().numpy(), g[..., self.free].cpu().numpy()
        return self.acqf.forward(Xt).cpu().numpy(), None


def optimize_acqf(acqf, bounds: np.ndarray, num_restarts: int, raw_samples: int, options: dict,
                  gen: torch.Generator, inequality_constraints: Sequence[LinearConstraint] = (),
                  equality_constraints: Sequence[LinearConstraint] = (), dist=None,
                  stats: Optional[OptimizeStats] = None, fixed_features: Optional[dict] = None, q: int = 1,
                  on_init: Optional[Callable[[], None]] = None):
    """Returns (best x, best value, stats); x is (d,) for q = 1, else the joint (q, d) batch
    ([upstream] optimize_acqf(q=...), sequential=False).  ``acqf`` exposes forward(X) and
    forward_backward(X) on device tensors of raw (transformed) inputs, X b x d (q = 1) or
    b x q x d.  ``fixed_features`` {column: value} are held fixed: raw samples get them set,
    the restarts optimise the free columns only ([upstream] optimize_acqf(fixed_features=...)).
    Linear constraints apply to every point of a q-batch."""
    q = int(q)
    if q < 1:
        raise ValueError("q must be >= 1")
    if fixed_features:
        bounds = np.asarray(bounds, dtype=np.float64)
        d_full = bounds.shape[1]
        fx = {int(k): float(v) for k, v in fixed_features.items()}
        wrap = _FixedFeatures(acqf, d_full, fx)
        x, v, st = optimize_acqf(wrap, bounds[:, wrap.free], num_restarts, raw_samples, options, gen,
                                 _reduce_constraints(inequality_constraints, fx, wrap.free),
                                 _reduce_constraints(equality_constraints, fx, wrap.free), dist=dist, stats=stats,
                                 q=q, on_init=on_init)
        return wrap.full_np(x), v, st
    import time

    stats = stats or OptimizeStats()
    bounds = np.asarray(bounds, dtype=np.float64)
    d = bounds.shape[1]
    dev = acqf.dev
    batch_limit = int(options.get("batch_limit") or num_restarts)
    maxiter = int(options.get("maxiter", 2000))
    world = dist.get_world_size() if dist is not None else 1
    rank = dist.get_rank() if dist is not None else 0
    cdev = comm_device(dist, dev)

    # 1. raw samples (seeded from the strategy's torch generator -> identical on every rank)
    seed = int(torch.randint(10_000_000, (1,), generator=gen).item())
    t0 = time.perf_counter()
    if inequality_constraints or equality_constraints:
        X_raw = hit_and_run(bounds, inequality_constraints, equality_constraints, raw_samples * q, seed)
        if q > 1:
            X_raw = X_raw.reshape(raw_samples, q, d)
    else:
        fut = _RAW_PREFETCHED.pop(_raw_key(bounds, raw_samples, seed, q), None)
        X_raw = fut.result() if fut is not None else draw_sobol_samples(bounds, raw_samples, seed, q)
    stats.t_raw_draw += time.perf_counter() - t0
    shp = (q, d) if q > 1 else (d,)          # one candidate (q-batch) of the acquisition
    # 2. evaluate (sharded over ranks, all-gather of the per-shard values)
    Xr = torch.as_tensor(X_raw, dtype=torch.float64, device=dev)
    if world > 1:
        per = math.ceil(raw_samples / world)
        lo_i, hi_i = rank * per, min(raw_samples, (rank + 1) * per)
        part = torch.zeros(per, dtype=torch.float64, device=cdev)
        if hi_i > lo_i:
            part[: hi_i - lo_i] = acqf.forward(Xr[lo_i:hi_i]).to(cdev)
        bufs = [torch.empty_like(part) for _ in range(world)]
        dist.all_gather(bufs, part)
        Y_raw = torch.cat(bufs)[:raw_samples]
    else:
        Y_raw = acqf.forward(Xr)
    Y_raw = host_values(Y_raw)
    stats.raw_evals += raw_samples
    stats.t_raw += time.perf_counter() - t0

    # 3. Boltzmann initial conditions
    init = initialize_q_batch if getattr(acqf, "log_acqf", False) else initialize_q_batch_nonneg
    X0, _ = init(X_raw, Y_raw, num_restarts, gen)
    stats.init_X = X0
    if on_init is not None:
        on_init()    # the generator's draws of this ask are done (e.g. the next ask's prefetch)

    # 4. restarts, chunks of batch_limit, L-BFGS-B (box) / SLSQP (linear constraints) on host
    #    with the analytic device value+gradient
    t0 = time.perf_counter()
    results = []
    chunks = [(s, min(num_restarts, s + batch_limit)) for s in range(0, num_restarts, batch_limit)]
    optimizer = options.get("optimizer") or os.environ.get("EVR_OPTIMIZER", "native")
    if optimizer not in ("native", "scipy"):
        raise ValueError(f"optimizer must be 'native' or 'scipy', got {optimizer!r}")
    # chunk -> ranks: every chunk is the reference's own problem (batch_limit restarts
    # optimised jointly); with at least as many chunks as ranks each rank owns whole chunks
    # (no per-iteration collective), with fewer the ranks form one group per chunk and each
    # group evaluates its chunk sharded
    layout = restart_layout(len(chunks), world)
    if world > 1:
        _Shard.ensure_groups(dist, layout)

    def run_chunk(s0: int, s1: int, shard: "_Shard"):
        nb = s1 - s0
        x0 = X0[s0:s1].reshape(-1)
        lbv, ubv = np.tile(bounds[0], nb * q), np.tile(bounds[1], nb * q)
        cons = _scipy_constraints(inequality_constraints, equality_constraints, nb * q, d)
        if (not cons and optimizer == "native" and shard.k == 1 and q == 1
                and getattr(acqf, "supports_plan", False)):
            # the whole L-BFGS-B loop in C++ on the device plan (no Python per iteration)
            Xc, vals, info = acqf.plan(nb, True).minimize(x0, lbv, ubv, maxiter)
            return vals, Xc.reshape(nb, d), {"restarts": nb, "evals": info[1], "nit": info[0], "status": info[2],
                                             "driver": "native-plan", "local_batch": nb}
        counter = {"n": 0}

        def f(x):
            a, g = shard.evaluate(acqf, x.reshape((nb,) + shp), True)
            counter["n"] += 1
            acc = 0.0
            for v in a.tolist():         # sequential, as evr_qnehvi_plan_minimize sums (bitwise equal paths)
                acc += v
            return -acc, -g.reshape(-1)

        if cons:
            res = minimize(f, x0, jac=True, method="SLSQP", bounds=list(zip(lbv, ubv)), constraints=cons,
                           options={"maxiter": maxiter})
            drv = "scipy-slsqp"
        elif optimizer == "native":
            res = minimize_lbfgsb(f, x0, lbv, ubv, maxiter=maxiter)
            drv = "native"
        else:
            res = minimize(f, x0, jac=True, method="L-BFGS-B", bounds=list(zip(lbv, ubv)),
                           options={"maxiter": maxiter})
            drv = "scipy"
        if shard.k > 1:
            drv += f"-sharded{shard.k}"
        Xc = np.clip(res.x.reshape((nb,) + shp), bounds[0], bounds[1])
        # re-scored through the evaluation path the iterations used (the restart batch's fused
        # scan forms acq in its own summation order; evr_qnehvi_plan_minimize re-scores the
        # same way), so both drivers return bitwise the same values
        vals, _ = shard.evaluate(acqf, Xc, True)
        return vals, Xc, {"restarts": nb, "evals": counter["n"], "nit": int(getattr(res, "nit", 0)),
                          "status": int(res.status), "driver": drv, "local_batch": shard.local_size(nb)}

    err: Optional[BaseException] = None
    for ci, (s0, s1) in enumerate(chunks):
        ranks = layout[ci]
        if rank not in ranks:
            continue
        shard = _Shard(dist, ranks, rank, world, cdev)
        try:
            vals, Xc, info = run_chunk(s0, s1, shard)
        except Exception as e:   # noqa: BLE001 — re-raised on every rank after the exchange below
            if world == 1:
                raise
            err = e
            break
        if shard.idx == 0:        # each chunk's work is counted once, by its group's first rank
            stats.opt_evals += info["evals"] * info["restarts"] + info["restarts"]
        stats.opt_iters += info["nit"]
        stats.chunks.append(info)
        stats.restart_X = Xc
        stats.restart_slice = shard.slice_of(s1 - s0)
        results.append((vals, Xc))
    if results:
        vals = np.concatenate([r[0] for r in results])
        Xs = np.concatenate([r[1] for r in results])
        k = int(np.argmax(vals))
        best_v, best_x = float(vals[k]), Xs[k]
    else:
        best_v, best_x = -np.inf, np.zeros(shp)
    if world > 1:
        # all-gather every rank's (error flag, best value, x) over RCCL; a failure on any rank
        # raises on every rank (no rank is left waiting in a collective); argmax, ties -> lowest rank
        flag = 0.0 if err is None else (2.0 if _is_notpsd(err) else 1.0)
        loc = torch.tensor(np.r_[flag, best_v, np.ravel(best_x)], dtype=torch.float64, device=cdev)
        bufs = [torch.empty_like(loc) for _ in range(world)]
        dist.all_gather(bufs, loc)
        allv = torch.stack(bufs).cpu().numpy()
        if (allv[:, 0] > 0).any():
            if err is not None:
                raise err
            bad = [int(r) for r in np.nonzero(allv[:, 0] > 0)[0]]
            if (allv[bad, 0] == 2.0).all():
                from .ops import NotPSDError
                raise NotPSDError(f"acquisition not p.d. on rank(s) {bad} (restart chunk)")
            raise RuntimeError(f"restart optimisation failed on rank(s) {bad}")
        k = int(np.argmax(allv[:, 1]))
        best_v, best_x = float(allv[k, 1]), allv[k, 2:].reshape(shp)
        cnt = torch.tensor([stats.opt_evals], dtype=torch.float64, device=cdev)
        dist.all_reduce(cnt)
        stats.opt_evals_global = int(cnt.item())
    else:
        stats.opt_evals_global = stats.opt_evals
    stats.t_opt += time.perf_counter() - t0
    return best_x, best_v, stats


def comm_device(dist, dev):
    """Where the exchange buffers live: the GPU for RCCL ("nccl"), the host for gloo (the
    CPU tests, and multi-rank rehearsals sharing one GPU)."""
    if dist is None or not dist.is_initialized():
        return dev
    return torch.device("cpu") if dist.get_backend() == "gloo" else dev


def restart_layout(n_chunks: int, world: int) -> List[Tuple[int, ...]]:
    """Ranks that optimise each restart chunk.  Chunks >= ranks: chunk c on rank c mod N
    alone; fewer chunks than ranks: the ranks split into one contiguous group per chunk
    (sizes differ by at most one), so no rank idles; a single chunk (BoFire's default
    batch_limit = num_restarts) is one joint problem evaluated by every rank."""
    if world <= 1:
        return [(0,)] * n_chunks
    if n_chunks >= world:
        return [(c % world,) for c in range(n_chunks)]
    out, r = [], 0
    for c in range(n_chunks):
        sz = world // n_chunks + (1 if c < world % n_chunks else 0)
        out.append(tuple(range(r, r + sz)))
        r += sz
    return out


_GROUPS: dict = {}


class _Shard:
    """One rank's part of a restart chunk optimised by the rank group ``ranks``: every member
    runs the same host optimiser on identical bytes (replicated, deterministic), evaluates its
    slice of the chunk's restarts on its GPU, and the (value[, gradient]) slices are
    all-gathered in the group (RCCL over xGMI) once per optimiser evaluation."""

    def __init__(self, dist, ranks: Tuple[int, ...], rank: int, world: int, dev):
        self.dist, self.ranks, self.dev = dist, tuple(ranks), dev
        self.k = len(self.ranks)
        self.idx = self.ranks.index(rank)
        self.pg = None
        if 1 < self.k < world:
            key = self.ranks
            if key not in _GROUPS:
                # new_group is collective over the world: every rank creates every group of the
                # layout in the same order (restart_layout is a function of (chunks, world) only)
                raise RuntimeError("restart group not created")
            self.pg = _GROUPS[key]

    @staticmethod
    def ensure_groups(dist, layout):
        for ranks in layout:
            if len(ranks) > 1 and len(ranks) < dist.get_world_size() and tuple(ranks) not in _GROUPS:
                _GROUPS[tuple(ranks)] = dist.new_group(list(ranks))

    def _bounds(self, nb: int):
        sizes = [nb // self.k + (1 if i < nb % self.k else 0) for i in range(self.k)]
        starts = np.cumsum([0] + sizes)
        return sizes, starts

    def slice_of(self, nb: int) -> slice:
        sizes, starts = self._bounds(nb)
        return slice(int(starts[self.idx]), int(starts[self.idx + 1]))

    def local_size(self, nb: int) -> int:
        return self._bounds(nb)[0][self.idx]

    def evaluate(self, acqf, X: np.ndarray, with_grad: bool):
        """(values (nb,), gradients shaped like X | None) of the whole chunk X on every member.
        One all-gather of [flag | value | gradient] rows into one tensor and one copy to the
        host per evaluation; a member whose local evaluation raises still joins the gather with
        its flag set, so every member raises together and no collective is left unmatched."""
        nb = X.shape[0]
        if self.k == 1:
            return _local_eval(acqf, X, with_grad)
        sizes, starts = self._bounds(nb)
        per = max(sizes)
        nx = int(np.prod(X.shape[1:]))
        i0, i1 = int(starts[self.idx]), int(starts[self.idx + 1])
        loc = np.zeros((per, 2 + nx))
        err: Optional[BaseException] = None
        if i1 > i0:
            try:
                a, g = _local_eval(acqf, X[i0:i1], with_grad, check=False)
                loc[: i1 - i0, 1] = a
                if with_grad:
                    loc[: i1 - i0, 2:] = g.reshape(i1 - i0, nx)
            except Exception as e:   # noqa: BLE001 — re-raised after the gather, on every member
                err = e
                loc[0, 0] = 2.0 if _is_notpsd(e) else 1.0
        lt = torch.as_tensor(loc, device=self.dev)
        out = torch.empty((self.k * per, 2 + nx), dtype=torch.float64, device=self.dev)
        self.dist.all_gather_into_tensor(out, lt, group=self.pg)
        allr = out.cpu().numpy().reshape(self.k, per, 2 + nx)
        flags = allr[:, 0, 0]
        if (flags > 0).any():
            if err is not None:
                raise err
            bad = [self.ranks[i] for i in np.nonzero(flags > 0)[0]]
            if (flags[flags > 0] == 2.0).all():
                from .ops import NotPSDError
                raise NotPSDError(f"acquisition not p.d. on rank(s) {bad} (sharded evaluation)")
            raise RuntimeError(f"sharded acquisition evaluation failed on rank(s) {bad}")
        full = np.concatenate([allr[i, :sz, 1:] for i, sz in enumerate(sizes)])
        host_values(torch.from_numpy(full[:, 0]))
        return full[:, 0], (full[:, 1:].reshape(X.shape) if with_grad else None)


def _local_eval(acqf, X: np.ndarray, with_grad: bool, check: bool = True):
    """This rank's evaluation of X (numpy) -> (values, gradients | None) numpy: one native plan
    round trip (eval_host) where the acquisition has it, else the device ops."""
    if hasattr(acqf, "eval_host"):
        a, g = acqf.eval_host(X, with_grad)
    else:
        Xt = torch.as_tensor(X, dtype=torch.float64, device=acqf.dev)
        if with_grad:
            a, g = acqf.forward_backward(Xt)
            a, g = a.cpu().numpy(), g.cpu().numpy()
        else:
            a, g = acqf.forward(Xt).cpu().numpy(), None
    if check:
        host_values(torch.from_numpy(np.asarray(a)))
    return np.asarray(a), g


def _is_notpsd(e: BaseException) -> bool:
    from .ops import NotPSDError
    return isinstance(e, NotPSDError)


def optimize_acqf_mixed(acqf, bounds: np.ndarray, fixed_features_list: Sequence[dict], num_restarts: int,
                        raw_samples: int, options: dict, gen: torch.Generator,
                        inequality_constraints: Sequence[LinearConstraint] = (),
                        equality_constraints: Sequence[LinearConstraint] = (), dist=None, q: int = 1):
    """[upstream] botorch.optim.optimize_acqf_mixed (q = 1), as BoFire calls it for the
    EXHAUSTIVE categorical method (bofire/strategies/predictives/botorch.py:358-378): one
    optimize_acqf per fixed-feature combination, best acquisition value wins (first on ties).
    q > 1 is BoTorch's sequential greedy over pending points, which needs the acquisition
    rebuilt with the chosen rows pending: BotorchStrategy._ask_mixed_sequential drives it."""
    if q != 1:
        raise ValueError("optimize_acqf_mixed runs q = 1 rounds; q > 1 is the strategy's sequential greedy "
                         "(BotorchStrategy._ask_mixed_sequential)")
    stats = OptimizeStats()
    best = (None, -np.inf)
    stats.mixed_values = []
    for ff in fixed_features_list:
        x, v, stats = optimize_acqf(acqf, bounds, num_restarts, raw_samples, options, gen, inequality_constraints,
                                    equality_constraints, dist=dist, stats=stats, fixed_features=ff)
        stats.mixed_values.append(float(v))     # each combination's optimum, in combination order
        if best[0] is None or v > best[1]:
            best = (x, v)
    return best[0], best[1], stats
