"""qNEHVI (q = 1) acquisition resident in HBM — construction, forward and analytic backward.

Replaces [upstream] ``qNoisyExpectedHypervolumeImprovement`` as built by
``QnehviStrategy._get_acqfs`` (bofire/strategies/predictives/qnehvi.py:23-53:
prune_baseline=True, cache_root=True, alpha=0, eta=1e-3 without output constraints).

Algebraic restructuring (results preserved): the reference forms, per
candidate, the joint posterior over [X_baseline; x] through a (n_base+1) x n x n GEMM and
then solves against the cached baseline root.  Because every baseline point is a training
point (get_acqf_input_tensors, bofire/strategies/predictives/botorch.py:696-724), all of
that collapses to one per-ask operator per output

    M_j = [ L^-1 ; G_j ; H_j^T ; alpha_j^T ]     (n + n_base + S + 1) x n
    G_j = s_j^2 L_base^-1 (P - A_b^T L^-1),  A_b = L^-1 K(X_tr, X_base),  H_j = G_j^T Z_base

applied to k(X_tr, x): R = M K_x is a dense MFMA GEMM over the candidate batch, and
    mu = m + s (c + alpha.k), var = s^2 (1 - |L^-1 k|^2), L21 = G k, L22^2 = var - |L21|^2,
    y_s = mu + L21.z_base,s + L22 z_q,s      (= sample_cached_cholesky, psd_safe max_tries=6)
followed by the box-cell HVI scan and the mean over samples.
"""
from __future__ import annotations

import ctypes
import math
import os
import warnings
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch

from . import _native, ops
from .gp import GPBatch


def sobol_base_samples(S: int, n_points: int, m: int, seed: int, device, scrambled=None) -> torch.Tensor:
    """Device Sobol-normal base samples in the GEMM-ready layout m x n_points x S
    ([upstream] draw_sobol_normal_samples(n_points*m, S, seed), Sobol dim = point*m + output)."""
    return ops.sobol_normal(S, n_points * m, seed, device, layout=1, m=m, scrambled=scrambled)


_SCRAMBLE_POOL = None


def _prefetch_scramble(dim: int, seed: int, d0: int = 0, nd: Optional[int] = None):
    """Start ops.sobol_scramble on a worker thread (the host half of a Sobol draw overlaps the
    device work queued meanwhile and the other draws); returns a future, or None for an empty
    range."""
    global _SCRAMBLE_POOL
    nd = dim - d0 if nd is None else nd
    if nd <= 0:
        return None
    key = (int(dim), int(seed), int(d0), int(nd))
    fut = _PREFETCHED.pop(key, None)   # started earlier by prefetch_scramble
    if fut is not None:
        return fut
    if _SCRAMBLE_POOL is None:
        from concurrent.futures import ThreadPoolExecutor

        _SCRAMBLE_POOL = ThreadPoolExecutor(max_workers=3, thread_name_prefix="evr-sobol")
    return _SCRAMBLE_POOL.submit(ops.sobol_scramble, dim, seed, d0, nd)


_PREFETCHED = {}


def prefetch_scramble(dim: int, seed: int, d0: int = 0, nd: Optional[int] = None) -> None:
    """Start the host scrambling of a Sobol draw as soon as its seed and dimension are known
    (a strategy draws its seeds before building the acquisition); the acquisition's own
    request for the same (dim, seed, range) takes the running future instead of starting
    another.  At most 8 are kept."""
    nd = dim - d0 if nd is None else nd
    key = (int(dim), int(seed), int(d0), int(nd))
    if nd <= 0 or key in _PREFETCHED:
        return
    while len(_PREFETCHED) >= 8:
        _PREFETCHED.pop(next(iter(_PREFETCHED)))
    _PREFETCHED[key] = _prefetch_scramble(dim, seed, d0, nd)


def _submit(fn, *args):
    global _SCRAMBLE_POOL
    if _SCRAMBLE_POOL is None:
        from concurrent.futures import ThreadPoolExecutor

        _SCRAMBLE_POOL = ThreadPoolExecutor(max_workers=3, thread_name_prefix="evr-sobol")
    return _SCRAMBLE_POOL.submit(fn, *args)


def _prefetch_from_stream(fut_stream, dim: int, d0: int = 0, nd: Optional[int] = None):
    """Scramble dims [d0, d0+nd) of a dim-dimensional draw from a seed stream a worker is
    generating (fut_stream).  The future's result is None when the stream cannot serve the
    draw; ops.sobol_normal then scrambles (or falls back to IID normals) itself."""
    nd = dim - d0 if nd is None else nd
    if nd <= 0:
        return None
    return _submit(lambda: fut_stream.result().scramble(dim, d0, nd))


def _result(fut):
    return None if fut is None else fut.result()


def _host_threads() -> int:
    v = os.environ.get("EVR_HOST_THREADS") or os.environ.get("OMP_NUM_THREADS")
    try:
        return max(1, int(v)) if v else min(16, os.cpu_count() or 1)
    except ValueError:
        return 1


def _single_cell(ref: torch.Tensor, S: int, m: int) -> ops.Cells:
    """Empty Pareto set: one cell [ref, +inf) per sample (the whole region above ref)."""
    dev = ref.device
    return ops.Cells(torch.arange(S + 1, dtype=torch.int32, device=dev), np.ones(S, dtype=np.int64), m,
                     lo=ref.unsqueeze(0).repeat(S, 1).contiguous(),
                     hi=torch.full((S, m), math.inf, dtype=torch.float64, device=dev))


def _decompose(O: torch.Tensor, ref: torch.Tensor, box_device=None, kd_scan=None, num_threads=None,
               alpha: float = 0.0):
    """Non-dominated box decomposition above ref of every sample of O (m x P x S): exact
    (device kernel + kd ordering, or the native host partition beyond the device limits), or
    for alpha > 0 with m > 2 the approximate partition of [upstream]
    NondominatedPartitioning(alpha) (host, explicit cells for the tiled scan; BoTorch's own
    partition for that case is a host loop too).  Returns (cells, path)."""
    m, P, _ = O.shape
    dev = O.device
    approx = alpha > 0.0 and m > 2
    if approx and box_device:
        raise ValueError("the device box decomposition is exact only (alpha = 0)")
    if not approx and (box_device if box_device is not None else ops.box_device_supported(P, m)):
        kd_built = False
        try:
            if kd_scan is False or os.environ.get("EVR_BOX_PIPELINE", "1") == "0":
                cells = ops.box_decompose_device(O, ref)
            else:   # box, pack and kd order in one native call (EVR_BOX_PIPELINE=0: the op sequence)
                cells, kd_built = ops.box_decompose_kd_device(O, ref, want_kd=True)
        except ops.BoxCapacityError as e:
            if box_device:      # explicitly requested: surface the limit
                raise
            warnings.warn(f"{e}; using the exact host partition", RuntimeWarning)
            cells = None
        if cells is not None:
            path = "device"
            if kd_built:
                path = "device+kd"
            elif kd_scan if kd_scan is not None else ops.kd_supported(cells):
                ops.cells_kd_order(cells)
                path = "device+kd"
            elif kd_scan is None:
                warnings.warn(f"{int(cells.counts.max())} cells in one sample exceed the sparse kd scan's limit; "
                              "using the dense tiled scan (~10x slower)", RuntimeWarning)
            return cells, path
    elif not approx and box_device is None:
        warnings.warn(f"{P} points x {m} objectives exceed the device box decomposition's limits; "
                      "using the host partition", RuntimeWarning)
    mask, _ = ops.pareto_mask(O, ref, dedup=True)
    lo, hi, off = ops.box_decompose(O.cpu().numpy(), ref.cpu().numpy(), mask.cpu().numpy(),
                                    num_threads or _host_threads(), layout="jis", alpha=alpha if approx else 0.0)
    f64 = dict(dtype=torch.float64, device=dev)
    return ops.Cells(torch.as_tensor(off, dtype=torch.int32, device=dev), np.diff(off), m,
                     lo=torch.as_tensor(lo, **f64), hi=torch.as_tensor(hi, **f64)), \
        ("host-approx" if approx else "host")


_BOX_POOL = None
_SIDE_STREAMS = {}


def _decompose_async(O: torch.Tensor, ref: torch.Tensor, *args):
    """_decompose on a side stream, driven from a worker thread, so that the box decomposition
    and kd ordering (one workgroup per MC sample: ~2.6 ms at the bench shape, with a host sync
    for the cell counts in between) overlap the fused-root operator the caller queues on its
    own stream meanwhile.  Returns join(): (cells, path), after which the caller's stream waits
    for the side stream.  EVR_BOX_OVERLAP=0 runs it inline."""
    global _BOX_POOL
    if os.environ.get("EVR_BOX_OVERLAP", "1") == "0" or not O.is_cuda:
        res = _decompose(O, ref, *args)
        return lambda: res
    dev = O.device
    main = torch.cuda.current_stream(dev)
    side = _SIDE_STREAMS.get(dev)
    if side is None:
        side = _SIDE_STREAMS[dev] = torch.cuda.Stream(dev)
    ready = torch.cuda.Event()
    ready.record(main)
    O.record_stream(side)
    ref.record_stream(side)
    if _BOX_POOL is None:
        from concurrent.futures import ThreadPoolExecutor

        _BOX_POOL = ThreadPoolExecutor(max_workers=1, thread_name_prefix="evr-box")

    def job():
        with torch.cuda.device(dev), torch.cuda.stream(side):
            side.wait_event(ready)
            return _decompose(O, ref, *args)

    fut = _BOX_POOL.submit(job)

    def join():
        cells, path = fut.result()
        main.wait_stream(side)
        ts = [cells.off, cells.lo, cells.hi, cells.keys, cells.pts, cells.rank0]
        if cells.kd is not None:
            kd = cells.kd
            ts += [kd.goff, kd.keys, kd.rank, kd.box, kd.sorted_lo]
        for t in ts:
            if isinstance(t, torch.Tensor) and t.is_cuda:
                t.record_stream(main)
        return cells, path

    return join


def _make_spec(m: int, obj_a, obj_b, objective, constraints) -> ops.GeneralSpec:
    """Objective / constraint description: explicit ``objective`` [(output, kind, p0, p1)],
    else one affine objective a_j*y_j + b_j per output."""
    if objective is None:
        a = np.asarray(obj_a, dtype=np.float64).reshape(-1)
        b = np.asarray(obj_b, dtype=np.float64).reshape(-1)
        if a.shape[0] != m or b.shape[0] != m:
            raise ValueError(f"obj_a / obj_b need one entry per model output ({m})")
        objective = [(j, ops.OBJ_AFFINE, a[j], b[j]) for j in range(m)]
    return ops.GeneralSpec(m, objective, constraints or ())


def _fast_affine(spec: ops.GeneralSpec, m: int, dev):
    """obj_a / obj_b of the q = 1 fast path (identity placeholders when it does not apply)."""
    f64 = dict(dtype=torch.float64, device=dev)
    if spec.affine_identity:
        return (torch.tensor([o[2] for o in spec.objectives], **f64),
                torch.tensor([o[3] for o in spec.objectives], **f64))
    return torch.ones(m, **f64), torch.zeros(m, **f64)


@dataclass
class ConstructionStats:
    n_train: int
    n_base: int
    total_cells: int
    max_cells: int
    prune_probs: Optional[np.ndarray] = None


class _BoxHviAcqf:
    """Evaluation side shared by qNEHVI and qEHVI: the per-ask operator ``M`` applied to the
    cross-covariance, the sampling step, the box-cell HVI scan and their analytic backward
    (subclasses set gp, dev, Xk, M, state, model and _plans)."""

    # the attributes the reference's tests read off BoTorch's acquisition objects
    # (tests/bofire/strategies/test_mobo.py:123-160): ref_point, constraints, eta
    @property
    def ref_point(self) -> torch.Tensor:
        return self.ref

    @property
    def constraints(self) -> list:
        """Output constraints (output, sign, threshold, eta): c = sign (y - threshold) <= 0."""
        return list(self.spec.constraints)

    @property
    def eta(self) -> Optional[torch.Tensor]:
        cs = self.spec.constraints
        if not cs:
            return None
        e = torch.tensor([c[3] for c in cs], dtype=torch.float64)
        return e[0] if len(set(c[3] for c in cs)) == 1 else e

    def _use_log_scan(self, tau_relu: float, tau_max: float):
        """Switch the scan to the log-space fat-smoothed HVI (qLogNEHVI / qLogEHVI): the
        q = 1 affine fast path runs hvi_log.hip (hvi_logk_kernel, log fatplus tabulated over the
        point table, over every compressed cell; the dense kernel over explicit ones, or with
        EVR_LOG=dense), every other case
        (output constraints, CloseToTarget / selected outputs, q > 1, qLogEHVI pending points)
        the general log scan (evr_qlog_eval), both over the explicit cell bounds (compressed
        cells are expanded once, on the device)."""
        if not (tau_relu > 0 and tau_max > 0):
            raise ValueError("tau_relu and tau_max must be positive")
        lo, hi = self.cells.explicit()

        def logify(src):
            st = _native.EvrQnehviState.from_buffer_copy(src)
            st.cell_lo, st.cell_hi = lo.data_ptr(), hi.data_ptr()
            # compressed cells stay: the q = 1 scan tabulates log fatplus over the point table
            # and visits every compressed cell (hvi_logk_kernel; the fat-smoothed terms have no
            # sparsity to skip); the general log scan reads the explicit rows
            st.log_hvi, st.tau_relu, st.tau_max = 1, float(tau_relu), float(tau_max)
            return st
        self._log_cells = (lo, hi)
        self.state_scan = logify(self.state_scan)
        self.state = logify(self.state)
        if self.spec.affine_identity:
            self.state_model = self.state
        self.tau_relu, self.tau_max = float(tau_relu), float(tau_max)
        self.log_acqf = True      # may be negative: optimize_acqf uses initialize_q_batch
        self._plans = {}

    @property
    def supports_plan(self) -> bool:
        """q = 1 candidates through the fused fast path (native plan / hipGraph): every
        output carries one affine objective, there are no output constraints, and no pending
        points join the candidates' joint batch (qEHVI / qEI X_pending; qNEHVI folds its
        pending points into the baseline, so its plan sees them)."""
        return self.spec.affine_identity and self._pending_rows() is None

    def _init_general(self, spec: ops.GeneralSpec, cells, nk: int, nb_rows: int, no_h: bool = False):
        """States of the general evaluation (qnehvi_general.hip): model side over the m
        outputs, scan side over the m_obj objectives and the cells."""
        gp, m = self.gp, self.m
        self.spec = spec
        self._zq_cache = {}
        if spec.affine_identity:
            self.state_model = self.state_scan = self.state
        else:
            ones = torch.ones(max(m, spec.m_obj), dtype=torch.float64, device=self.dev)
            self._dummy = (ones, torch.zeros_like(ones))
            self.state_model = ops.make_state(nk, nb_rows, self.S, m, gp.const, gp.ym, gp.ys, gp.kxx, self.zq,
                                              ones, ones, cells, no_h=no_h)
            self.state_scan = ops.make_state(nk, nb_rows, self.S, spec.m_obj, ones, ones, ones, ones, self.zq,
                                             ones, ones, cells, no_h=no_h)

    def _zq(self, q: int) -> torch.Tensor:
        """S x q x m base samples of q new points (cached per q)."""
        z = self._zq_cache.get(q)
        if z is None:
            z = self._draw_zq(q).to(dtype=torch.float64, device=self.dev).reshape(self.S, q, self.m).contiguous()
            self._zq_cache[q] = z
        return z

    def set_new_point_samples(self, q: int, z: torch.Tensor):
        """Inject the S x q x m base samples of q new points (parity tests)."""
        self._zq_cache[int(q)] = z.to(dtype=torch.float64, device=self.dev).reshape(self.S, q, self.m).contiguous()

    def _pending_rows(self) -> Optional[torch.Tensor]:
        return None

    def _general(self, X: torch.Tensor, backward: bool, gout: Optional[torch.Tensor] = None):
        """X: b x q x d -> (acq (b), dX b x q x d | None) through evr_qng_eval; fixed pending
        points (qEHVI) join every candidate's joint batch."""
        b, q, d = X.shape
        Xp = self._pending_rows()
        qq = q
        if Xp is not None:
            X = torch.cat([X, Xp.unsqueeze(0).expand(b, Xp.shape[0], d)], 1)
            qq = X.shape[1]
        if qq > ops.QNG_MAX_Q:
            raise ValueError(f"joint batch of {qq} points (q + pending) exceeds the device limit of {ops.QNG_MAX_Q} "
                             f"(the inclusion-exclusion runs over all 2^q - 1 subsets)")
        g = self.spec.struct(qq, self._zq(qq))
        ev = ops.qlog_eval if getattr(self, "log_acqf", False) else ops.qng_eval
        acq, dX = ev(self.state_model, self.state_scan, g, self.model, X.reshape(b * qq, d).contiguous(),
                     backward, gout)
        if dX is not None:
            dX = dX.view(b, qq, d)[:, :q].contiguous()
        return acq, dX

    def _device_tensors(self):
        """Every device tensor the acquisition (and its model and cells) holds: the state /
        model structs point into these, so the torch-side acquisition object keeps them alive."""
        out, seen = [], set()

        def walk(v, depth=0):
            if isinstance(v, torch.Tensor):
                if v.device.type == "cuda" and id(v) not in seen:
                    seen.add(id(v))
                    out.append(v)
            elif depth >= 4 or id(v) in seen:
                return
            elif isinstance(v, (list, tuple)):
                for x in v:
                    walk(x, depth + 1)
            elif isinstance(v, dict):
                for x in v.values():
                    walk(x, depth + 1)
            elif type(v).__module__.startswith("everest_amd") and hasattr(v, "__dict__"):
                # the package's own holders (Cells, KdGroups, GPBatch, ...): their tensors are
                # what the state's cell / group pointers refer to
                seen.add(id(v))
                for k, x in vars(v).items():
                    if k not in ("_torch_acqs", "_plans"):
                        walk(x, depth + 1)
        walk(self)
        return out

    def _torch_acq(self, q: int, fast: bool):
        """The torch.classes.everest_amd.QnehviAcq behind torch.ops.everest_amd.qnehvi_*
        (torch_ops.cpp): owns copies of the state / model structs, references to every device
        tensor they point into, and a plan cache across calls (cached here per path)."""
        from . import torch_ops

        torch_ops.load()
        cache = self.__dict__.setdefault("_torch_acqs", {})
        acq = cache.get(fast)
        if acq is None:
            def raw(st):
                return torch.frombuffer(bytearray(bytes(st)), dtype=torch.uint8)
            stm = self.state if fast else self.state_model
            sth = self.state if fast else self.state_scan
            acq = torch.classes.everest_amd.QnehviAcq(raw(stm), raw(sth), raw(self.model), bool(fast),
                                                      bool(getattr(self, "log_acqf", False)), self._device_tensors())
            cache[fast] = acq
        done = self.__dict__.setdefault("_torch_general_q", set())
        if not fast and q not in done:
            spec = self.spec
            oo, ok, p0, p1 = spec._arrs
            cons = spec.constraints
            co = torch.tensor([c[0] for c in cons], dtype=torch.int32)
            cs, ct, ce = (torch.tensor([c[k] for c in cons], dtype=torch.float64) for k in (1, 2, 3))
            acq.set_general(int(q), torch.from_numpy(oo), torch.from_numpy(ok), torch.from_numpy(p0),
                            torch.from_numpy(p1), co, cs, ct, ce, self._zq(q))
            done.add(q)
        return acq

    def __call__(self, X: torch.Tensor) -> torch.Tensor:
        """BoTorch AcquisitionFunction protocol: X (b x q x d, or b x d for q = 1) -> acq (b),
        differentiable through the device backward — torch.ops.everest_amd.qnehvi_forward /
        qnehvi_backward in a torch.autograd.Function (torch_ops.QnehviFunction)."""
        from .torch_ops import QnehviFunction

        X3, _ = self._split(X)
        if self._fast(X3):
            return QnehviFunction.apply(X3[:, 0].contiguous(), self._torch_acq(1, True))
        Xp = self._pending_rows()
        if Xp is not None:
            X3 = torch.cat([X3, Xp.unsqueeze(0).expand(X3.shape[0], Xp.shape[0], X3.shape[2])], 1)
        if X3.shape[1] > ops.QNG_MAX_Q:
            raise ValueError(f"joint batch of {X3.shape[1]} points (q + pending) exceeds the device limit of "
                             f"{ops.QNG_MAX_Q} (the inclusion-exclusion runs over all 2^q - 1 subsets)")
        return QnehviFunction.apply(X3.contiguous(), self._torch_acq(X3.shape[1], False))

    def _split(self, X: torch.Tensor):
        """(X as b x q x d, squeeze-back flag): 2-D input is q = 1."""
        X = X.to(device=self.dev, dtype=torch.float64)
        if X.dim() == 2:
            return X.unsqueeze(1), True
        if X.dim() != 3:
            raise ValueError(f"candidates must be b x d or b x q x d, got {tuple(X.shape)}")
        return X, False

    def _fast(self, X3: torch.Tensor) -> bool:
        return X3.shape[1] == 1 and self.supports_plan and self._pending_rows() is None

    def plan(self, b: int, backward: bool) -> ops.QnehviPlan:
        """Native evaluation plan for batch size b (cached; hipGraph unless EVR_GRAPH=0)."""
        if not self.supports_plan:
            raise NotImplementedError("the native plan covers q = 1 with affine objectives on every output")
        key = (int(b), bool(backward))
        p = self._plans.get(key)
        if p is None:
            if len(self._plans) >= 8:
                self._plans.pop(next(iter(self._plans)))
            p = ops.QnehviPlan(self.state, self.model, int(b), bool(backward), self.dev,
                               graph=os.environ.get("EVR_GRAPH", "1") != "0")
            self._plans[key] = p
        return p

    def forward(self, X: torch.Tensor, return_cache: bool = False):
        """X: b x d (q = 1) or b x q x d raw (transformed) candidates on device ->
        acquisition values (b).  q = 1 with affine objectives runs the native plan (one C-ABI
        call; see forward_ops for the op-by-op chain), everything else the general kernels."""
        if return_cache:
            return self.forward_ops(X, return_cache=True)
        X3, _ = self._split(X)
        if not self._fast(X3):
            return self._general(X3, False)[0]
        p = self.plan(X3.shape[0], False)
        p.X.copy_(X3[:, 0])
        p.run()
        return p.acq.clone()

    def forward_backward(self, X: torch.Tensor, gout: Optional[torch.Tensor] = None):
        """Returns (acq (b), d sum_c gout_c acq_c / dX (shaped like X))."""
        X3, flat = self._split(X)
        if not self._fast(X3):
            acq, dX = self._general(X3, True, gout)
            return acq, (dX[:, 0] if flat else dX)
        if gout is not None:
            acq, dX = self.forward_backward_ops(X3[:, 0], gout)
            return acq, (dX if flat else dX.unsqueeze(1))
        p = self.plan(X3.shape[0], True)
        p.X.copy_(X3[:, 0])
        p.run()
        return p.acq.clone(), (p.dX.clone() if flat else p.dX.clone().unsqueeze(1))

    def eval_host(self, x: np.ndarray, backward: bool):
        """Host round trip for the scipy optimiser: x (b x d or b x q x d numpy) -> (acq,
        dX or None) numpy; q = 1 fast path: one evr_qnehvi_plan_eval_host (x and the results
        through pinned host memory inside the plan's host graph)."""
        b = x.shape[0]
        if x.ndim == 2 and self.supports_plan and self._pending_rows() is None:
            out = self.plan(b, backward).run_host(x)
            acq = out[:b].copy()
            return acq, (out[b:].reshape(b, -1).copy() if backward else None)
        Xt = torch.as_tensor(x, dtype=torch.float64, device=self.dev)
        if backward:
            a, g = self.forward_backward(Xt)
            return a.cpu().numpy(), g.cpu().numpy()
        return self.forward(Xt).cpu().numpy(), None

    def _cross(self, X: torch.Tensor) -> torch.Tensor:
        """K(X_k, normalize(X)) : m x nk x b over the training (+ pending) rows."""
        gp = self.gp
        return ops.kernel_matrix(self.Xk, X, gp.ls, gp.kind, shift2=gp.lo, scale2=gp.inv_range)

    def forward_ops(self, X: torch.Tensor, return_cache: bool = False):
        """X: b x d raw (transformed) candidates on device -> acquisition values (b).

        A candidate whose new-point Cholesky block stays not p.d. after the 6-rung jitter
        ladder gets NaN (no device->host sync here); ``optim.host_values`` turns a NaN into
        the NotPSDError BoTorch raises from sample_cached_cholesky."""
        X = X.to(device=self.dev, dtype=torch.float64).contiguous()
        b = X.shape[0]
        Kx = self._cross(X)                         # m x nk x b
        R, P = ops.qnehvi_project(self.state, self.M, Kx, b)    # m x Rr x b + partial norms
        G, L22, flags = ops.qnehvi_samples_norms(self.state, R, P, b)
        acq = ops.hvi_forward(self.state, G, b, flags)
        if return_cache:
            return acq, (X, R, G, L22, flags)
        return acq

    def forward_backward_ops(self, X: torch.Tensor, gout: Optional[torch.Tensor] = None):
        """Op-by-op chain: returns (acq (b), d sum_c gout_c acq_c / dX (b x d))."""
        X = X.to(device=self.dev, dtype=torch.float64).contiguous()
        b = X.shape[0]
        Kx = self._cross(X)
        R, P = ops.qnehvi_project(self.state, self.M, Kx, b)
        G, L22, flags = ops.qnehvi_samples_norms(self.state, R, P, b)
        acq, dG = ops.hvi_forward_backward(self.state, G, b, flags, gout)
        dKx = ops.qnehvi_project_backward(self.state, self.M, R, L22, dG, b)    # m x nk x b
        gp = self.gp
        dX = ops.kernel_cross_grad(self.Xk, X, gp.ls, dKx, gp.kind, shift2=gp.lo, scale2=gp.inv_range)
        return acq, dX


class QNEHVI(_BoxHviAcqf):
    """Device qNEHVI over the GPs of ``gp`` (one output per objective).

    Parameters mirror the reference constructor: ``X_baseline`` raw (transformed) inputs,
    ``ref_point`` in objective space, affine objective ``g = a*y + b`` per output.  Base
    samples may be passed explicitly (parity tests) or are drawn from Sobol seeds.
    """

    def __init__(self, gp: GPBatch, X_train_raw: np.ndarray, X_baseline_raw: np.ndarray, ref_point, obj_a, obj_b,
                 S: int = 512, sampler_seed: int = 0, prune_baseline: bool = True, prune_seed: int = 0,
                 prune_samples: int = 2048, max_frac: float = 1.0, z_prune: Optional[torch.Tensor] = None,
                 z_base_full: Optional[torch.Tensor] = None, z_new_full: Optional[torch.Tensor] = None,
                 num_threads: Optional[int] = None, box_device: Optional[bool] = None,
                 kd_scan: Optional[bool] = None, X_pending_raw: Optional[np.ndarray] = None,
                 root: Optional[str] = None, objective=None, constraints=(), alpha: float = 0.0):
        dev = gp.device
        self.gp = gp
        self.dev = dev
        m = gp.B
        n = gp.n
        self.m, self.n, self.S = m, n, int(S)
        f64 = dict(dtype=torch.float64, device=dev)
        spec = _make_spec(m, obj_a, obj_b, objective, constraints)
        self.spec = spec
        self.ref = torch.as_tensor(np.asarray(ref_point, dtype=np.float64), **f64)
        if self.ref.numel() != spec.m_obj:
            raise ValueError(f"reference point has {self.ref.numel()} entries for {spec.m_obj} objectives")
        self.obj_a, self.obj_b = _fast_affine(spec, m, dev)
        self.sampler_seed = int(sampler_seed)
        self._z_new_full = z_new_full
        # baseline rows -> training rows (exact match of the transformed inputs)
        X_train_raw = np.asarray(X_train_raw, dtype=np.float64)
        X_baseline_raw = np.asarray(X_baseline_raw, dtype=np.float64)
        nbl = X_baseline_raw.shape[0]
        def _distinct_rows(a):
            a = np.ascontiguousarray(a)
            if not np.isfinite(a).all() or np.any((a == 0) & np.signbit(a)):   # byte != value equality
                return False
            return len(np.unique(a.view(np.dtype((np.void, a.dtype.itemsize * a.shape[1]))))) == a.shape[0]

        # a baseline point's row must be a training row of EVERY output (heterogeneous models:
        # the rows all outputs are trained on)
        all_rows = gp.valid_all_rows() if hasattr(gp, "valid_all_rows") else np.ones(X_train_raw.shape[0], bool)
        if (nbl <= X_train_raw.shape[0] and X_baseline_raw.ndim == 2 and X_baseline_raw.shape[1] > 0
                and np.array_equal(X_baseline_raw, X_train_raw[:nbl]) and _distinct_rows(X_baseline_raw)
                and all_rows[:nbl].all()):
            base_rows = np.arange(nbl, dtype=np.int64)   # the usual case: the deduplicated training rows
        else:
            first = {}
            for i, row in enumerate(map(tuple, X_train_raw)):
                if all_rows[i]:
                    first.setdefault(row, i)
            try:
                base_rows = np.array([first[tuple(r)] for r in X_baseline_raw], dtype=np.int64)
            except KeyError as e:
                raise ValueError("qNEHVI: every baseline point must be a training point of the models") from e

        # pending points ([upstream] set_X_pending with cache_pending=True, max_iep=0) join
        # the baseline after pruning: the kernel-vector row set grows to X_k = [X_train;
        # X_pending] (n_k = n + n_p rows), L^-1 / alpha are zero-padded over the pending
        # columns, and every formula below runs unchanged over n_k.
        npend = 0 if X_pending_raw is None else int(np.asarray(X_pending_raw).shape[0])
        self.n_pending = npend
        if npend > 0:
            Xp = torch.as_tensor(np.asarray(X_pending_raw, dtype=np.float64).reshape(npend, gp.d), **f64)
            self.Xk = torch.cat([gp.Xn, (Xp - gp.lo) * gp.inv_range], 0).contiguous()
        else:
            self.Xk = gp.Xn
        nk = n + npend
        self.nk = nk

        import time as _time
        tm = {}
        t0 = _time.perf_counter()
        _probe_on = os.environ.get("EVR_CONSTRUCTION_PROBES") == "1"   # diagnosis: synchronised split times
        _last = [t0]

        def probe(name):
            if _probe_on:
                torch.cuda.synchronize(dev)
                t = _time.perf_counter()
                tm["probe_" + name] = t - _last[0]
                _last[0] = t
        fut_prune = (_prefetch_scramble(len(base_rows) * m, prune_seed)
                     if prune_baseline and z_prune is None else None)
        # the sampler seed's raw stream covers the new-point and baseline draws of every
        # possible pruning outcome (draws of one seed are prefixes of one stream): start it now,
        # scramble the needed dimension ranges once the pruned baseline size is known
        max_dim = (len(base_rows) + npend + 1) * m
        def _stream_job(after=fut_prune if _host_threads() < 4 else None):
            # beside the prune draw's scrambling when the host has the threads for both (the
            # stream is one sequential mt19937 run; generated after the prune draw it held the
            # baseline draw — and the device — ~0.5 ms at the bench shape, profiles/r05/r)
            if after is not None:
                after.result()
            return ops.SobolStream(int(sampler_seed), max_dim)

        fut_stream = (_submit(_stream_job)
                      if max_dim <= ops.SOBOL_MAXDIM and (z_new_full is None or z_base_full is None) else None)
        # ---- joint posterior at the training (+ pending) inputs, shared by prune and baseline
        K = ops.kernel_matrix(self.Xk, self.Xk, gp.ls, gp.kind) if npend else gp.kernel_train(noise=False)
        Kt = K[:, :, :n].contiguous() if npend else K                      # m x nk x n
        mu_t = ops.gemm(Kt, gp.alpha.unsqueeze(-1))[..., 0]                # K alpha
        mu_train = gp.ym[:, None] + gp.ys[:, None] * (gp.const[:, None] + mu_t)
        A = ops.gemm(gp.Linv, K[:, :n].contiguous() if npend else K)      # L^-1 K  (m x n x nk)
        Sig = ops.gemm(A, A, transA=True, alpha=-1.0, beta=1.0, out=K)    # K - A^T A (in place)
        ops.scale_batched(Sig, (gp.ys ** 2).contiguous())                 # unstandardize
        probe("joint_posterior")

        # ---- prune_inferior_points_multi_objective --------------------------------------
        probs = None
        if prune_baseline:
            cand = torch.as_tensor(base_rows, device=dev)
            Sig_c = Sig[:, cand][:, :, cand].contiguous()
            mu_c = mu_train[:, cand].contiguous()
            nc = cand.shape[0]
            Lp, _, _ = ops.cholesky(Sig_c, 1e-8, 3)
            probe("prune_chol")
            if z_prune is None:
                Zp = sobol_base_samples(prune_samples, nc, m, prune_seed, dev, _result(fut_prune))  # m x nc x S'
            else:
                Zp = z_prune.to(dev).permute(2, 1, 0).contiguous()
            probe("prune_sobol")
            Yp = ops.gemm(Lp, Zp)
            Op = self._objective(Yp, mu_c)
            _, counts = ops.pareto_mask(Op, self.ref, dedup=False, want_mask=False, want_counts=True)
            probs = counts.cpu().numpy().astype(np.float64) / Zp.shape[2]
            tm["prune"] = _time.perf_counter() - t0
            keep = np.nonzero(probs)[0]
            max_points = math.ceil(max_frac * nc)
            if keep.shape[0] > max_points:
                order = np.argsort(-probs, kind="stable")
                keep = order[:max_points]
            keep = np.unique(keep)
            base_rows = base_rows[keep]
        nb_t = int(base_rows.shape[0])                 # pruned training baseline
        if npend:
            base_rows = np.concatenate([base_rows, n + np.arange(npend, dtype=np.int64)])
        nb = int(base_rows.shape[0])
        self.nb = nb
        self.base_rows = base_rows
        idx = torch.as_tensor(base_rows, device=dev)
        S_ = self.S
        if fut_stream is not None:
            fut_q = _prefetch_from_stream(fut_stream, (nb + 1) * m, nb * m, m) if z_new_full is None else None
            fut_b = (_prefetch_from_stream(fut_stream, nb_t * m)
                     if nb > 0 and nb_t > 0 and z_base_full is None else None)
        else:
            fut_q = _prefetch_scramble((nb + 1) * m, sampler_seed, nb * m, m) if z_new_full is None else None
            fut_b = _prefetch_scramble(nb_t * m, sampler_seed) if nb > 0 and z_base_full is None else None

        # ---- baseline posterior root, samples, box decomposition ----------------------
        if nb > 0:
            Sig_b = Sig[:, idx][:, :, idx].contiguous()
            self.L_base, self.base_jitter, _ = ops.cholesky(Sig_b, 1e-8, 3)
            mu_b = mu_train[:, idx].contiguous()
            probe("baseline_chol")
        # the new point's samples come from a (nb+1)*m-dimensional draw of the same seed;
        # pending rows from the (nb_t+n_p)*m-dimensional draw ([upstream] _update_base_samples
        # keeps the earlier rows of the base sampler, the same seed draws the new ones)
        if z_new_full is None:
            self.zq = ops.sobol_normal(S_, (nb + 1) * m, sampler_seed, dev, d0=nb * m, nd=m,
                                       scrambled=_result(fut_q))                           # S x m
        else:
            self.zq = z_new_full[:, nb, :].to(**f64).contiguous()
        if nb > 0:
            if z_base_full is None:
                Zb = sobol_base_samples(S_, nb_t, m, sampler_seed, dev, _result(fut_b))   # m x nb x S
                if npend:
                    Zp_ = ops.sobol_normal(S_, nb * m, sampler_seed, dev, d0=nb_t * m, nd=npend * m, layout=1, m=m)
                    Zb = torch.cat([Zb, Zp_], 1).contiguous()
            else:
                Zb = z_base_full.to(dev).permute(2, 1, 0).contiguous()
            self._Zb = Zb
            probe("baseline_sobol")
            Yb = ops.gemm(self.L_base, Zb)
            Ob = self._objective(Yb, mu_b)
            tm["baseline"] = _time.perf_counter() - t0 - tm.get("prune", 0.0)
            t1 = _time.perf_counter()
            # on a side stream: the operator below does not depend on the cells
            join_box = _decompose_async(Ob, self.ref, box_device, kd_scan, num_threads, alpha) \
                if not _probe_on else (lambda r: (lambda: r))(_decompose(Ob, self.ref, box_device, kd_scan,
                                                                         num_threads, alpha))
        else:  # no baseline: one cell [ref, inf)
            cells0 = _single_cell(self.ref, S_, spec.m_obj)
            join_box = lambda: (cells0, "none")  # noqa: E731
        probe("box")

        # ---- forward operator over the nk kernel rows -------------------------------------
        # "split" (default, the literal restatement): M = [Linv; G; H^T; alpha^T], L22^2 =
        #   s^2 (kxx - |Linv k|^2) - |G k|^2.  Each quadratic form keeps the size of its own
        #   result: Linv (entries <= 1 / sqrt(noise)) gives the O(1) vector Linv k, and G (entries
        #   up to ~5e5 at the bench state) gives the small vector G k (|G k|^2 ~ var ~ 1e-6), so
        #   their rounding stays below the cancellation L22^2 / (s^2 kxx) ~ 1e-7 .. 1e-11 that
        #   ordinary candidates reach at the bench state (tests/test_gpu_hp_truth.py: within
        #   ~2e-6 of the 60-digit truth, values and gradients).
        # "fused" (opt-in): the two quadratic forms share one root C with
        #   C^T C = Linv^T Linv + G^T G / s^2,  C = Lv^T Lp^-1,  Lv = chol(D0 + V^T V),
        #   V = (G / s) Lp,  Lp = diag(L, I_pending),  D0 = diag(1_n, 0_pending)
        # (I + V^T V >= I is well conditioned; no Gram matrix of Linv is ever formed), so
        # M = [C; H^T; alpha^T] has nk + S + 1 rows instead of nk + nb + S + 1 and the
        # samples / backward kernels see a baseline-free layout (state nb = 0).  C has entries
        # ~1e4 - 1e5 but |C k| ~ 1, so C k carries ~1e-10 absolute rounding: up to 100 % of
        # L22^2 at the bench state (HVI 5.6e-4 off the truth, gradients 2.6e-2; round 6).
        root = root or os.environ.get("EVR_ROOT", "split")
        if root not in ("fused", "split"):
            raise ValueError(f"root must be 'fused' or 'split', got {root!r}")
        fused = root == "fused" and nb > 0
        self.root = "fused" if fused else "split"
        nb_rows = 0 if fused else nb
        Rr = nk + nb_rows + S_ + 1
        self.Rr = Rr
        M = torch.zeros(m, Rr, nk, **f64) if npend else torch.empty(m, Rr, n, **f64)
        M[:, :n, :n].copy_(gp.Linv)
        if nb > 0:
            A_b = A[:, :, idx].contiguous()                                     # m x n x nb
            E = ops.gemm(A_b, gp.Linv, transA=True, alpha=-1.0)                 # -A_b^T Linv
            if npend:
                E = torch.cat([E, torch.zeros(m, nb, npend, **f64)], 2).contiguous()
            ops.add_selection(E, idx.to(torch.int32), None)                      # + P
            ops.scale_batched(E, (gp.ys ** 2).contiguous())                      # s^2 (...)
            # G = L_base^-1 E by forward substitution (an explicit inverse of the ill-conditioned
            # baseline root loses digits the near-training-point L22 cancellation exposes)
            ops.trsm(self.L_base, E)
            ops.gemm_into(M[:, nk + nb_rows:nk + nb_rows + S_], Zb, E, transA=True)   # H^T = Z^T G
            if fused:
                if npend:
                    Lp = torch.zeros(m, nk, nk, **f64)
                    Lp[:, :n, :n].copy_(gp.L)
                    Lpi = torch.zeros(m, nk, nk, **f64)
                    Lpi[:, :n, :n].copy_(gp.Linv)
                    Lp[:, n:, n:].copy_(torch.eye(npend, **f64))
                    Lpi[:, n:, n:].copy_(torch.eye(npend, **f64))
                else:   # Lp = L, Lp^-1 = L^-1 (no padded copies)
                    Lp, Lpi = gp.L, gp.Linv
                ops.scale_batched(E, (1.0 / gp.ys).contiguous())                 # G / s
                V = ops.gemm(E, Lp)                                              # nb x nk
                Iv = ops.gemm(V, V, transA=True)                                 # V^T V
                Iv.diagonal(dim1=-2, dim2=-1)[:, :n] += 1.0                      # + D0
                probe("root_gemms")
                Lv, _, _ = ops.cholesky(Iv, 1e-8, 3)
                probe("root_chol")
                ops.gemm_into(M[:, :nk], Lv, Lpi, transA=True)                   # C = Lv^T Lp^-1
            else:
                M[:, nk:nk + nb].copy_(E)
        else:
            M[:, nk:nk + S_].zero_()
        cells, self.box_path = join_box()
        if nb > 0:
            tm["box_decomposition"] = _time.perf_counter() - t1   # completion, overlapped with the operator
        self.cells = cells
        counts_c = cells.counts
        self.stats = ConstructionStats(n_train=n, n_base=nb, total_cells=int(np.sum(counts_c)),
                                       max_cells=int(counts_c.max()) if len(counts_c) else 0, prune_probs=probs)
        M[:, Rr - 1, :n].copy_(gp.alpha)
        self.M = M
        self.state = ops.make_state(nk, nb_rows, S_, m, gp.const, gp.ym, gp.ys, gp.kxx, self.zq, self.obj_a,
                                    self.obj_b, cells)
        self._keep = (self.zq, self.obj_a, self.obj_b)
        self._init_general(spec, cells, nk, nb_rows)
        if not spec.affine_identity:
            self.state = self.state_scan
        self._lo_c = gp.lo.to(torch.float64).contiguous()
        self._scale_c = gp.inv_range.to(torch.float64).contiguous()
        self.model = _native.EvrQnehviModel(n=nk, d=gp.d, kind=gp.kind, Xn=self.Xk.data_ptr(), lengthscales=gp.ls.data_ptr(),
                                            shift=self._lo_c.data_ptr(), scale=self._scale_c.data_ptr(),
                                            M=self.M.data_ptr())
        probe("operator")
        self._plans = {}
        torch.cuda.synchronize(dev)
        tm["total"] = _time.perf_counter() - t0
        self.timings = tm


    def z_base_host(self) -> Optional[torch.Tensor]:
        """The baseline base samples (S x nb x m, host), the oracle's layout; None without a
        baseline."""
        zb = getattr(self, "_Zb", None)
        return None if zb is None else zb.permute(2, 1, 0).cpu().contiguous()

    def _objective(self, Y: torch.Tensor, mu: torch.Tensor) -> torch.Tensor:
        """m x P x S model samples (+ mean) -> m_obj x P x S objectives; infeasible samples
        (output constraints) are set to the reference point."""
        if self.spec.affine_identity:
            return ops.objective_affine(Y, mu, self.obj_a, self.obj_b)
        return ops.objective_general(Y, mu, self.spec, self.ref)

    def _draw_zq(self, q: int) -> torch.Tensor:
        """New-point base samples of a q-batch: rows nb .. nb+q-1 of the (nb+q)*m-dim draw of
        the sampler seed ([upstream] _update_base_samples keeps the baseline rows)."""
        nb, m = self.nb, self.m
        if self._z_new_full is not None:
            if self._z_new_full.shape[1] < nb + q:
                raise ValueError(f"z_new_full has {self._z_new_full.shape[1]} rows, need {nb + q}")
            return self._z_new_full[:, nb:nb + q, :]
        return ops.sobol_normal(self.S, (nb + q) * m, self.sampler_seed, self.dev, d0=nb * m, nd=q * m)


class QEHVI(_BoxHviAcqf):
    """Device qEHVI (q = 1) — [upstream] ``qExpectedHypervolumeImprovement`` as built by
    ``QehviStrategy._get_acqfs`` (bofire/strategies/predictives/qehvi.py:37-79:
    NondominatedPartitioning of the observed objectives better than the reference point)
    and by ``get_acquisition_function("qEHVI")`` from ``MoboStrategy._get_acqfs``
    (bofire/strategies/predictives/mobo.py:44-90: FastNondominatedPartitioning of the
    objective-transformed observations).  Both partitions are exact (alpha = 0), so the
    cells cover the same region and the HVI values agree.

    Unlike qNEHVI the cells are fixed (one partition of ``Y_part`` shared by all samples) and
    the samples are independent per output: y_s = mu(x) + sqrt(var(x)) z_s, z_s the s-th
    row of an m-dimensional Sobol-normal draw (the 1x1 posterior root with the same
    jitter ladder).  The device layout is the qNEHVI one with nb = 0 and no H^T rows
    (M = [L^-1; alpha^T], state.no_h = 1): one (n + 1)-row projection GEMM, the same
    sampling, sparse-scan and backward kernels."""

    def __init__(self, gp: GPBatch, Y_part: np.ndarray, ref_point, obj_a, obj_b, S: int = 512,
                 sampler_seed: int = 0, z: Optional[torch.Tensor] = None, box_device: Optional[bool] = None,
                 kd_scan: Optional[bool] = None, num_threads: Optional[int] = None, objective=None,
                 constraints=(), X_pending_raw: Optional[np.ndarray] = None, alpha: float = 0.0):
        """Y_part: points of the partition in objective space (m_obj columns); pending
        points ([upstream] concatenate_pending_points) join every candidate's joint batch;
        alpha > 0: [upstream] NondominatedPartitioning(alpha) instead of the exact partition."""
        dev = gp.device
        self.gp, self.dev = gp, dev
        m, n = gp.B, gp.n
        self.m, self.n, self.S, self.nb, self.nk = m, n, int(S), 0, n
        f64 = dict(dtype=torch.float64, device=dev)
        spec = _make_spec(m, obj_a, obj_b, objective, constraints)
        self.spec = spec
        mo = spec.m_obj
        self.ref = torch.as_tensor(np.asarray(ref_point, dtype=np.float64), **f64)
        if self.ref.numel() != mo:
            raise ValueError(f"reference point has {self.ref.numel()} entries for {mo} objectives")
        self.obj_a, self.obj_b = _fast_affine(spec, m, dev)
        self.sampler_seed = int(sampler_seed)
        Y_part = np.asarray(Y_part, dtype=np.float64).reshape(-1, mo)
        self.Y_part = Y_part
        self.Xk = gp.Xn
        S_ = self.S
        if Y_part.shape[0] > 0:
            O = torch.as_tensor(np.ascontiguousarray(Y_part.T), **f64)[:, :, None].expand(mo, Y_part.shape[0], S_)
            cells, self.box_path = _decompose(O.contiguous(), self.ref, box_device, kd_scan, num_threads, alpha)
        else:
            cells, self.box_path = _single_cell(self.ref, S_, mo), "none"
        self.cells = cells
        cnt = cells.counts
        self.stats = ConstructionStats(n_train=n, n_base=0, total_cells=int(np.sum(cnt)),
                                       max_cells=int(cnt.max()) if len(cnt) else 0)
        self._z1 = z
        if z is None:
            self.zq = ops.sobol_normal(S_, m, sampler_seed, dev)                  # S x m
        else:
            self.zq = z.reshape(S_, m).to(**f64).contiguous()
        self.X_pending = None
        if X_pending_raw is not None and np.asarray(X_pending_raw).shape[0] > 0:
            self.X_pending = torch.as_tensor(np.asarray(X_pending_raw, dtype=np.float64).reshape(-1, gp.d), **f64)
        self.Rr = n + 1
        M = torch.empty(m, n + 1, n, **f64)
        M[:, :n].copy_(gp.Linv)
        M[:, n].copy_(gp.alpha)
        self.M = M
        self.state = ops.make_state(n, 0, S_, m, gp.const, gp.ym, gp.ys, gp.kxx, self.zq, self.obj_a, self.obj_b,
                                    cells, no_h=True)
        self._lo_c = gp.lo.to(torch.float64).contiguous()
        self._scale_c = gp.inv_range.to(torch.float64).contiguous()
        self.model = _native.EvrQnehviModel(n=n, d=gp.d, kind=gp.kind, Xn=self.Xk.data_ptr(),
                                            lengthscales=gp.ls.data_ptr(), shift=self._lo_c.data_ptr(),
                                            scale=self._scale_c.data_ptr(), M=self.M.data_ptr())
        self._plans = {}
        self._init_general(spec, cells, n, 0, no_h=True)
        if not spec.affine_identity:
            self.state = self.state_scan
        torch.cuda.synchronize(dev)

    def _pending_rows(self) -> Optional[torch.Tensor]:
        return self.X_pending

    def _draw_zq(self, q: int) -> torch.Tensor:
        """S x (q*m) Sobol-normal draw of the joint batch (Sobol dim = point*m + output)."""
        if q == 1 and self._z1 is not None:
            return self.zq
        return ops.sobol_normal(self.S, q * self.m, self.sampler_seed, self.dev)


TAU_RELU = 1e-6     # [upstream] botorch.acquisition.logei.TAU_RELU
TAU_MAX_MO = 1e-3   # [upstream] qLogExpectedHypervolumeImprovement default tau_max


class QLogNEHVI(QNEHVI):
    """Device qLogNEHVI (q = 1, fat = True) — [upstream] qLogNoisyExpectedHypervolumeImprovement,
    MoboStrategy's default acquisition (bofire/data_models/strategies/predictives/mobo.py:27-29,
    built at bofire/strategies/predictives/mobo.py:68-90).  Same construction, operator and
    samples as QNEHVI; the scan is the dense log-space one (hvi_log.hip):
    acq = logmeanexp_s logsumexp_cells sum_j fatmin(log fatplus(y_j - l_j; tau_relu),
    log(min(u_j, 1e10) - l_j); tau_max)."""

    def __init__(self, *args, tau_relu: float = TAU_RELU, tau_max: float = TAU_MAX_MO, **kw):
        super().__init__(*args, **kw)
        self._use_log_scan(tau_relu, tau_max)


class QLogEHVI(QEHVI):
    """Device qLogEHVI (q = 1, fat = True) — [upstream] qLogExpectedHypervolumeImprovement as
    built by get_acquisition_function("qLogEHVI") in MoboStrategy: the qEHVI partition and
    samples with the log-space scan."""

    def __init__(self, *args, tau_relu: float = TAU_RELU, tau_max: float = TAU_MAX_MO, **kw):
        super().__init__(*args, **kw)
        self._use_log_scan(tau_relu, tau_max)


class QEIJoint(QEHVI):
    """Device qEI over joint batches — q > 1 candidates and/or pending points ([upstream]
    qExpectedImprovement with X_pending, bofire/strategies/predictives/sobo.py:51-90;
    optimize_acqf(q=...) at botorch.py:385).  With one objective, the region above any
    reference r < best_f not dominated by best_f is the single cell [best_f, inf), and the
    hypervolume improvement of q samples over it is max_i (g(y_i) - best_f)_+ — exactly qEI's
    integrand.  So the joint posterior of the q (+ pending) points, its psd_safe q x q root,
    the subset scan and their analytic backward are the general qEHVI kernels at m = 1
    (``qg_*``), with best_f = max over X_train of g(posterior mean) as in QEI and the
    S x (q + n_pending) Sobol-normal draw of the sampler seed."""

    def __init__(self, gp: GPBatch, X_train_raw: np.ndarray, obj_a: float, obj_b: float, S: int = 512,
                 seed: int = 0, X_pending_raw: Optional[np.ndarray] = None):
        if gp.B != 1:
            raise ValueError("QEIJoint takes a single-output model")
        Xt = torch.as_tensor(np.asarray(X_train_raw, dtype=np.float64), device=gp.device)
        mean, _ = gp.posterior(Xt)
        best_f = float((float(obj_a) * mean[0] + float(obj_b)).max().item())
        super().__init__(gp, np.array([[best_f]]), [best_f - 1.0], [float(obj_a)], [float(obj_b)], S=S,
                         sampler_seed=seed, box_device=False, X_pending_raw=X_pending_raw)
        self.best_f = best_f
        self.a, self.b = float(obj_a), float(obj_b)


class QEI:
    """Device qEI (q = 1, one output) — [upstream] qExpectedImprovement as built by
    ``get_acquisition_function("qEI", ...)`` from SoboStrategy._get_acqfs
    (bofire/strategies/predictives/sobo.py:51-90): best_f = max over X_train of g(posterior
    mean), plain MC sampling with S Sobol-normal base samples."""

    def __init__(self, gp: GPBatch, X_train_raw: np.ndarray, obj_a: float, obj_b: float, S: int = 512,
                 seed: int = 0, z: Optional[torch.Tensor] = None):
        if gp.B != 1:
            raise ValueError("QEI takes a single-output model")
        self.gp = gp
        self.dev = gp.device
        self.a, self.b = float(obj_a), float(obj_b)
        Xt = torch.as_tensor(np.asarray(X_train_raw, dtype=np.float64), device=self.dev)
        mean, _ = gp.posterior(Xt)
        self.best_f = float((self.a * mean[0] + self.b).max().item())
        if z is None:
            z = ops.sobol_normal(S, 1, seed, self.dev)
        self.z = z.reshape(-1).to(device=self.dev, dtype=torch.float64).contiguous()
        h = gp.hypers[0]
        self._scal = (h.constant, h.y_mean, h.y_std, 1.0)

    def _run(self, X, with_grad):
        X = X.to(device=self.dev, dtype=torch.float64).contiguous()
        R = ops.gemm(self.gp.M, self.gp.cross(X))[0]          # (n+1) x b
        acq, gR, flags = ops.qei(R, *self._scal, self.z, self.a, self.b, self.best_f, with_grad)
        # NaN marks a candidate whose variance stayed not p.d. after the jitter ladder; no host
        # sync here — optim.host_values raises NotPSDError after the (all-)gather, so every
        # rank of a sharded evaluation raises together (as QNEHVI does)
        acq = torch.where(flags != 0, torch.full_like(acq, math.nan), acq)
        return X, acq, gR

    def forward(self, X: torch.Tensor) -> torch.Tensor:
        return self._run(X, False)[1]

    def forward_backward(self, X: torch.Tensor, gout: Optional[torch.Tensor] = None):
        X, acq, gR = self._run(X, True)
        if gout is not None:
            gR = gR * gout.unsqueeze(0)
        gp = self.gp
        dK = ops.gemm(gp.M, gR.unsqueeze(0), transA=True)      # 1 x n x b
        dX = ops.kernel_cross_grad(gp.Xn, X, gp.ls, dK, gp.kind, shift2=gp.lo, scale2=gp.inv_range)
        return acq, dX
