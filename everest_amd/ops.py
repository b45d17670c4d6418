"""Torch-tensor level wrappers over the C-ABI (include/everest_amd.h).

Every op runs on torch's *current* HIP stream, takes float64 device tensors, allocates
its outputs with the torch caching allocator and never frees caller memory.  Shape,
dtype and device errors raise (``ValueError`` / ``RuntimeError``); there is no CPU path.
The posterior, kernel matrix, Cholesky and qNEHVI entry points are also registered as PyTorch
custom operators (``torch.ops.everest_amd.*``, everest_amd/csrc/torch_ops.cpp, everest_amd/torch_ops.py).
"""
from __future__ import annotations

import ctypes
import os
import warnings
from typing import Optional, Tuple

import numpy as np
import torch

from . import _native
from ._native import EvrQnehviState, EvrQnGeneral, call

KERNELS = {"rbf": 0, "matern05": 1, "matern15": 2, "matern25": 3}
KIND_BY_NU = {0.5: 1, 1.5: 2, 2.5: 3}


class NotPSDError(RuntimeError):
    """Raised when the jitter ladder of psd_safe_cholesky is exhausted ([upstream]
    linear_operator NotPSDError, caught by fit_gpytorch_mll's retries)."""


# joint batch limit of the general q-point kernels (include/everest_amd.h EVR_QNG_MAX_Q): the
# [upstream] inclusion-exclusion enumerates all 2^q - 1 subsets of the q (+ pending) points
QNG_MAX_Q = 12

def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _dev(t: torch.Tensor, name: str, dtype=torch.float64) -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor")
    if t.device.type != "cuda":
        raise RuntimeError(f"{name}: everest_amd ops run on the MI355X only (got device {t.device}); "
                           "there is no CPU fallback")
    if t.dtype != dtype:
        raise ValueError(f"{name}: expected {dtype}, got {t.dtype}")
    return t.contiguous()


def _p(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


# ---------------------------------------------------------------------------------------
# kernel matrices
# ---------------------------------------------------------------------------------------
def kernel_matrix(X1, X2, lengthscales, kind: int = 0, shift1=None, scale1=None, shift2=None, scale2=None,
                  outputscale=None, diag_add=None) -> torch.Tensor:
    """K[b] = os_b * k(norm(X1), norm(X2); ls_b) (+ diag_add_b on i==j).  ls: B x d."""
    X1 = _dev(X1, "X1")
    X2 = _dev(X2, "X2")
    ls = _dev(lengthscales, "lengthscales")
    if ls.dim() == 1:
        ls = ls.unsqueeze(0)
    B, d = ls.shape
    if X1.shape[-1] != d or X2.shape[-1] != d:
        raise ValueError(f"kernel_matrix: dims mismatch X1 {tuple(X1.shape)} X2 {tuple(X2.shape)} ls {tuple(ls.shape)}")
    n1, n2 = X1.shape[0], X2.shape[0]
    K = torch.empty(B, n1, n2, dtype=torch.float64, device=X1.device)
    opt = [None if t is None else _dev(t, "aux") for t in (shift1, scale1, shift2, scale2, outputscale, diag_add)]
    call("evr_kernel_matrix", _stream(), int(kind), B, n1, n2, d, X1.data_ptr(), _p(opt[0]), _p(opt[1]),
         X2.data_ptr(), _p(opt[2]), _p(opt[3]), ls.data_ptr(), _p(opt[4]), _p(opt[5]), K.data_ptr())
    return K


def _workspace(ndoubles: int, device) -> torch.Tensor:
    """Scratch for a native op (torch caching allocator; no device-side malloc)."""
    return torch.empty(max(int(ndoubles), 1), dtype=torch.float64, device=device)


def kernel_cross_grad(X1, X2, lengthscales, G, kind=0, shift1=None, scale1=None, shift2=None, scale2=None,
                      outputscale=None) -> torch.Tensor:
    X1, X2, ls, G = _dev(X1, "X1"), _dev(X2, "X2"), _dev(lengthscales, "ls"), _dev(G, "G")
    B, d = ls.shape
    n1, n2 = X1.shape[0], X2.shape[0]
    if tuple(G.shape) != (B, n1, n2):
        raise ValueError(f"kernel_cross_grad: G shape {tuple(G.shape)} != {(B, n1, n2)}")
    dX = torch.empty(n2, d, dtype=torch.float64, device=X1.device)
    opt = [None if t is None else _dev(t, "aux") for t in (shift1, scale1, shift2, scale2, outputscale)]
    work = _workspace(_native.load().evr_kernel_cross_grad_workspace_doubles(n1, n2, d), X1.device)
    call("evr_kernel_cross_grad", _stream(), int(kind), B, n1, n2, d, X1.data_ptr(), _p(opt[0]), _p(opt[1]),
         X2.data_ptr(), _p(opt[2]), _p(opt[3]), ls.data_ptr(), _p(opt[4]), G.data_ptr(), dX.data_ptr(),
         work.data_ptr())
    return dX


def kernel_lengthscale_grad(X, lengthscales, W, kind=0) -> torch.Tensor:
    X, ls, W = _dev(X, "X"), _dev(lengthscales, "ls"), _dev(W, "W")
    B, d = ls.shape
    n = X.shape[0]
    g = torch.empty(B, d, dtype=torch.float64, device=X.device)
    work = torch.empty(B, n, d, dtype=torch.float64, device=X.device)
    call("evr_kernel_lengthscale_grad", _stream(), int(kind), B, n, d, X.data_ptr(), ls.data_ptr(), W.data_ptr(),
         g.data_ptr(), work.data_ptr())
    return g


def mll_terms(L, Linv, r, alpha) -> torch.Tensor:
    """B x 5: logdet, quad, tr(K^-1), sum(alpha), sum(alpha^2)."""
    L, Linv, r, alpha = _dev(L, "L"), _dev(Linv, "Linv"), _dev(r, "r"), _dev(alpha, "alpha")
    B, n, _ = L.shape
    out = torch.empty(B, 5, dtype=torch.float64, device=L.device)
    call("evr_gp_mll_terms", _stream(), B, n, L.data_ptr(), Linv.data_ptr(), r.data_ptr(), alpha.data_ptr(),
         out.data_ptr())
    return out


# ---------------------------------------------------------------------------------------
# dense linear algebra
# ---------------------------------------------------------------------------------------
def gemm(A, B, transA=False, transB=False, alpha=1.0, beta=0.0, out=None) -> torch.Tensor:
    """Batched C = alpha op(A) op(B) + beta C on the f64 MFMA kernel.  A, B: (batch) x r x c."""
    A, B = _dev(A, "A"), _dev(B, "B")
    a3, b3 = A.dim() == 3, B.dim() == 3
    if A.dim() == 2:
        A = A.unsqueeze(0)
    if B.dim() == 2:
        B = B.unsqueeze(0)
    batch = max(A.shape[0], B.shape[0])
    if A.shape[0] not in (1, batch) or B.shape[0] not in (1, batch):
        raise ValueError("gemm: batch mismatch")
    M, K = (A.shape[2], A.shape[1]) if transA else (A.shape[1], A.shape[2])
    K2, N = (B.shape[2], B.shape[1]) if transB else (B.shape[1], B.shape[2])
    if K != K2:
        raise ValueError(f"gemm: inner dims {K} != {K2}")
    if out is None:  # beta = 0: the kernel never reads C
        out = torch.empty(batch, M, N, dtype=torch.float64, device=A.device)
        beta = 0.0
    else:
        if out.dim() == 2:
            out = out.unsqueeze(0)
        if tuple(out.shape) != (batch, M, N) or not out.is_contiguous():
            raise ValueError("gemm: bad out tensor")
    sA = 0 if A.shape[0] == 1 else A.shape[1] * A.shape[2]
    sB = 0 if B.shape[0] == 1 else B.shape[1] * B.shape[2]
    call("evr_gemm_f64", _stream(), int(transA), int(transB), M, N, K, float(alpha), A.data_ptr(), A.shape[2], sA,
         B.data_ptr(), B.shape[2], sB, float(beta), out.data_ptr(), N, M * N, batch)
    return out if (a3 or b3) else out[0]


def gemm_into(out_view: torch.Tensor, A, B, transA=False, transB=False, alpha=1.0, beta=0.0, batch_strides=None):
    """GEMM writing into a strided 2-D/3-D row block (rows contiguous with leading dim ld)."""
    A, B = _dev(A, "A"), _dev(B, "B")
    if A.dim() == 2:
        A = A.unsqueeze(0)
    if B.dim() == 2:
        B = B.unsqueeze(0)
    o = out_view if out_view.dim() == 3 else out_view.unsqueeze(0)
    batch = o.shape[0]
    M, K = (A.shape[2], A.shape[1]) if transA else (A.shape[1], A.shape[2])
    K2, N = (B.shape[2], B.shape[1]) if transB else (B.shape[1], B.shape[2])
    if K != K2 or o.shape[1] != M or o.shape[2] != N or o.stride(2) != 1:
        raise ValueError("gemm_into: shape mismatch")
    sA = 0 if A.shape[0] == 1 else A.stride(0)
    sB = 0 if B.shape[0] == 1 else B.stride(0)
    call("evr_gemm_f64", _stream(), int(transA), int(transB), M, N, K, float(alpha), A.data_ptr(), A.stride(1), sA,
         B.data_ptr(), B.stride(1), sB, float(beta), o.data_ptr(), o.stride(1), o.stride(0), batch)


def cholesky(A: torch.Tensor, jitter0: float = 1e-8, max_tries: int = 3, raise_on_fail: bool = True):
    """psd_safe_cholesky on a batch (B x n x n).  Returns (L, jitter_used[B], info[B])."""
    A = _dev(A, "A")
    squeeze = A.dim() == 2
    if squeeze:
        A = A.unsqueeze(0)
    B, n, n2 = A.shape
    if n != n2:
        raise ValueError("cholesky: matrix not square")
    L = torch.empty_like(A)
    jit = torch.empty(B, dtype=torch.float64, device=A.device)
    info = torch.empty(B, dtype=torch.int32, device=A.device)
    call("evr_cholesky", _stream(), B, n, A.data_ptr(), n, n * n, L.data_ptr(), n, n * n, float(jitter0),
         int(max_tries), jit.data_ptr(), info.data_ptr())
    if raise_on_fail:
        bad = info.cpu()
        if bool(bad.any()):
            raise NotPSDError(f"Matrix not positive definite after repeatedly adding jitter up to "
                              f"{jitter0 * 10 ** (max_tries - 1):.1e} (batch members {bad.nonzero().view(-1).tolist()})")
    if squeeze:
        return L[0], jit[0], info[0]
    return L, jit, info


def cholesky_inverse(A: torch.Tensor, jitter0: float = 1e-8, max_tries: int = 3, raise_on_fail: bool = True):
    """(L, L^-1, jitter_used, info) from one blocked pass (psd_safe_cholesky semantics)."""
    A = _dev(A, "A")
    squeeze = A.dim() == 2
    if squeeze:
        A = A.unsqueeze(0)
    B, n, n2 = A.shape
    if n != n2:
        raise ValueError("cholesky_inverse: matrix not square")
    L = torch.empty_like(A)
    Li = torch.empty_like(A)
    jit = torch.empty(B, dtype=torch.float64, device=A.device)
    info = torch.empty(B, dtype=torch.int32, device=A.device)
    call("evr_cholesky_inverse", _stream(), B, n, A.data_ptr(), n, n * n, L.data_ptr(), n, n * n, Li.data_ptr(), n,
         n * n, float(jitter0), int(max_tries), jit.data_ptr(), info.data_ptr())
    if raise_on_fail:
        bad = info.cpu()
        if bool(bad.any()):
            raise NotPSDError(f"Matrix not positive definite after repeatedly adding jitter up to "
                              f"{jitter0 * 10 ** (max_tries - 1):.1e} (batch members {bad.nonzero().view(-1).tolist()})")
    if squeeze:
        return L[0], Li[0], jit[0], info[0]
    return L, Li, jit, info


def trsm(L: torch.Tensor, B: torch.Tensor, transpose: bool = False) -> torch.Tensor:
    """In place: B <- L^-1 B (or L^-T B).  L: (batch) x n x n, B: (batch) x n x nrhs."""
    L = _dev(L, "L")
    if not B.is_contiguous() or B.dtype != torch.float64 or B.device.type != "cuda":
        raise ValueError("trsm: B must be a contiguous float64 device tensor (solved in place)")
    L3 = L if L.dim() == 3 else L.unsqueeze(0)
    B3 = B if B.dim() == 3 else B.unsqueeze(0)
    batch = B3.shape[0]
    n = L3.shape[1]
    nrhs = B3.shape[2]
    sL = 0 if L3.shape[0] == 1 else n * n
    call("evr_trsm_lower", _stream(), batch, n, nrhs, L3.data_ptr(), n, sL, int(transpose), B3.data_ptr(), nrhs,
         n * nrhs)
    return B


def tri_inv(L: torch.Tensor) -> torch.Tensor:
    L = _dev(L, "L")
    L3 = L if L.dim() == 3 else L.unsqueeze(0)
    batch, n, _ = L3.shape
    out = torch.empty_like(L3)
    call("evr_tri_inv_lower", _stream(), batch, n, L3.data_ptr(), n, n * n, out.data_ptr(), n, n * n)
    return out if L.dim() == 3 else out[0]


def posterior_finalize(R, c, ym, ys, kxx, noise_add=None):
    R = _dev(R, "R")
    B, n1, nt = R.shape
    mean = torch.empty(B, nt, dtype=torch.float64, device=R.device)
    var = torch.empty_like(mean)
    args = [_dev(t, "aux") for t in (c, ym, ys, kxx)]
    na = None if noise_add is None else _dev(noise_add, "noise")
    call("evr_gp_posterior_finalize", _stream(), B, n1 - 1, nt, R.data_ptr(), *[a.data_ptr() for a in args],
         _p(na), mean.data_ptr(), var.data_ptr())
    return mean, var


def gp_posterior(Xn, X, shift, scale, lengthscales, M, kind, c, ym, ys, kxx, noise_add=None):
    """Mean and variance (B x nt) in one native call: kernel_matrix -> R = M K_x -> finalize."""
    Xn, X, M = _dev(Xn, "Xn"), _dev(X, "X"), _dev(M, "M")
    B, n1, n = M.shape
    nt, d = X.shape
    if n1 != n + 1 or Xn.shape != (n, d):
        raise ValueError("gp_posterior: shape mismatch")
    mean = torch.empty(B, nt, dtype=torch.float64, device=X.device)
    var = torch.empty_like(mean)
    work = _workspace(_native.load().evr_gp_posterior_workspace_doubles(B, n, nt), X.device)
    aux = [_dev(t, "aux") for t in (shift, scale, lengthscales, c, ym, ys, kxx)]
    na = None if noise_add is None else _dev(noise_add, "noise")
    call("evr_gp_posterior", _stream(), B, n, nt, d, int(kind), Xn.data_ptr(), X.data_ptr(), aux[0].data_ptr(),
         aux[1].data_ptr(), aux[2].data_ptr(), M.data_ptr(), aux[3].data_ptr(), aux[4].data_ptr(), aux[5].data_ptr(),
         aux[6].data_ptr(), _p(na), mean.data_ptr(), var.data_ptr(), work.data_ptr())
    return mean, var


# ---------------------------------------------------------------------------------------
# qNEHVI pieces
# ---------------------------------------------------------------------------------------
def make_state(n, nb, S, m, c, ym, ys, kxx, zq, obj_a, obj_b, cells: "Cells", no_h: bool = False) -> EvrQnehviState:
    """no_h: the operator M carries no H^T rows (qEHVI: samples mu + L22 z, nb = 0)."""
    st = EvrQnehviState()
    st.n, st.nb, st.S, st.m = int(n), int(nb), int(S), int(m)
    st.no_h = int(bool(no_h))
    st.c, st.ym, st.ys, st.kxx = c.data_ptr(), ym.data_ptr(), ys.data_ptr(), kxx.data_ptr()
    st.zq, st.obj_a, st.obj_b = zq.data_ptr(), obj_a.data_ptr(), obj_b.data_ptr()
    st.cell_lo, st.cell_hi = _p(cells.lo), _p(cells.hi)
    st.cell_off = cells.off.data_ptr()
    st.max_cells = int(cells.max_cells)
    st.cell_keys, st.cell_pts, st.cell_rank0 = _p(cells.keys), _p(cells.pts), _p(cells.rank0)
    st.pts_stride = int(cells.stride)
    kd = cells.kd
    if kd is not None:
        st.grp_off, st.grp_keys, st.grp_rank = kd.goff.data_ptr(), kd.keys.data_ptr(), kd.rank.data_ptr()
        st.grp_box, st.sorted_lo, st.max_groups = kd.box.data_ptr(), kd.sorted_lo.data_ptr(), int(kd.max_groups)
    return st


def qnehvi_samples(st: EvrQnehviState, R: torch.Tensor, b: int):
    dev = R.device
    G = torch.empty(st.S, st.m, b, dtype=torch.float64, device=dev)
    L22 = torch.empty(st.m, b, dtype=torch.float64, device=dev)
    flags = torch.empty(st.m, b, dtype=torch.int32, device=dev)
    call("evr_qnehvi_samples", _stream(), ctypes.byref(st), b, R.data_ptr(), G.data_ptr(), L22.data_ptr(),
         flags.data_ptr())
    return G, L22, flags


def qnehvi_project(st: EvrQnehviState, M: torch.Tensor, Kx: torch.Tensor, b: int):
    """R = M Kx (m x Rr x b) and the partial norms the sampling step needs (one fused GEMM)."""
    dev = Kx.device
    Rr = st.n + st.nb + (0 if st.no_h else st.S) + 1
    R = torch.empty(st.m, Rr, b, dtype=torch.float64, device=dev)
    nrt = _native.load().evr_qnehvi_norms_rows(ctypes.byref(st))
    P = torch.empty(st.m, nrt, 2, b, dtype=torch.float64, device=dev)
    work = _workspace(_native.load().evr_qnehvi_project_workspace_doubles(ctypes.byref(st), b), dev)
    call("evr_qnehvi_project", _stream(), ctypes.byref(st), b, _dev(M, "M").data_ptr(), _dev(Kx, "Kx").data_ptr(),
         R.data_ptr(), P.data_ptr(), work.data_ptr())
    return R, P


def qnehvi_samples_norms(st: EvrQnehviState, R: torch.Tensor, P: torch.Tensor, b: int):
    dev = R.device
    G = torch.empty(st.S, st.m, b, dtype=torch.float64, device=dev)
    L22 = torch.empty(st.m, b, dtype=torch.float64, device=dev)
    flags = torch.empty(st.m, b, dtype=torch.int32, device=dev)
    call("evr_qnehvi_samples_norms", _stream(), ctypes.byref(st), b, R.data_ptr(), P.data_ptr(), G.data_ptr(),
         L22.data_ptr(), flags.data_ptr())
    return G, L22, flags


def qnehvi_project_backward(st: EvrQnehviState, M: torch.Tensor, R: torch.Tensor, L22: torch.Tensor,
                            dG: torch.Tensor, b: int) -> torch.Tensor:
    """dKx = M^T gR (m x n x b) with gR generated inside the GEMM."""
    dK = torch.empty(st.m, st.n, b, dtype=torch.float64, device=R.device)
    work = _workspace(_native.load().evr_qnehvi_project_backward_workspace_doubles(ctypes.byref(st), b), R.device)
    call("evr_qnehvi_project_backward", _stream(), ctypes.byref(st), b, M.data_ptr(), R.data_ptr(), L22.data_ptr(),
         dG.data_ptr(), dK.data_ptr(), work.data_ptr())
    return dK


def qnehvi_small_applies(st: EvrQnehviState, b: int, d: int) -> bool:
    """Whether the native plan runs the b <= 32 restart-batch kernels (qnehvi_small.hip) for
    this batch (EVR_SMALL=0 disables them, as in the plan)."""
    return (os.environ.get("EVR_SMALL", "1") != "0"
            and bool(_native.load().evr_qnehvi_small_applies(ctypes.byref(st), int(b), int(d))))


def qnehvi_small_forward(st: EvrQnehviState, model, Kx: torch.Tensor, b: int):
    """Restart-batch projection: R = M Kx and 16-row-tile partial norms (qs_fwd)."""
    dev = Kx.device
    lib = _native.load()
    Rr = st.n + st.nb + (0 if st.no_h else st.S) + 1
    R = torch.empty(st.m, Rr, b, dtype=torch.float64, device=dev)
    P = _workspace(lib.evr_qnehvi_small_workspace_doubles(ctypes.byref(st), b, model.d, 0), dev)
    call("evr_qnehvi_small_forward", _stream(), ctypes.byref(st), ctypes.byref(model), b,
         _dev(Kx, "Kx").data_ptr(), R.data_ptr(), P.data_ptr())
    return R, P


def qnehvi_small_samples(st: EvrQnehviState, R: torch.Tensor, P: torch.Tensor, b: int):
    dev = R.device
    G = torch.empty(st.S, st.m, b, dtype=torch.float64, device=dev)
    L22 = torch.empty(st.m, b, dtype=torch.float64, device=dev)
    flags = torch.empty(st.m, b, dtype=torch.int32, device=dev)
    call("evr_qnehvi_small_samples", _stream(), ctypes.byref(st), b, R.data_ptr(), P.data_ptr(), G.data_ptr(),
         L22.data_ptr(), flags.data_ptr())
    return G, L22, flags


def qnehvi_small_backward(st: EvrQnehviState, model, X: torch.Tensor, R: torch.Tensor, L22: torch.Tensor,
                          dG: torch.Tensor, b: int) -> torch.Tensor:
    """Restart-batch backward: dX (b x d) = d sum acq / dX with the cross-covariance gradient
    fused into the M^T gR product (qs_bwd + qs_dx_reduce)."""
    dev = R.device
    lib = _native.load()
    dXp = _workspace(lib.evr_qnehvi_small_workspace_doubles(ctypes.byref(st), b, model.d, 1), dev)
    dX = torch.empty(b, model.d, dtype=torch.float64, device=dev)
    call("evr_qnehvi_small_backward", _stream(), ctypes.byref(st), ctypes.byref(model), b,
         _dev(X, "X").contiguous().data_ptr(), R.data_ptr(), L22.data_ptr(), dG.data_ptr(), dXp.data_ptr(),
         dX.data_ptr())
    return dX


OBJ_AFFINE, OBJ_CLOSE_TO_TARGET = 0, 1


class GeneralSpec:
    """Objectives over selected model outputs and output constraints for the general
    qNEHVI / qEHVI kernels (qnehvi_general.hip, evr_qn_general).

    objectives: [(output, kind, p0, p1)] — kind OBJ_AFFINE: g = p0*y + p1 (Maximize /
    Minimize, bofire/utils/torch_tools.py:389-398), OBJ_CLOSE_TO_TARGET: g = -|y - p0|^p1
    (:399-402).  constraints: [(output, sign, threshold, eta)] — c = sign*(y - threshold)
    <= 0 is feasible, weight exp(sum logsigmoid(-c/eta)) (torch_tools.py:258-337)."""

    def __init__(self, m_model: int, objectives, constraints=()):
        self.m_model = int(m_model)
        self.objectives = [(int(o), int(k), float(a), float(b)) for o, k, a, b in objectives]
        self.constraints = [(int(o), float(sg), float(t), float(e)) for o, sg, t, e in constraints]
        if not 1 <= len(self.objectives) <= 8 or len(self.constraints) > 16:
            raise ValueError("general qNEHVI: 1..8 objectives and at most 16 output constraints")
        for o, *_ in self.objectives + self.constraints:
            if not 0 <= o < self.m_model:
                raise ValueError(f"general qNEHVI: output index {o} outside the model's {self.m_model} outputs")
        ob = self.objectives
        self._arrs = (np.array([o[0] for o in ob], np.int32), np.array([o[1] for o in ob], np.int32),
                      np.array([o[2] for o in ob], np.float64), np.array([o[3] for o in ob], np.float64))
        cs = self.constraints or [(0, 0.0, 0.0, 1.0)]
        self._carrs = (np.array([c[0] for c in cs], np.int32), np.array([c[1] for c in cs], np.float64),
                       np.array([c[2] for c in cs], np.float64), np.array([c[3] for c in cs], np.float64))

    @property
    def m_obj(self) -> int:
        return len(self.objectives)

    @property
    def affine_identity(self) -> bool:
        """Every output carries one affine objective, in output order, and no constraints:
        the q = 1 fast path (obj_a / obj_b fused into the sampling kernel) applies."""
        return (not self.constraints and self.m_obj == self.m_model and
                all(o == j and k == OBJ_AFFINE for j, (o, k, _, _) in enumerate(self.objectives)))

    def struct(self, q: int = 1, zq: Optional[torch.Tensor] = None) -> EvrQnGeneral:
        g = EvrQnGeneral()
        g.q, g.m_obj, g.n_con = int(q), self.m_obj, len(self.constraints)
        g.obj_out, g.obj_kind, g.obj_p0, g.obj_p1 = (a.ctypes.data for a in self._arrs)
        g.con_out, g.con_sign, g.con_thr, g.con_eta = (a.ctypes.data for a in self._carrs)
        g.zq = _p(zq)
        return g

    def host_weights(self, Y: np.ndarray) -> np.ndarray:
        """Smoothed feasibility weights exp(sum_c logsigmoid(-c / eta)) of model-output rows Y
        (... x m_model) on the host ([upstream] compute_smoothed_feasibility_indicator,
        fat=False); 1 without constraints."""
        lw = np.zeros(Y.shape[:-1])
        for o, sg, t, eta in self.constraints:
            x = -sg * (Y[..., o] - t) / eta
            lw += np.minimum(x, 0.0) - np.log1p(np.exp(-np.abs(x)))
        return np.exp(lw)

    def host_objective(self, Y: np.ndarray) -> np.ndarray:
        """Objectives of model-output rows Y (... x m_model) on the host (observed data)."""
        cols = []
        for o, k, a, b in self.objectives:
            y = Y[..., o]
            cols.append(a * y + b if k == OBJ_AFFINE else -np.abs(y - a) ** b)
        return np.stack(cols, -1)


def objective_general(Y: torch.Tensor, mu: Optional[torch.Tensor], spec: GeneralSpec, ref: torch.Tensor):
    """Y: m_model x n x S (+ mu m_model x n) -> objectives m_obj x n x S, infeasible samples
    (any constraint c > 0) set to the reference point."""
    Y = _dev(Y, "Y")
    m, n, S = Y.shape
    O = torch.empty(spec.m_obj, n, S, dtype=torch.float64, device=Y.device)
    g = spec.struct()
    call("evr_objective_general", _stream(), m, n, S, ctypes.byref(g), Y.data_ptr(),
         _p(None if mu is None else _dev(mu, "mu")), _dev(ref, "ref").data_ptr(), O.data_ptr())
    return O


def objective_weights(Y: torch.Tensor, spec: GeneralSpec):
    """Y: m_model x n model-output rows on device -> (objectives m_obj x n, feasibility
    weights n) through the general scan's per-point device function (evr_objective_weights)."""
    Y = _dev(Y, "Y")
    m, n = Y.shape
    if m != spec.m_model:
        raise ValueError(f"Y has {m} outputs, the spec {spec.m_model}")
    G = torch.empty(spec.m_obj, n, dtype=torch.float64, device=Y.device)
    W = torch.empty(n, dtype=torch.float64, device=Y.device)
    g = spec.struct()
    call("evr_objective_weights", _stream(), m, n, ctypes.byref(g), Y.data_ptr(), G.data_ptr(), W.data_ptr())
    return G, W


def qng_eval(stm: EvrQnehviState, sth: EvrQnehviState, g: EvrQnGeneral, model: "_native.EvrQnehviModel",
             X: torch.Tensor, backward: bool, gout: Optional[torch.Tensor] = None):
    """General qNEHVI / qEHVI: X (b*q) x d raw candidates (point i of candidate c at row
    c*q + i) -> acq (b) [, dX (b*q) x d]."""
    X = _dev(X, "X")
    q = int(g.q)
    bq, d = X.shape
    if bq % q:
        raise ValueError(f"{bq} rows are not a multiple of q = {q}")
    b = bq // q
    lib = _native.load()
    work = _workspace(lib.evr_qng_workspace_doubles(ctypes.byref(stm), ctypes.byref(sth), ctypes.byref(g),
                                                    ctypes.byref(model), b, int(backward)), X.device)
    acq = torch.empty(b, dtype=torch.float64, device=X.device)
    dX = torch.empty_like(X) if backward else None
    call("evr_qng_eval", _stream(), ctypes.byref(stm), ctypes.byref(sth), ctypes.byref(g), ctypes.byref(model), b,
         X.data_ptr(), _p(None if gout is None else _dev(gout, "gout")), work.data_ptr(), acq.data_ptr(), _p(dX))
    return acq, dX


def qlog_eval(stm: EvrQnehviState, sth: EvrQnehviState, g: EvrQnGeneral, model: "_native.EvrQnehviModel",
              X: torch.Tensor, backward: bool, gout: Optional[torch.Tensor] = None):
    """Log-space general qLogNEHVI / qLogEHVI (evr_qlog_eval): X (b*q) x d raw candidates ->
    acq (b) [, dX (b*q) x d]; ``sth`` carries the explicit cells and tau_relu / tau_max."""
    X = _dev(X, "X")
    q = int(g.q)
    bq, d = X.shape
    if bq % q:
        raise ValueError(f"{bq} rows are not a multiple of q = {q}")
    b = bq // q
    lib = _native.load()
    work = _workspace(lib.evr_qlog_workspace_doubles(ctypes.byref(stm), ctypes.byref(sth), ctypes.byref(g),
                                                     ctypes.byref(model), b, int(backward)), X.device)
    acq = torch.empty(b, dtype=torch.float64, device=X.device)
    dX = torch.empty_like(X) if backward else None
    call("evr_qlog_eval", _stream(), ctypes.byref(stm), ctypes.byref(sth), ctypes.byref(g), ctypes.byref(model), b,
         X.data_ptr(), _p(None if gout is None else _dev(gout, "gout")), work.data_ptr(), acq.data_ptr(), _p(dX))
    return acq, dX


class QnehviPlan:
    """Native evaluation plan of the whole qNEHVI chain for a fixed batch size b
    (qnehvi_plan.hip): persistent device buffers X (b x d), out = [acq (b) | dX (b x d)] and
    the workspace; run() is one C-ABI call (one hipGraph launch when ``graph``)."""

    def __init__(self, st: EvrQnehviState, model: "_native.EvrQnehviModel", b: int, backward: bool, device,
                 graph: bool = True):
        lib = _native.load()
        d = int(model.d)
        self.b, self.d, self.backward = int(b), d, bool(backward)
        self.X = torch.zeros(b, d, dtype=torch.float64, device=device)
        self.out = torch.empty(b * (1 + d), dtype=torch.float64, device=device)
        nbytes = lib.evr_qnehvi_plan_workspace_bytes(ctypes.byref(st), ctypes.byref(model), b, int(backward))
        self.work = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
        self.acq = self.out[:b]
        self.dX = self.out[b:].view(b, d)
        self.host = torch.zeros(b * (1 + d), dtype=torch.float64)
        h = ctypes.c_void_p()
        call("evr_qnehvi_plan_create", _stream(), ctypes.byref(st), ctypes.byref(model), b, int(backward),
             self.X.data_ptr(), self.work.data_ptr(), self.acq.data_ptr(),
             self.dX.data_ptr() if backward else None, int(graph), ctypes.byref(h))
        self._h = h
        self._lib = lib

    def run(self):
        call("evr_qnehvi_plan_run", _stream(), self._h)

    def run_host(self, x: np.ndarray) -> np.ndarray:
        """x (b x d numpy) -> host [acq | dX] (evr_qnehvi_plan_eval_host: one graph launch
        reading x from and writing the results to pinned host memory)."""
        xh = np.ascontiguousarray(x, dtype=np.float64).reshape(self.b, self.d)
        out = self.host.numpy()
        call("evr_qnehvi_plan_eval_host", _stream(), self._h, xh.ctypes.data, out.ctypes.data)
        return out

    def minimize(self, x0: np.ndarray, lb: np.ndarray, ub: np.ndarray, maxiter: int, maxfun: int = 15000,
                 maxcor: int = 10, ftol: float = 2.220446049250313e-09, gtol: float = 1e-5, maxls: int = 20):
        """Native L-BFGS-B over the b restarts of this (backward) plan, the whole loop in C++
        (evr_qnehvi_plan_minimize): returns (x (b*d, clipped), acq (b) at x,
        [iterations, evaluations, status, task]).  Raises NotPSDError on a NaN evaluation."""
        if not self.backward:
            raise ValueError("minimize needs a backward plan")
        n = self.b * self.d
        f64 = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(n))  # noqa: E731
        x0, lb, ub = f64(x0), f64(lb), f64(ub)
        x = np.empty(n)
        acq = np.empty(self.b)
        info = np.zeros(4, dtype=np.int32)
        rc = self._lib.evr_qnehvi_plan_minimize(_stream(), self._h, x0.ctypes.data, lb.ctypes.data, ub.ctypes.data,
                                                int(maxiter), int(maxfun), ftol / float(np.finfo(float).eps),
                                                float(gtol), int(maxcor), int(maxls), x.ctypes.data,
                                                acq.ctypes.data, info.ctypes.data)
        if rc == 7:
            raise NotPSDError(self._lib.evr_last_error().decode(errors="replace"))
        _native.check(rc, "evr_qnehvi_plan_minimize")
        return x, acq, info.tolist()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.evr_qnehvi_plan_destroy(h)
            self._h = None


def _hvi_work(st: EvrQnehviState, b: int, backward: bool, device) -> torch.Tensor:
    n = _native.load().evr_hvi_workspace_doubles(ctypes.byref(st), b, int(backward))
    return torch.empty(max(1, n), dtype=torch.float64, device=device)


def hvi_forward(st: EvrQnehviState, G: torch.Tensor, b: int, flags: Optional[torch.Tensor] = None) -> torch.Tensor:
    """acq[c] = mean_s HVI_s (register-tiled scan + deterministic reduction); NaN where
    ``flags`` (m x b int32 from qnehvi_samples) marks a failed new-point Cholesky."""
    acq = torch.empty(b, dtype=torch.float64, device=G.device)
    work = _hvi_work(st, b, False, G.device)
    call("evr_hvi_forward", _stream(), ctypes.byref(st), b, G.data_ptr(), _p(flags), work.data_ptr(),
         acq.data_ptr())
    return acq


def mean_over_samples(partial: torch.Tensor):
    S, b = partial.shape
    acq = torch.empty(b, dtype=torch.float64, device=partial.device)
    call("evr_mean_over_samples", _stream(), S, b, partial.data_ptr(), acq.data_ptr())
    return acq


def hvi_backward(st: EvrQnehviState, G: torch.Tensor, gout: Optional[torch.Tensor], b: int):
    """dG = gout/S * dHVI/dG (gout None = ones)."""
    dG = torch.empty_like(G)
    if gout is not None:
        gout = _dev(gout, "gout")
    work = _hvi_work(st, b, True, G.device)
    call("evr_hvi_backward", _stream(), ctypes.byref(st), b, G.data_ptr(), _p(gout), work.data_ptr(),
         dG.data_ptr())
    return dG


def hvi_forward_backward(st: EvrQnehviState, G: torch.Tensor, b: int, flags: Optional[torch.Tensor] = None,
                         gout: Optional[torch.Tensor] = None):
    """One fused scan: (acq (b), dG = gout/S * dHVI/dG)."""
    acq = torch.empty(b, dtype=torch.float64, device=G.device)
    dG = torch.empty_like(G)
    if gout is not None:
        gout = _dev(gout, "gout")
    work = _hvi_work(st, b, True, G.device)
    call("evr_hvi_forward_backward", _stream(), ctypes.byref(st), b, G.data_ptr(), _p(flags), _p(gout),
         work.data_ptr(), acq.data_ptr(), dG.data_ptr())
    return acq, dG


def hvi_restart_fb_applies(st: EvrQnehviState, b: int) -> bool:
    return bool(_native.load().evr_hvi_restart_fb_applies(ctypes.byref(st), int(b)))


def hvi_restart_fb(st: EvrQnehviState, G: torch.Tensor, b: int):
    """The restart-batch scan in one launch (hvi_kd3, b <= 32): (per-sample values S x b,
    dG = dHVI/dG / S); acq = mean_over_samples(values)."""
    S = int(st.S)
    sval = torch.empty(S, b, dtype=torch.float64, device=G.device)
    dG = torch.empty_like(G)
    call("evr_hvi_restart_fb", _stream(), ctypes.byref(st), b, G.data_ptr(), sval.data_ptr(), dG.data_ptr())
    return sval, dG


def qnehvi_samples_backward(st: EvrQnehviState, R, L22, dG, b: int):
    gR = torch.empty_like(R)
    call("evr_qnehvi_samples_backward", _stream(), ctypes.byref(st), b, R.data_ptr(), L22.data_ptr(), dG.data_ptr(),
         gR.data_ptr())
    return gR


def pareto_mask(O: torch.Tensor, ref: torch.Tensor, dedup: bool, want_mask=True, want_counts=False):
    """O: m x n x S.  Returns (mask S x n uint8 | None, counts n int32 | None)."""
    O, ref = _dev(O, "O"), _dev(ref, "ref")
    m, n, S = O.shape
    mask = torch.empty(S, n, dtype=torch.uint8, device=O.device) if want_mask else None
    counts = torch.zeros(n, dtype=torch.int32, device=O.device) if want_counts else None
    call("evr_pareto_mask", _stream(), S, n, m, O.data_ptr(), ref.data_ptr(), int(dedup), _p(mask), _p(counts))
    return mask, counts


def objective_affine(Y: torch.Tensor, mu: Optional[torch.Tensor], a: torch.Tensor, b: torch.Tensor):
    Y = _dev(Y, "Y")
    m, n, S = Y.shape
    O = torch.empty_like(Y)
    mu = None if mu is None else _dev(mu, "mu")
    call("evr_objective_affine", _stream(), m, n, S, Y.data_ptr(), _p(mu), _dev(a, "a").data_ptr(),
         _dev(b, "b").data_ptr(), O.data_ptr())
    return O


def qei(R: torch.Tensor, c: float, ym: float, ys: float, kxx: float, z: torch.Tensor, a: float, b: float,
        best_f: float, with_grad: bool):
    R, z = _dev(R, "R"), _dev(z, "z")
    n1, nb = R.shape
    acq = torch.empty(nb, dtype=torch.float64, device=R.device)
    gR = torch.empty_like(R) if with_grad else None
    flags = torch.empty(nb, dtype=torch.int32, device=R.device)
    call("evr_qei", _stream(), n1 - 1, nb, z.numel(), R.data_ptr(), float(c), float(ym), float(ys), float(kxx),
         z.data_ptr(), float(a), float(b), float(best_f), acq.data_ptr(), _p(gR), flags.data_ptr())
    return acq, gR, flags


def scale_batched(X: torch.Tensor, alpha: torch.Tensor) -> torch.Tensor:
    """In place X[b] *= alpha[b]."""
    if not X.is_contiguous():
        raise ValueError("scale_batched: X must be contiguous")
    B = X.shape[0]
    call("evr_scale_batched", _stream(), B, X.numel() // B, _dev(alpha, "alpha").data_ptr(), X.data_ptr())
    return X


def add_selection(E: torch.Tensor, idx: torch.Tensor, val: Optional[torch.Tensor]) -> torch.Tensor:
    """In place E[b][r][idx[r]] += val[b]; E: B x nb x n, idx int32 (nb)."""
    B, nb, n = E.shape
    idx = _dev(idx, "idx", torch.int32)
    call("evr_add_selection", _stream(), B, nb, n, idx.data_ptr(), _p(None if val is None else _dev(val, "val")),
         E.data_ptr())
    return E


def box_device_supported(n: int, m: int) -> bool:
    return _native.load().evr_box_device_limits(int(n), int(m), None, None) == 0


class Cells:
    """Box cells of S samples on the device, ragged by ``off`` (S+1 int32): either explicit
    (``lo``/``hi``, C x m) or compressed (``keys`` C uint64 + per-sample point tables ``pts``
    S x stride x m and ``rank0`` S x stride, the device box decomposition's output)."""

    def __init__(self, off, counts, m, lo=None, hi=None, keys=None, pts=None, rank0=None, stride=0):
        self.off, self.counts, self.m = off, np.asarray(counts, dtype=np.int64), int(m)
        self.lo, self.hi, self.keys, self.pts, self.rank0, self.stride = lo, hi, keys, pts, rank0, int(stride)
        self.kd: Optional[KdGroups] = None

    @property
    def S(self) -> int:
        return int(self.counts.shape[0])

    @property
    def total(self) -> int:
        return int(self.counts.sum())

    @property
    def max_cells(self) -> int:
        return int(self.counts.max()) if self.S else 0

    def explicit(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """(lo, hi) rows (C x m, maximisation space); expands compressed cells on the device."""
        if self.keys is None:
            return self.lo, self.hi
        lo = torch.empty(self.total, self.m, dtype=torch.float64, device=self.off.device)
        hi = torch.empty_like(lo)
        call("evr_cells_from_keys", _stream(), self.S, self.m, self.stride, self.off.data_ptr(), self.max_cells,
             self.keys.data_ptr(), self.pts.data_ptr(), self.rank0.data_ptr(), lo.data_ptr(), hi.data_ptr())
        return lo, hi


class KdGroups:
    """kd-ordered groups of 16 compressed cells (cells_kd.hip) for the sparse HVI scan."""

    def __init__(self, goff, keys, rank, box, sorted_lo, max_groups):
        self.goff, self.keys, self.rank, self.box = goff, keys, rank, box
        self.sorted_lo, self.max_groups = sorted_lo, int(max_groups)


def kd_supported(cells: Cells) -> bool:
    if cells.keys is None or cells.S == 0:
        return False
    return _native.load().evr_cells_kd_limits(cells.stride, cells.m, cells.max_cells, None) == 0


def cells_kd_order(cells: Cells) -> KdGroups:
    """kd order + rank index of compressed cells (one workgroup per sample); attaches and
    returns the KdGroups (the HVI scan then runs the sparse three-level filter)."""
    if cells.keys is None:
        raise ValueError("cells_kd_order needs compressed cells (device box decomposition)")
    S, m, stride = cells.S, cells.m, cells.stride
    dev = cells.off.device
    ng = (cells.counts + 15) // 16
    goff_h = np.zeros(S + 1, dtype=np.int64)
    np.cumsum(ng, out=goff_h[1:])
    G = int(goff_h[-1])
    goff = torch.as_tensor(goff_h.astype(np.int32)).to(dev)
    keys = torch.empty(max(G, 1) * 16, dtype=torch.int64, device=dev)
    rank = torch.empty(max(G, 1) * m * 16, dtype=torch.int16, device=dev)       # uint16 bit patterns
    box = torch.empty(max(G, 1) * 8, dtype=torch.int16, device=dev)
    sorted_lo = torch.empty(S, m, stride, dtype=torch.float64, device=dev)
    call("evr_cells_kd_order_device", _stream(), S, m, stride, cells.off.data_ptr(), goff.data_ptr(),
         cells.max_cells, cells.keys.data_ptr(), cells.pts.data_ptr(), cells.rank0.data_ptr(), keys.data_ptr(),
         rank.data_ptr(), box.data_ptr(), sorted_lo.data_ptr())
    cells.kd = KdGroups(goff, keys, rank, box, sorted_lo, int(ng.max()) if S else 0)
    return cells.kd


class BoxCapacityError(RuntimeError):
    """The device box decomposition needs more LUB slots than its capacity / memory bound
    (the caller falls back to the exact host partition)."""


def box_decompose_device(O: torch.Tensor, ref: torch.Tensor, cap: int = 16384, max_cap: int = 1 << 20,
                         max_workspace_bytes: int = 8 << 30) -> Cells:
    """Device box decomposition of every sample of O (m x n x S objective values) above ref,
    returned compressed (64-bit keys + point tables, see Cells).

    One host sync (the per-sample cell counts size the packed arrays and the HVI plan); a
    sample overflowing ``cap`` LUB slots reruns the batch with 4x the capacity, up to
    ``max_cap`` slots and ``max_workspace_bytes`` of workspace, beyond which it raises
    BoxCapacityError."""
    O, ref = _dev(O, "O"), _dev(ref, "ref")
    m, n, S = O.shape
    dev = O.device
    while True:
        nbytes = _native.load().evr_box_device_workspace_bytes(S, n, m, cap)
        if nbytes > max_workspace_bytes:
            raise BoxCapacityError(f"box decomposition: {cap} LUB slots x {S} samples need {nbytes} B of workspace")
        ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        cs = torch.empty(2, S, dtype=torch.int32, device=dev)
        call("evr_box_decompose_device", _stream(), S, n, m, O.data_ptr(), ref.data_ptr(), cap, ws.data_ptr(),
             cs[0].data_ptr(), cs[1].data_ptr())
        h = cs.cpu().numpy()
        if not h[1].any():
            break
        if cap >= max_cap:
            raise BoxCapacityError(f"box decomposition: more than {max_cap} local upper bounds in one sample")
        cap *= 4
    counts = h[0].astype(np.int64)
    off_h = np.zeros(S + 1, dtype=np.int64)
    np.cumsum(counts, out=off_h[1:])
    total = int(off_h[-1])
    off = torch.as_tensor(off_h.astype(np.int32)).to(dev)
    stride = n + m
    keys = torch.empty(max(total, 1), dtype=torch.int64, device=dev)      # uint64 bit patterns
    pts = torch.empty(S, stride, m, dtype=torch.float64, device=dev)
    rank0 = torch.empty(S, stride, dtype=torch.int32, device=dev)
    call("evr_box_pack_keys_device", _stream(), S, n, m, cap, ws.data_ptr(), off.data_ptr(),
         int(counts.max()) if S else 0, keys.data_ptr(), pts.data_ptr(), rank0.data_ptr())
    return Cells(off, counts, m, keys=keys, pts=pts, rank0=rank0, stride=stride)


def box_decompose_kd_device(O: torch.Tensor, ref: torch.Tensor, want_kd: bool = True, cap: int = 16384,
                            max_cap: int = 1 << 20, max_workspace_bytes: int = 8 << 30):
    """box_decompose_device + cells_kd_order in one native call (evr_box_kd_pipeline): the
    count read-back, the offsets and the pack / kd launches happen in C++ with the GIL released,
    so no Python runs between the kernels.  Outputs are allocated for the capacity and returned
    as views of the used prefix.  Returns (cells, kd_built); cells.kd is attached when built."""
    O, ref = _dev(O, "O"), _dev(ref, "ref")
    m, n, S = O.shape
    dev = O.device
    stride = n + m
    lib = _native.load()
    counts_h = np.zeros(S, dtype=np.int32)
    info = np.zeros(3, dtype=np.int32)
    cap0 = cap
    while True:
        nbytes = lib.evr_box_device_workspace_bytes(S, n, m, cap)
        G = S * cap // 16 + S
        # the capacity-sized outputs count against the budget too (they live as long as the
        # acquisition when not trimmed below)
        out_bytes = 8 * S * cap + 8 * S * stride * m + 4 * S * stride + 16 * S + 8
        if want_kd:
            out_bytes += G * 16 * 8 + G * m * 16 * 2 + G * 8 * 2 + 8 * S * m * stride
        if nbytes + out_bytes > max_workspace_bytes:
            raise BoxCapacityError(f"box decomposition: {cap} LUB slots x {S} samples need {nbytes + out_bytes} B "
                                   "of workspace and outputs")
        try:
            ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            cs = torch.empty(2, S, dtype=torch.int32, device=dev)
            offs = torch.empty(2, S + 1, dtype=torch.int32, device=dev)
            keys = torch.empty(S * cap, dtype=torch.int64, device=dev)           # uint64 bit patterns
            pts = torch.empty(S, stride, m, dtype=torch.float64, device=dev)
            rank0 = torch.empty(S, stride, dtype=torch.int32, device=dev)
            if want_kd:
                okeys = torch.empty(G * 16, dtype=torch.int64, device=dev)
                ork = torch.empty(G * m * 16, dtype=torch.int16, device=dev)    # uint16 bit patterns
                ogb = torch.empty(G * 8, dtype=torch.int16, device=dev)
                osv = torch.empty(S, m, stride, dtype=torch.float64, device=dev)
            else:
                okeys = ork = ogb = osv = None
        except torch.OutOfMemoryError as e:
            raise BoxCapacityError(f"box decomposition: out of device memory at {cap} LUB slots x {S} samples") from e
        call("evr_box_kd_pipeline", _stream(), S, n, m, O.data_ptr(), ref.data_ptr(), cap, ws.data_ptr(),
             cs[0].data_ptr(), cs[1].data_ptr(), offs[0].data_ptr(), offs[1].data_ptr(), keys.data_ptr(),
             pts.data_ptr(), rank0.data_ptr(), int(bool(want_kd)), _p(okeys), _p(ork), _p(ogb), _p(osv),
             counts_h.ctypes.data, info.ctypes.data)
        if not info[0]:
            break
        if cap >= max_cap:
            raise BoxCapacityError(f"box decomposition: more than {max_cap} local upper bounds in one sample")
        cap *= 4
    counts = counts_h.astype(np.int64)
    total = int(counts.sum())
    del ws
    # a capacity rerun leaves outputs sized for 4x the slots or more: keep copies of the used
    # prefixes instead of views that pin the whole allocation (the first-try capacity keeps
    # views: no copy on the ask's critical path)
    trim = (lambda t: t.clone()) if cap > cap0 else (lambda t: t)
    cells = Cells(offs[0], counts, m, keys=trim(keys[:max(total, 1)]), pts=pts, rank0=rank0, stride=stride)
    if info[1]:
        ng = (counts + 15) // 16
        Gu = int(ng.sum())
        cells.kd = KdGroups(offs[1], trim(okeys[:max(Gu, 1) * 16]), trim(ork[:max(Gu, 1) * m * 16]),
                            trim(ogb[:max(Gu, 1) * 8]), osv, int(ng.max()) if S else 0)
    return cells, bool(info[1])


_SOBOL_DIRECTIONS = {}


def _sobol_directions(dim: int) -> torch.Tensor:
    """Unscrambled 30-bit direction numbers of torch's SobolEngine (Joe-Kuo D(6) table as
    torch ships it), cached per dimension; scrambled per seed by evr_sobol_scramble."""
    V = _SOBOL_DIRECTIONS.get(dim)
    if V is None:
        V = torch.zeros(dim, 30, dtype=torch.long)
        torch._sobol_engine_initialize_state_(V, dim)
        if len(_SOBOL_DIRECTIONS) > 16:
            _SOBOL_DIRECTIONS.clear()
        _SOBOL_DIRECTIONS[dim] = V
    return V


SOBOL_MAXDIM = 21201     # torch.quasirandom.SobolEngine.MAXDIM


def _iid_normal(n: int, dim: int, seed: int, device, d0: int, nd: int, layout: int, m: int) -> torch.Tensor:
    """[upstream] get_sampler's fallback beyond SobolEngine.MAXDIM dims: IIDNormalSampler,
    torch.randn of the (n, dim) base-sample shape under manual_seed(seed) (CPU generator),
    restricted to dims [d0, d0+nd) in the requested layout."""
    warnings.warn(f"{dim} base-sample dims exceed SobolEngine.MAXDIM={SOBOL_MAXDIM}: IID normal base samples",
                  RuntimeWarning)
    g = torch.Generator().manual_seed(int(seed))
    Z = torch.randn(n, dim, generator=g, dtype=torch.float64)[:, d0:d0 + nd]
    if layout == 0:
        return Z.contiguous().to(device)
    return Z.reshape(n, nd // m, m).permute(2, 1, 0).contiguous().to(device)


def sobol_scramble(dim: int, seed: int, d0: int = 0, nd: Optional[int] = None):
    """Host half of draw_sobol_normal_samples: the scrambled direction numbers (nd x 30) and
    shifts (nd) of dims [d0, d0+nd) of SobolEngine(dim, scramble=True, seed) (CPU int64
    tensors; evr_sobol_scramble_range).  None beyond SOBOL_MAXDIM (IID fallback).  Releases the
    GIL: the acquisition prefetches it on a worker thread."""
    nd = dim - d0 if nd is None else nd
    if not (0 <= d0 and nd >= 1 and d0 + nd <= dim):
        raise ValueError("sobol_scramble: dims out of range")
    if dim > SOBOL_MAXDIM:
        return None
    V, shift = _pinned_scramble_out(dim, d0, nd)
    call("evr_sobol_scramble_range", dim, int(seed), d0, nd, V.data_ptr(), shift.data_ptr())
    return V, shift


def _pinned_scramble_out(dim: int, d0: int, nd: int):
    """(direction numbers of dims [d0, d0+nd), shift buffer) in pinned host memory when a GPU
    is present, so that sobol_normal's uploads are asynchronous (a pageable .to(device) blocks
    the host until the stream has drained)."""
    pin = os.environ.get("EVR_SOBOL_PINNED", "1") != "0" and torch.cuda.is_available()
    V = torch.empty(nd, 30, dtype=torch.long, pin_memory=pin)
    V.copy_(_sobol_directions(dim)[d0:d0 + nd])
    return V, torch.empty(nd, dtype=torch.long, pin_memory=pin)


class SobolStream:
    """The raw mt19937 stream of one seed, long enough for draws of up to ``max_dim``
    dimensions (evr_sobol_stream_create; releases the GIL, so it can be generated on a worker
    thread before the draw's dimension count is known)."""

    def __init__(self, seed: int, max_dim: int):
        lib = _native.load()
        self._lib = lib
        self.seed, self.max_dim = int(seed), int(max_dim)
        h = ctypes.c_void_p()
        call("evr_sobol_stream_create", self.seed, lib.evr_sobol_stream_words(self.max_dim), ctypes.byref(h))
        self._h = h

    def scramble(self, dim: int, d0: int = 0, nd: Optional[int] = None):
        """(V, shift) of dims [d0, d0+nd) of SobolEngine(dim, scramble=True, seed) — as
        sobol_scramble — or None beyond SOBOL_MAXDIM / this stream's length."""
        nd = dim - d0 if nd is None else nd
        if dim > SOBOL_MAXDIM or dim > self.max_dim or nd < 1:
            return None
        V, shift = _pinned_scramble_out(dim, d0, nd)
        call("evr_sobol_scramble_stream", self._h, dim, d0, nd, V.data_ptr(), shift.data_ptr())
        return V, shift

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None:
            try:
                self._lib.evr_sobol_stream_destroy(h)
            except Exception:
                pass
            self._h = None


def sobol_normal(n: int, dim: int, seed: int, device, d0: int = 0, nd: Optional[int] = None,
                 layout: int = 0, m: int = 1, scrambled=None) -> torch.Tensor:
    """Device draw_sobol_normal_samples(dim, n, seed) restricted to dims [d0, d0+nd).

    layout 0 -> n x nd; layout 1 -> m x (nd/m) x n (sample index fastest, the GEMM-ready
    layout of the baseline / prune samples: dim t = point*m + output).  ``scrambled``: the
    (V, shift) of sobol_scramble(dim, seed, d0, nd) when already computed."""
    nd = dim - d0 if nd is None else nd
    if not (0 <= d0 and d0 + nd <= dim):
        raise ValueError("sobol_normal: dims out of range")
    if dim > SOBOL_MAXDIM:
        return _iid_normal(n, dim, seed, device, d0, nd, layout, m)
    if layout == 0:
        out = torch.empty(n, nd, dtype=torch.float64, device=device)
    else:
        out = torch.empty(m, nd // m, n, dtype=torch.float64, device=device)
    if nd == 0:
        return out
    V, shift = scrambled if scrambled is not None else sobol_scramble(dim, seed, d0, nd)
    Vd = V.to(device, non_blocking=V.is_pinned())
    sd = shift.to(device, non_blocking=shift.is_pinned())
    call("evr_sobol_normal", _stream(), n, nd, 0, Vd.data_ptr(), sd.data_ptr(), layout, m, out.data_ptr())
    return out


def box_decompose(obj: np.ndarray, ref: np.ndarray, mask: Optional[np.ndarray] = None, num_threads: int = 0,
                  layout: str = "jis", alpha: float = 0.0):
    """Host box decomposition.  obj: float64 numpy array, layout 'jis' (m x n x S) or 'sij'
    (S x n x m).  alpha > 0 (m > 2): the approximate partition of [upstream]
    NondominatedPartitioning(alpha).  Returns (lo [C x m], hi [C x m], off [S+1]) numpy arrays."""
    lib = _native.load()
    obj = np.ascontiguousarray(obj, dtype=np.float64)
    if layout == "jis":
        m, n, S = obj.shape
        ss, si, sj = 1, S, n * S
    elif layout == "sij":
        S, n, m = obj.shape
        ss, si, sj = n * m, m, 1
    else:
        raise ValueError(layout)
    ref = np.ascontiguousarray(ref, dtype=np.float64)
    mk = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
    handle = ctypes.c_void_p()
    _native.check(lib.evr_box_decompose_approx(S, n, m, obj.ctypes.data, ss, si, sj,
                                               None if mk is None else mk.ctypes.data, ref.ctypes.data,
                                               float(alpha), int(num_threads), ctypes.byref(handle)),
                  "evr_box_decompose_approx")
    try:
        total = lib.evr_cells_total(handle)
        lo = np.empty((total, m), dtype=np.float64)
        hi = np.empty((total, m), dtype=np.float64)
        off = np.empty(S + 1, dtype=np.int32)
        lib.evr_cells_copy(handle, lo.ctypes.data, hi.ctypes.data, off.ctypes.data)
    finally:
        lib.evr_cells_free(handle)
    return lo, hi, off


def device_arch(device: int = 0) -> str:
    buf = ctypes.create_string_buffer(64)
    call("evr_device_arch", device, buf, 64)
    return buf.value.decode()
