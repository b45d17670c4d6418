"""PyTorch-ROCm custom operators of the hot path (TORCH_LIBRARY(everest_amd), built from
everest_amd/csrc/torch_ops.cpp into _lib/libeverest_amd_torch.so) and their autograd
wrappers — SURVEY.md §8(b)'s numeric op boundary, replacing the BoTorch Model.posterior /
AcquisitionFunction.forward protocols called at bofire/strategies/predictives/botorch.py:
180,223,384:

    torch.ops.everest_amd.kernel_matrix(X1, X2, lengthscales, kind) -> K (B x n1 x n2)
    torch.ops.everest_amd.cholesky(A, jitter0, max_tries) -> (L, jitter, info)
    torch.ops.everest_amd.gp_posterior(Xn, X, shift, scale, ls, M, kind, c, ym, ys, kxx, noise?)
    torch.classes.everest_amd.QnehviAcq(state, scan_state, model, fast, keep)  (owns state + plans)
    torch.ops.everest_amd.qnehvi_forward(acq, X) -> acq values
    torch.ops.everest_amd.qnehvi_forward_backward(acq, X) -> (acq values, dX)
    torch.ops.everest_amd.qnehvi_backward(acq, X, grad_out) -> dX

No fallback: a missing library raises NativeLibraryError."""
from __future__ import annotations

import os

import torch

from ._native import NativeLibraryError

_HERE = os.path.dirname(os.path.abspath(__file__))
TORCH_LIB_PATH = os.path.join(_HERE, "_lib", "libeverest_amd_torch.so")
_loaded = False


def load():
    """Register the operators (once); returns the torch.ops.everest_amd namespace."""
    global _loaded
    if not _loaded:
        if not os.path.exists(TORCH_LIB_PATH):
            raise NativeLibraryError(f"everest_amd torch operator library not found at {TORCH_LIB_PATH}; build it "
                                     "with `python -c 'import __graft_entry__ as g; g.build()'`")
        from . import _native
        _native.load()            # the C-ABI library first (same file the operators link)
        torch.ops.load_library(TORCH_LIB_PATH)
        _loaded = True
    return torch.ops.everest_amd


class QnehviFunction(torch.autograd.Function):
    """acq = qNEHVI / qEHVI(X) through the torch operators on a
    torch.classes.everest_amd.QnehviAcq (which owns the acquisition state and caches its
    plans).  When X needs a gradient the forward runs qnehvi_forward_backward — ONE device
    chain for the value and the analytic gradient — and saves dX; backward only scales it by
    grad_out (candidates are independent)."""

    @staticmethod
    def forward(ctx, X: torch.Tensor, acq):
        ops = load()
        if ctx.needs_input_grad[0]:
            a, dX = ops.qnehvi_forward_backward(acq, X)
            ctx.save_for_backward(dX)
            return a
        ctx.save_for_backward(None)
        return ops.qnehvi_forward(acq, X)

    @staticmethod
    def backward(ctx, grad_out: torch.Tensor):
        (dX,) = ctx.saved_tensors
        shape = (dX.shape[0],) + (1,) * (dX.dim() - 1)
        return dX * grad_out.reshape(shape), None
