"""ctypes binding of the C-ABI in include/everest_amd.h (libeverest_amd.so, gfx950).

The library is built in-tree (``everest_amd/_lib``) by ``__graft_entry__.build()`` /
``make -C everest_amd/csrc``.  There is no fallback: if the library is missing every op
raises ``NativeLibraryError``.  ``torch`` is imported first so that the HIP runtime torch
ships (SONAME libamdhip64.so.7) is the one the library binds to — one runtime, one set of
streams per process.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_longlong, c_void_p

import torch  # noqa: F401  (must precede loading the HIP library)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("EVR_LIB_PATH") or os.path.join(_HERE, "_lib", "libeverest_amd.so")

c_double_p = c_void_p  # device / host pointers are passed as integers
c_int_p = c_void_p


class NativeLibraryError(RuntimeError):
    pass


class EvrQnehviState(ctypes.Structure):
    _fields_ = [
        ("n", c_int), ("nb", c_int), ("S", c_int), ("m", c_int),
        ("c", c_void_p), ("ym", c_void_p), ("ys", c_void_p), ("kxx", c_void_p),
        ("zq", c_void_p), ("obj_a", c_void_p), ("obj_b", c_void_p),
        ("cell_lo", c_void_p), ("cell_hi", c_void_p), ("cell_off", c_void_p), ("max_cells", c_int),
        ("cell_keys", c_void_p), ("cell_pts", c_void_p), ("cell_rank0", c_void_p), ("pts_stride", c_int),
        ("grp_off", c_void_p), ("grp_keys", c_void_p), ("grp_rank", c_void_p), ("grp_box", c_void_p),
        ("sorted_lo", c_void_p), ("max_groups", c_int), ("scan_counters", c_void_p), ("no_h", c_int),
        ("log_hvi", c_int), ("tau_relu", c_double), ("tau_max", c_double),
    ]


class EvrQnehviModel(ctypes.Structure):
    _fields_ = [
        ("n", c_int), ("d", c_int), ("kind", c_int),
        ("Xn", c_void_p), ("lengthscales", c_void_p), ("shift", c_void_p), ("scale", c_void_p), ("M", c_void_p),
    ]


class EvrQnGeneral(ctypes.Structure):
    _fields_ = [
        ("q", c_int), ("m_obj", c_int),
        ("obj_out", c_void_p), ("obj_kind", c_void_p), ("obj_p0", c_void_p), ("obj_p1", c_void_p),
        ("n_con", c_int),
        ("con_out", c_void_p), ("con_sign", c_void_p), ("con_thr", c_void_p), ("con_eta", c_void_p),
        ("zq", c_void_p),
    ]



_SIGS = {
    "evr_version": ([], c_int),
    "evr_last_error": ([], c_char_p),
    "evr_device_arch": ([c_int, c_char_p, c_int], c_int),
    "evr_stream_sync": ([c_void_p], c_int),
    "evr_kernel_matrix": ([c_void_p, c_int, c_int, c_int, c_int, c_int] + [c_void_p] * 10, c_int),
    "evr_kernel_cross_grad": ([c_void_p, c_int, c_int, c_int, c_int, c_int] + [c_void_p] * 11, c_int),
    "evr_kernel_cross_grad_workspace_doubles": ([c_int, c_int, c_int], c_longlong),
    "evr_kernel_lengthscale_grad": ([c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_void_p], c_int),
    "evr_gp_mll_terms": ([c_void_p, c_int, c_int] + [c_void_p] * 5, c_int),
    "evr_gemm_f64": ([c_void_p, c_int, c_int, c_int, c_int, c_int, c_double, c_void_p, c_int, c_longlong,
                      c_void_p, c_int, c_longlong, c_double, c_void_p, c_int, c_longlong, c_int], c_int),
    "evr_cholesky": ([c_void_p, c_int, c_int, c_void_p, c_int, c_longlong, c_void_p, c_int, c_longlong,
                      c_double, c_int, c_void_p, c_void_p], c_int),
    "evr_cholesky_inverse": ([c_void_p, c_int, c_int, c_void_p, c_int, c_longlong, c_void_p, c_int, c_longlong,
                              c_void_p, c_int, c_longlong, c_double, c_int, c_void_p, c_void_p], c_int),
    "evr_trsm_lower":([c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_longlong, c_int, c_void_p, c_int,
                        c_longlong], c_int),
    "evr_tri_inv_lower": ([c_void_p, c_int, c_int, c_void_p, c_int, c_longlong, c_void_p, c_int, c_longlong],
                          c_int),
    "evr_gp_posterior_finalize": ([c_void_p, c_int, c_int, c_int] + [c_void_p] * 8, c_int),
    "evr_gp_posterior_workspace_doubles": ([c_int, c_int, c_int], c_longlong),
    "evr_gp_posterior": ([c_void_p, c_int, c_int, c_int, c_int, c_int] + [c_void_p] * 14, c_int),
    "evr_qnehvi_samples": ([c_void_p, POINTER(EvrQnehviState), c_int, c_void_p, c_void_p, c_void_p, c_void_p],
                           c_int),
    "evr_hvi_workspace_doubles": ([POINTER(EvrQnehviState), c_int, c_int], c_longlong),
    "evr_hvi_forward": ([c_void_p, POINTER(EvrQnehviState), c_int, c_void_p, c_void_p, c_void_p, c_void_p],
                        c_int),
    "evr_mean_over_samples": ([c_void_p, c_int, c_int, c_void_p, c_void_p], c_int),
    "evr_hvi_backward": ([c_void_p, POINTER(EvrQnehviState), c_int, c_void_p, c_void_p, c_void_p, c_void_p],
                         c_int),
    "evr_qnehvi_samples_backward": ([c_void_p, POINTER(EvrQnehviState), c_int, c_void_p, c_void_p, c_void_p,
                                     c_void_p], c_int),
    "evr_pareto_mask": ([c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p], c_int),
    "evr_objective_affine": ([c_void_p, c_int, c_int, c_int] + [c_void_p] * 5, c_int),
    "evr_qei": ([c_void_p, c_int, c_int, c_int, c_void_p, c_double, c_double, c_double, c_double, c_void_p,
                 c_double, c_double, c_double, c_void_p, c_void_p, c_void_p], c_int),
    "evr_scale_batched":([c_void_p, c_int, c_longlong, c_void_p, c_void_p], c_int),
    "evr_add_selection": ([c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p], c_int),
    "evr_box_decompose": ([c_int, c_int, c_int, c_void_p, c_longlong, c_longlong, c_longlong, c_void_p,
                           c_void_p, c_int, POINTER(c_void_p)], c_int),
    "evr_box_decompose_approx": ([c_int, c_int, c_int, c_void_p, c_longlong, c_longlong, c_longlong, c_void_p,
                                  c_void_p, c_double, c_int, POINTER(c_void_p)], c_int),
    "evr_cells_total": ([c_void_p], c_longlong),
    "evr_cells_copy": ([c_void_p, c_void_p, c_void_p, c_void_p], c_int),
    "evr_cells_free": ([c_void_p], None),
    "evr_box_device_limits": ([c_int, c_int, c_void_p, c_void_p], c_int),
    "evr_box_device_workspace_bytes": ([c_int, c_int, c_int, c_int], c_longlong),
    "evr_box_decompose_device": ([c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                  c_void_p], c_int),
    "evr_box_pack_keys_device": ([c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                  c_void_p, c_void_p], c_int),
    "evr_box_kd_pipeline": ([c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int] + [c_void_p] * 8
                            + [c_int] + [c_void_p] * 6, c_int),
    "evr_cells_from_keys": ([c_void_p, c_int, c_int, c_int, c_void_p, c_int] + [c_void_p] * 5, c_int),
    "evr_hvi_forward_backward": ([c_void_p, POINTER(EvrQnehviState), c_int] + [c_void_p] * 6, c_int),
    "evr_hvi_restart_fb_applies": ([POINTER(EvrQnehviState), c_int], c_int),
    "evr_hvi_restart_fb": ([c_void_p, POINTER(EvrQnehviState), c_int] + [c_void_p] * 3, c_int),
    "evr_qnehvi_norms_rows": ([POINTER(EvrQnehviState)], c_int),
    "evr_qnehvi_project": ([c_void_p, POINTER(EvrQnehviState), c_int] + [c_void_p] * 5, c_int),
    "evr_qnehvi_project_workspace_doubles": ([POINTER(EvrQnehviState), c_int], c_longlong),
    "evr_qnehvi_samples_norms": ([c_void_p, POINTER(EvrQnehviState), c_int] + [c_void_p] * 5, c_int),
    "evr_qnehvi_project_backward": ([c_void_p, POINTER(EvrQnehviState), c_int] + [c_void_p] * 6, c_int),
    "evr_qnehvi_project_backward_workspace_doubles": ([POINTER(EvrQnehviState), c_int], c_longlong),
    "evr_qnehvi_plan_workspace_bytes": ([POINTER(EvrQnehviState), POINTER(EvrQnehviModel), c_int, c_int],
                                        c_longlong),
    "evr_qnehvi_plan_create": ([c_void_p, POINTER(EvrQnehviState), POINTER(EvrQnehviModel), c_int, c_int, c_void_p,
                               c_void_p, c_void_p, c_void_p, c_int, POINTER(c_void_p)], c_int),
    "evr_qnehvi_plan_run": ([c_void_p, c_void_p], c_int),
    "evr_qnehvi_small_applies": ([POINTER(EvrQnehviState), c_int, c_int], c_int),
    "evr_qnehvi_small_workspace_doubles": ([POINTER(EvrQnehviState), c_int, c_int, c_int], ctypes.c_longlong),
    "evr_qnehvi_small_forward": ([c_void_p, POINTER(EvrQnehviState), POINTER(EvrQnehviModel), c_int, c_void_p,
                                  c_void_p, c_void_p], c_int),
    "evr_qnehvi_small_samples": ([c_void_p, POINTER(EvrQnehviState), c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p], c_int),
    "evr_qnehvi_small_backward": ([c_void_p, POINTER(EvrQnehviState), POINTER(EvrQnehviModel), c_int, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_void_p], c_int),
    "evr_mll_plan_create": ([c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p], c_int),
    "evr_mll_plan_eval": ([c_void_p, c_void_p, c_void_p, c_void_p], c_int),
    "evr_mll_plan_destroy": ([c_void_p], None),
    "evr_mll_fit_rounds": ([c_void_p, c_void_p, c_void_p] + [c_void_p] * 7 + [c_int, c_int, c_void_p, c_void_p,
                                                                             c_void_p], c_int),
    "evr_mll_assemble": ([c_int, c_int, c_int] + [c_void_p] * 6, c_int),
    "evr_lbfgsb_advance": ([c_void_p, c_double] + [c_void_p] * 6 + [c_int, c_int], c_int),
    "evr_qnehvi_plan_eval_host": ([c_void_p, c_void_p, c_void_p, c_void_p], c_int),
    "evr_qnehvi_plan_destroy": ([c_void_p], None),
    "evr_lbfgsb_create": ([c_int, c_int, c_void_p, c_void_p, c_double, c_double, c_int, POINTER(c_void_p)], c_int),
    "evr_lbfgsb_start": ([c_void_p, c_void_p, c_void_p], c_int),
    "evr_lbfgsb_step": ([c_void_p, c_double, c_void_p, c_void_p], c_int),
    "evr_lbfgsb_stats": ([c_void_p, c_void_p, c_void_p, c_void_p, c_void_p], None),
    "evr_lbfgsb_destroy": ([c_void_p], None),
    "evr_hit_and_run": ([c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_longlong, ctypes.c_ulonglong,
                         c_longlong, c_longlong, c_void_p], c_int),
    "evr_qnehvi_plan_minimize": ([c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_double,
                                  c_double, c_int, c_int, c_void_p, c_void_p, c_void_p], c_int),
    "evr_qng_workspace_doubles": ([POINTER(EvrQnehviState), POINTER(EvrQnehviState), POINTER(EvrQnGeneral),
                                   POINTER(EvrQnehviModel), c_int, c_int], c_longlong),
    "evr_qng_eval": ([c_void_p, POINTER(EvrQnehviState), POINTER(EvrQnehviState), POINTER(EvrQnGeneral),
                      POINTER(EvrQnehviModel), c_int] + [c_void_p] * 5, c_int),
    "evr_qlog_workspace_doubles": ([POINTER(EvrQnehviState), POINTER(EvrQnehviState), POINTER(EvrQnGeneral),
                                    POINTER(EvrQnehviModel), c_int, c_int], ctypes.c_longlong),
    "evr_qlog_eval": ([c_void_p, POINTER(EvrQnehviState), POINTER(EvrQnehviState), POINTER(EvrQnGeneral),
                       POINTER(EvrQnehviModel), c_int] + [c_void_p] * 5, c_int),
    "evr_objective_general": ([c_void_p, c_int, c_int, c_int, POINTER(EvrQnGeneral)] + [c_void_p] * 4, c_int),
    "evr_objective_weights": ([c_void_p, c_int, c_int, POINTER(EvrQnGeneral)] + [c_void_p] * 3, c_int),
    "evr_cells_kd_limits": ([c_int, c_int, c_int, c_void_p], c_int),
    "evr_cells_kd_order_device": ([c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int] + [c_void_p] * 7,
                                  c_int),
    "evr_sobol_scramble": ([c_int, ctypes.c_ulonglong, c_void_p, c_void_p], c_int),
    "evr_sobol_scramble_range": ([c_int, ctypes.c_ulonglong, c_int, c_int, c_void_p, c_void_p], c_int),
    "evr_sobol_stream_words": ([c_int], ctypes.c_longlong),
    "evr_sobol_stream_create": ([ctypes.c_ulonglong, ctypes.c_longlong, c_void_p], c_int),
    "evr_sobol_scramble_stream": ([c_void_p, c_int, c_int, c_int, c_void_p, c_void_p], c_int),
    "evr_sobol_stream_destroy": ([c_void_p], None),
    "evr_sobol_normal": ([c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p], c_int),
}

EXPORTED_SYMBOLS = tuple(_SIGS)

_lib = None


def load() -> ctypes.CDLL:
    """Load (once) and return the native library; raise loudly if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryError(
            f"everest_amd native library not found at {LIB_PATH}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)."
        )
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


def check(status: int, what: str = ""):
    if status != 0:
        msg = load().evr_last_error().decode(errors="replace")
        raise RuntimeError(f"everest_amd {what} failed (status {status}): {msg}")


def call(name: str, *args):
    lib = load()
    check(getattr(lib, name)(*args), name)
