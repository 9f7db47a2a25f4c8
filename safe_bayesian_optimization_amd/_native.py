"""ctypes binding of libsbo.so (the C ABI declared in include/sbo.h).

The library is built in-tree (``make -C safe_bayesian_optimization_amd``) and
loaded from ``safe_bayesian_optimization_amd/lib/libsbo.so``.  There is no
fallback: if the library is missing or fails to load, every entry point
raises.  torch (when importable) is imported first so that libsbo.so binds to
the same HIP runtime instance torch uses (identical SONAMEs).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SBO_LIB") or os.path.join(_PKG, "lib", "libsbo.so")  # SBO_LIB: instrumented builds (tools/)

SBO_DEVICE_PTRS = 0x1
SBO_ASYNC = 0x2
SCORE_WIDTH = 0
SCORE_UCB = 1
SBO_E_STATE = 6

STATUS = {0: "SBO_OK", 1: "SBO_E_INVAL", 2: "SBO_E_NOT_SPD", 3: "SBO_E_DEVICE", 4: "SBO_E_OOM",
          5: "SBO_E_EMPTY", 6: "SBO_E_STATE"}

# Every symbol include/sbo.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "sbo_version", "sbo_status_string", "sbo_create", "sbo_destroy", "sbo_set_stream", "sbo_last_error",
    "sbo_fit", "sbo_append", "sbo_num_train", "sbo_predict", "sbo_compute_sets", "sbo_compute_sets_f64", "sbo_argmax", "sbo_tick",
    "sbo_key_combine", "sbo_find_safety_contour_indices", "sbo_next_subgoal", "sbo_find_contours_external",
    "sbo_rbf_fill", "sbo_get_factor", "sbo_profile", "sbo_profile_read", "sbo_set_option", "sbo_get_inverse",
    "sbo_get_order", "sbo_profile_work", "sbo_profile_mfma", "sbo_debug_x3_stamps", "sbo_get_skip", "sbo_frontier", "sbo_subgoal",
    "sbo_get_bounds", "sbo_get_jitter", "sbo_get_tile_bounds", "sbo_state_bytes", "sbo_export_state", "sbo_import_state", "sbo_query_cost",
    "sbo_polygon_correct", "sbo_polydist", "sbo_point_within", "sbo_project_subgoal", "sbo_get_precision",
    "sbo_kd_order", "sbo_get_probe", "sbo_keys_reduce", "sbo_get_inverse_check", "sbo_trim", "sbo_warmup",
)
SBO_OPT_INVERSE_BITS = 1
SBO_OPT_SPATIAL_ORDER = 2
SBO_OPT_TILE_SKIP = 3
SBO_OPT_QUERY_ORDER = 4
SBO_OPT_KERNEL_VARIANT = 5
SBO_OPT_SWEEP_GROUPS = 6
SBO_OPT_SKIP_BUDGET = 7
SBO_OPT_CHOLESKY = 8
SBO_OPT_INVERSE = 9
SBO_OPT_JITTER_RETRIES = 10
SBO_OPT_PRECISION = 11
SBO_OPT_RESORT = 12
SBO_OPT_CHOL_RESERVE = 13
SBO_OPT_INV_OVERLAP = 14
SBO_OPT_CHOL_OUTER = 15
SBO_OPT_CHOL_DIAG = 16
SBO_OPT_CHOL_GEMM = 17
SBO_OPT_INV_BASE = 18
SBO_OPT_INV_PANELS = 19
SBO_OPT_INV_LEAVES = 20
SBO_OPT_REPROBE = 21
SBO_OPT_PRECISE_KERNEL = 22
SBO_OPT_TABLE_MB = 23
SBO_OPT_INV_OZ = 24
SBO_OPT_INV_CHECK = 25
SBO_OPT_PLAN_BLOCK = 26
SBO_OPT_PROBE_SIZE = 27
SBO_OPT_INV_OZ_MIN = 28
SBO_OPT_INV_OZ_ADAPT = 29


class SboError(RuntimeError):
    def __init__(self, status: int, message: str = ""):
        self.status = status
        super().__init__(f"{STATUS.get(status, status)}: {message}")


class NotSPDError(SboError):
    pass


class sbo_hyper(ctypes.Structure):
    _fields_ = [("length_scale", ctypes.c_double), ("sigma_f", ctypes.c_double),
                ("noise_level", ctypes.c_double), ("prior_mean", ctypes.c_double)]


class sbo_key(ctypes.Structure):
    _fields_ = [("score", ctypes.c_double), ("idx", ctypes.c_int64)]


class sbo_probe(ctypes.Structure):
    _fields_ = [("precise", ctypes.c_int32), ("m_grid", ctypes.c_int32), ("m_train", ctypes.c_int32),
                ("precise_kernel", ctypes.c_int32), ("n_at_probe", ctypes.c_int64), ("err", ctypes.c_double),
                ("err_grid", ctypes.c_double), ("err_train", ctypes.c_double), ("var_min", ctypes.c_double),
                ("var_max", ctypes.c_double), ("var_max_grid", ctypes.c_double), ("var_max_train", ctypes.c_double)]


class sbo_inv_check(ctypes.Structure):
    _fields_ = [("ran", ctypes.c_int32), ("fired", ctypes.c_int32), ("digits", ctypes.c_int32), ("m", ctypes.c_int32),
                ("err", ctypes.c_double), ("err_grid", ctypes.c_double), ("err_train", ctypes.c_double),
                ("err_fallback", ctypes.c_double), ("tol", ctypes.c_double), ("var_max", ctypes.c_double),
                ("ms", ctypes.c_double), ("err_mean", ctypes.c_double), ("mean_max", ctypes.c_double),
                ("err_mean_fallback", ctypes.c_double), ("kept_digits", ctypes.c_int32), ("reserved", ctypes.c_int32)]


_lib = None


def build(jobs: int = 8) -> str:
    subprocess.run(["make", "-s", "-j", str(jobs), "-C", _PKG], check=True)
    return LIB_PATH


def lib():
    """Load libsbo.so (raises if it is missing: no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    try:  # share torch's HIP runtime when both live in one process
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libsbo.so not built: {LIB_PATH} (run `make -C {_PKG}` or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    vp, i64, u32, dbl, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint32, ctypes.c_double, ctypes.c_int
    st = ctypes.c_int
    L.sbo_version.restype = ctypes.c_char_p
    L.sbo_status_string.argtypes = [st]
    L.sbo_status_string.restype = ctypes.c_char_p
    L.sbo_create.argtypes = [i32, ctypes.POINTER(vp)]
    L.sbo_create.restype = st
    L.sbo_destroy.argtypes = [vp]
    L.sbo_destroy.restype = None
    L.sbo_set_stream.argtypes = [vp, vp]
    L.sbo_set_stream.restype = st
    L.sbo_last_error.argtypes = [vp]
    L.sbo_last_error.restype = ctypes.c_char_p
    L.sbo_fit.argtypes = [vp, vp, vp, vp, i64, sbo_hyper, u32]
    L.sbo_fit.restype = st
    L.sbo_append.argtypes = [vp, vp, vp, vp, i64, u32]
    L.sbo_append.restype = st
    L.sbo_num_train.argtypes = [vp]
    L.sbo_num_train.restype = i64
    L.sbo_predict.argtypes = [vp, vp, vp, i64, vp, vp, u32]
    L.sbo_predict.restype = st
    L.sbo_compute_sets.argtypes = [vp, vp, vp, i64, dbl, dbl, vp, vp, vp, u32]
    L.sbo_compute_sets.restype = st
    L.sbo_compute_sets_f64.argtypes = [vp, vp, vp, i64, dbl, dbl, vp, vp, vp, u32]
    L.sbo_compute_sets_f64.restype = st
    L.sbo_argmax.argtypes = [vp, vp, vp, i64, i64, ctypes.POINTER(sbo_key), u32]
    L.sbo_argmax.restype = st
    L.sbo_tick.argtypes = [vp, vp, vp, i64, dbl, dbl, i32, i64, vp, vp, vp, vp, vp, vp, u32]
    L.sbo_tick.restype = st
    L.sbo_query_cost.argtypes = [vp, vp, vp, i64, vp, u32]
    L.sbo_query_cost.restype = st
    L.sbo_key_combine.argtypes = [sbo_key, sbo_key]
    L.sbo_key_combine.restype = sbo_key
    L.sbo_keys_reduce.argtypes = [vp, vp, i64, vp, u32]
    L.sbo_keys_reduce.restype = st
    L.sbo_find_safety_contour_indices.argtypes = [vp, vp, vp, i64, i32, i32, vp, i64, ctypes.POINTER(i64)]
    L.sbo_find_safety_contour_indices.restype = st
    L.sbo_next_subgoal.argtypes = [vp, vp, vp, vp, vp, i64, i32, i32, dbl, dbl]
    L.sbo_next_subgoal.restype = i64
    L.sbo_frontier.argtypes = [vp, vp, vp, vp, i64, i32, i32, vp, i64, ctypes.POINTER(i64), u32]
    L.sbo_frontier.restype = st
    L.sbo_subgoal.argtypes = [vp, vp, vp, vp, vp, vp, i64, i32, i32, dbl, dbl, ctypes.POINTER(i64), u32]
    L.sbo_subgoal.restype = st
    L.sbo_get_tile_bounds.argtypes = [vp, vp, i64]
    L.sbo_get_tile_bounds.restype = st
    L.sbo_get_bounds.argtypes = [vp, vp]
    L.sbo_get_bounds.restype = st
    L.sbo_get_jitter.argtypes = [vp, ctypes.POINTER(dbl)]
    L.sbo_get_jitter.restype = st
    L.sbo_state_bytes.argtypes = [vp, ctypes.POINTER(i64)]
    L.sbo_state_bytes.restype = st
    L.sbo_export_state.argtypes = [vp, vp, i64]
    L.sbo_export_state.restype = st
    L.sbo_import_state.argtypes = [vp, vp, i64]
    L.sbo_import_state.restype = st
    L.sbo_find_contours_external.argtypes = [vp, i32, i32, vp, i64, vp, i64]
    L.sbo_find_contours_external.restype = i64
    L.sbo_rbf_fill.argtypes = [vp, vp, vp, i64, sbo_hyper, vp, u32]
    L.sbo_rbf_fill.restype = st
    L.sbo_get_factor.argtypes = [vp, vp, vp, u32]
    L.sbo_get_factor.restype = st
    L.sbo_set_option.argtypes = [vp, i32, i64]
    L.sbo_set_option.restype = st
    L.sbo_get_skip.argtypes = [vp, ctypes.POINTER(i32), ctypes.POINTER(dbl), ctypes.POINTER(dbl)]
    L.sbo_get_skip.restype = st
    L.sbo_get_precision.argtypes = [vp, ctypes.POINTER(i32), ctypes.POINTER(dbl), ctypes.POINTER(dbl),
                                    ctypes.POINTER(dbl)]
    L.sbo_get_precision.restype = st
    L.sbo_get_probe.argtypes = [vp, ctypes.POINTER(sbo_probe)]
    L.sbo_get_probe.restype = st
    L.sbo_get_inverse_check.argtypes = [vp, ctypes.POINTER(sbo_inv_check)]
    L.sbo_get_inverse_check.restype = st
    L.sbo_trim.argtypes = [vp]
    L.sbo_trim.restype = st
    L.sbo_warmup.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, sbo_hyper]
    L.sbo_warmup.restype = st
    L.sbo_get_order.argtypes = [vp, vp]
    L.sbo_get_order.restype = st
    L.sbo_kd_order.argtypes = [vp, vp, i64, i64, vp]
    L.sbo_kd_order.restype = st
    L.sbo_get_inverse.argtypes = [vp, vp]
    L.sbo_get_inverse.restype = st
    L.sbo_profile.argtypes = [vp, i32]
    L.sbo_profile.restype = st
    L.sbo_profile_read.argtypes = [vp, ctypes.POINTER(dbl), ctypes.POINTER(i64), ctypes.POINTER(dbl),
                                   ctypes.POINTER(i64)]
    L.sbo_profile_read.restype = st
    L.sbo_profile_work.argtypes = [vp, ctypes.POINTER(dbl)]
    L.sbo_profile_work.restype = st
    L.sbo_profile_mfma.argtypes = [vp, ctypes.POINTER(dbl), ctypes.POINTER(i64)]
    L.sbo_profile_mfma.restype = st
    L.sbo_debug_x3_stamps.argtypes = [vp, ctypes.POINTER(dbl), ctypes.c_int]
    L.sbo_debug_x3_stamps.restype = st
    pd = ctypes.POINTER(dbl)
    L.sbo_polygon_correct.argtypes = [vp, vp, i64, i64, ctypes.POINTER(i64)]
    L.sbo_polygon_correct.restype = st
    L.sbo_polydist.argtypes = [vp, vp, i64, dbl, dbl, pd, pd, pd]
    L.sbo_polydist.restype = st
    L.sbo_point_within.argtypes = [vp, vp, i64, dbl, dbl]
    L.sbo_point_within.restype = ctypes.c_int
    L.sbo_project_subgoal.argtypes = [vp, vp, i64, dbl, dbl, i64, vp, vp, i64, pd, pd, pd]
    L.sbo_project_subgoal.restype = ctypes.c_int
    _lib = L
    return L


def check(status: int, ctx=None) -> None:
    if status == 0:
        return
    msg = ""
    if ctx is not None:
        msg = lib().sbo_last_error(ctx).decode(errors="replace")
    if status == 2:
        raise NotSPDError(status, msg)
    raise SboError(status, msg)
