"""ctypes binding of libsgp.so (include/sgp.h).

There is no CPU fallback: if the HIP library is missing or cannot be loaded, every entry
point raises.  Compute entry points additionally require a visible GPU.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

from ._build import LIB, VARIANT_ROOT, HipccMissing, build

_lock = threading.Lock()
_lib = None

c_double_p = C.POINTER(C.c_double)
c_int_p = C.POINTER(C.c_int)

SGP_OK, SGP_EINVAL, SGP_ENOTPD, SGP_EHIP, SGP_ENOMEM = 0, 1, 2, 3, 4
KERNELS = {"sqexp": 0, "ard": 1, "exp": 2}
SGP_FLAG_R_DET = 1
SGP_FLAG_OBJ_ONLY = 2
SGP_PRED_VI, SGP_PRED_LAPLACE, SGP_PRED_FULL = 0, 1, 2
SGP_EXPO_ROWS = 0.0   # expo argument: the per-row exposure of sgp_lap_set_expo

# name -> (restype, argtypes); exactly the functions declared in include/sgp.h
PROTOTYPES = {
    "sgp_last_error": (C.c_char_p, []),
    "sgp_abi_version": (C.c_int, []),
    "sgp_device_count": (C.c_int, [c_int_p]),
    "sgp_num_params": (C.c_int, [C.c_int, C.c_int]),
    "sgp_make_cov": (C.c_int, [C.c_int, C.c_int, c_double_p, C.c_int64, C.c_int64, c_double_p,
                               C.c_int64, C.c_int64, C.c_int, c_double_p, C.c_double, c_double_p,
                               C.c_int64]),
    "sgp_dsig_dtheta": (C.c_int, [C.c_int, C.c_int, c_double_p, C.c_int64, C.c_int64, c_double_p,
                                  C.c_int64, C.c_int64, C.c_int, c_double_p, C.c_int, c_double_p,
                                  C.c_int64]),
    "sgp_kernel_pair": (C.c_double, [C.c_int, c_double_p, c_double_p, C.c_int, c_double_p]),
    "sgp_dkernel_pair": (C.c_double, [C.c_int, c_double_p, c_double_p, C.c_int, c_double_p,
                                      C.c_int]),
    "sgp_ctx_create": (C.c_int, [C.POINTER(C.c_void_p), C.c_int, c_double_p, C.c_int64, C.c_int64,
                                 C.c_int, c_double_p, c_double_p, C.c_int64]),
    "sgp_ctx_create_multi": (C.c_int, [C.POINTER(C.c_void_p), c_int_p, C.c_int, c_double_p,
                                       C.c_int64, C.c_int64, C.c_int, c_double_p, c_double_p,
                                       C.c_int64]),
    "sgp_ctx_shards": (C.c_int, [C.c_void_p, c_int_p, c_int_p]),
    "sgp_ctx_destroy": (C.c_int, [C.c_void_p]),
    "sgp_ctx_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "sgp_ctx_set_data": (C.c_int, [C.c_void_p, c_double_p, c_double_p]),
    "sgp_ctx_rows": (C.c_int64, [C.c_void_p]),
    "sgp_eval_vi": (C.c_int, [C.c_void_p, C.c_int, c_double_p, c_double_p, C.c_int64, C.c_int64,
                              C.c_double, C.c_uint, c_double_p, c_double_p]),
    "sgp_eval_fitc": (C.c_int, [C.c_void_p, C.c_int, c_double_p, c_double_p, C.c_int64, C.c_int64,
                                C.c_double, C.c_uint, c_double_p, c_double_p]),
    "sgp_vi_red1_count": (C.c_int64, [C.c_int64]),
    "sgp_vi_red1_packed_count": (C.c_int64, [C.c_int64]),
    "sgp_ctx_set_packed_reduction": (C.c_int, [C.c_void_p, C.c_int]),
    "sgp_vi_red2_count": (C.c_int64, [C.c_int, C.c_int]),
    "sgp_vi_phase1": (C.c_int, [C.c_void_p, C.c_int, c_double_p, c_double_p, C.c_int64, C.c_int64,
                                C.c_double, C.c_void_p]),
    "sgp_vi_phase2": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_uint, C.c_void_p]),
    "sgp_vi_finish": (C.c_int, [C.c_void_p, C.c_void_p, c_double_p, c_double_p]),
    "sgp_fitc_red1_count": (C.c_int64, [C.c_int64]),
    "sgp_fitc_red2_count": (C.c_int64, [C.c_int, C.c_int, C.c_int64]),
    "sgp_fitc_phase1": (C.c_int, [C.c_void_p, C.c_int, c_double_p, c_double_p, C.c_int64, C.c_int64,
                                  C.c_double, C.c_void_p]),
    "sgp_fitc_phase2": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_uint, C.c_void_p]),
    "sgp_fitc_finish": (C.c_int, [C.c_void_p, C.c_void_p, c_double_p, c_double_p]),
    "sgp_lap_set_f": (C.c_int, [C.c_void_p, c_double_p, C.c_double]),
    "sgp_lap_set_expo": (C.c_int, [C.c_void_p, c_double_p, C.c_double]),
    # include/sgp_diag.h (diagnostics: GPU tests and bench.py)
    "sgp_diag_gj_pair": (C.c_int, [C.c_int, C.c_int64, c_double_p, c_double_p, C.c_double, C.c_int,
                                   c_double_p, c_double_p, c_double_p]),
    "sgp_diag_store_bw": (C.c_int, [C.c_int, C.c_int64, C.c_int, C.c_int, c_double_p]),
    "sgp_lap_get_f": (C.c_int, [C.c_void_p, c_double_p]),
    "sgp_lap_get_grad_psi": (C.c_int, [C.c_void_p, c_double_p]),
    "sgp_lap_objective_values": (C.c_int, [C.c_void_p, c_double_p, C.c_int, c_int_p]),
    "sgp_eval_laplace": (C.c_int, [C.c_void_p, C.c_int, c_double_p, c_double_p, C.c_int64,
                                   C.c_int64, C.c_double, C.c_double, C.c_double, C.c_int,
                                   c_double_p, c_double_p, c_int_p]),
    "sgp_lap_red_count": (C.c_int64, [C.c_int, C.c_int, C.c_int64]),
    "sgp_lap_begin": (C.c_int, [C.c_void_p, C.c_int, c_double_p, c_double_p, C.c_int64, C.c_int64,
                                C.c_double, C.c_double, C.c_double, C.c_int, C.c_uint,
                                C.c_void_p, C.POINTER(C.c_int64)]),
    "sgp_lap_step": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_int64), c_int_p,
                               c_double_p, c_double_p, c_int_p]),
    "sgp_lap_nr": (C.c_int, [C.c_void_p, C.c_int, c_double_p, c_double_p, C.c_int64, C.c_int64,
                             C.c_double, C.c_double, C.c_double, C.c_int, c_double_p, c_int_p]),
    "sgp_eval_full": (C.c_int, [C.c_void_p, C.c_int, c_double_p, C.c_double, C.c_uint,
                                c_double_p, c_double_p]),
    "sgp_posterior_u": (C.c_int, [C.c_void_p, c_double_p, c_double_p, c_double_p]),
    "sgp_predict": (C.c_int, [C.c_int, C.c_int, c_double_p, C.c_double, C.c_int, C.c_int, c_double_p,
                              C.c_int64, C.c_int64, c_double_p, c_double_p, c_double_p, C.c_int64,
                              c_double_p, C.c_int64, C.c_int64, C.c_int, c_double_p, C.c_int,
                              c_double_p, c_double_p, C.c_int64]),
    "sgp_ctx_enable_knot_grad": (C.c_int, [C.c_void_p, C.c_int]),
    "sgp_knot_red_extra": (C.c_int64, [C.c_int, C.c_int64]),
    "sgp_knot_gradient": (C.c_int, [C.c_void_p, c_double_p, c_double_p]),
    "sgp_ctx_row_bounds": (C.c_int, [C.c_void_p, c_double_p, c_double_p]),
    "sgp_vi_candidates": (C.c_int, [C.c_void_p, C.c_int, c_double_p, c_double_p, C.c_int64,
                                    C.c_int64, C.c_double, C.c_uint, c_double_p, C.c_int64,
                                    C.c_int64, c_double_p]),
    "sgp_fitc_candidates": (C.c_int, [C.c_void_p, C.c_int, c_double_p, c_double_p, C.c_int64,
                                      C.c_int64, C.c_double, C.c_uint, c_double_p, C.c_int64,
                                      C.c_int64, c_double_p]),
    "sgp_lap_candidates": (C.c_int, [C.c_void_p, C.c_int, c_double_p, c_double_p, C.c_int64,
                                     C.c_int64, C.c_double, C.c_double, C.c_double, C.c_int,
                                     c_double_p, C.c_int64, C.c_int64, c_double_p]),
    "sgp_ctx_enable_timing": (C.c_int, [C.c_void_p, C.c_int]),
    "sgp_ctx_timing_filter": (C.c_int, [C.c_void_p, C.c_char_p]),
    "sgp_ctx_timing_evals": (C.c_int64, [C.c_void_p]),
    "sgp_ctx_timings": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int64, c_double_p, C.c_int, c_int_p]),
}


class SGPError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"sgp status {status}: {msg}")
        self.status = status


class NotPositiveDefinite(SGPError):
    """R's chol() failure (caught by try() in the reference's knot proposals)."""


def _ab_lib():
    """SGP_AB_LIB: an experiment library built by _build.build_variant() (tools/ab/<name>/),
    for A/B timing runs only.  Any other path is refused, so the variable cannot point the
    product at an arbitrary binary."""
    p = os.environ.get("SGP_AB_LIB")
    if not p:
        return None
    p = os.path.realpath(p)
    root = os.path.realpath(VARIANT_ROOT) + os.sep
    if not p.startswith(root):
        raise RuntimeError(f"SGP_AB_LIB must name a library under {root} (got {p})")
    return p


def lib(auto_build: bool = True):
    """Load (building if needed) libsgp.so.  Raises if it cannot be loaded."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = _ab_lib()
        if path is None and auto_build:
            # rebuilds when a source or header is newer than an object or its compile command
            # changed (a stale .so would otherwise be loaded silently).  Only a missing hipcc
            # lets the existing library be used; a compile or link error always propagates.
            try:
                build()
            except HipccMissing:
                if not os.path.exists(LIB):
                    raise
        path = path or LIB
        if not os.path.exists(path):
            raise RuntimeError(f"libsgp.so not found at {path}; run sparsergps_amd._build.build()")
        h = C.CDLL(path, mode=C.RTLD_GLOBAL)
        ab = path != LIB
        for name, (res, args) in PROTOTYPES.items():
            if ab and not hasattr(h, name):   # an A/B library of an older revision
                continue
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _lib = h
        return h


def check(status: int):
    if status == SGP_OK:
        return
    msg = lib().sgp_last_error().decode(errors="replace")
    if status == SGP_ENOTPD:
        raise NotPositiveDefinite(status, msg)
    raise SGPError(status, msg)


def dptr(a):
    return a.ctypes.data_as(c_double_p)


def require_gpu():
    n = C.c_int(0)
    st = lib().sgp_device_count(C.byref(n))
    if st != SGP_OK or n.value < 1:
        raise RuntimeError("sparsergps_amd: no HIP device visible (the MI355X path has no CPU fallback)")
    return n.value
