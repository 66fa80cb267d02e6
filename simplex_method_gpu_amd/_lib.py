"""ctypes loader for libsimplex.so (the C-ABI of include/simplex.h).

The HIP path is the only compute path: if the library is missing or cannot be
loaded this raises — there is no CPU fallback in the product.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# SPX_LIB: alternative build of the same library (e.g. a cache-policy variant
# from a cache-policy sweep; tools/pass_ab.py); default is the in-tree product build.
LIB_PATH = os.environ.get("SPX_LIB") or os.path.join(_HERE, "libsimplex.so")

# symbol -> (restype, argtypes); mirrors include/simplex.h
_d, _i32, _i64, _u64, _p = ctypes.c_double, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_void_p
_pp = ctypes.POINTER(ctypes.c_void_p)


class SpxOpts(ctypes.Structure):
    _fields_ = [
        ("eps", ctypes.c_double),
        ("device", ctypes.c_int32),
        ("rank", ctypes.c_int32),
        ("nranks", ctypes.c_int32),
        ("graph_batch", ctypes.c_int32),
        ("price_block", ctypes.c_int32),
        ("update_rows", ctypes.c_int32),
        ("price_grid", ctypes.c_int32),
        ("flags", ctypes.c_int32),
        ("update_block", ctypes.c_int32),
        ("window", ctypes.c_int32),
        ("ratio_test", ctypes.c_int32),
        ("refactor_every", ctypes.c_int32),
        ("piv_tol", ctypes.c_double),
        ("feas_tol", ctypes.c_double),
        ("pricing", ctypes.c_int32),
        ("loop_block", ctypes.c_int32),
        ("trace_cap", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


SIGNATURES = {
    "spx_default_opts": (None, [ctypes.POINTER(SpxOpts)]),
    "spx_create": (ctypes.c_int, [_pp, _i64, _i64, _p, _p, _p, ctypes.POINTER(SpxOpts)]),
    "spx_create_generated": (ctypes.c_int, [_pp, _i64, _i64, _u64, ctypes.POINTER(SpxOpts)]),
    "spx_destroy": (None, [_p]),
    "spx_comm_unique_id": (ctypes.c_int, [_p]),
    "spx_attach_comm": (ctypes.c_int, [_p, _p]),
    "spx_comm_info": (ctypes.c_int, [_p, _p, _p]),
    "spx_mbox_export": (ctypes.c_int, [_p, _p]),
    "spx_ftran_cols": (ctypes.c_int, [_p, _p]),
    "spx_mbox_attach": (ctypes.c_int, [_p, _p]),
    "spx_reset": (ctypes.c_int, [_p]),
    "spx_reinvert": (ctypes.c_int, [_p]),
    "spx_set_basis": (ctypes.c_int, [_p, _p]),
    "spx_group_iterate": (ctypes.c_int, [_p, _i32, _i64, _p, _p]),
    "spx_group_sync": (ctypes.c_int, [_p, _i32]),
    "spx_solve": (ctypes.c_int, [_p, _i64, _p, _p, _p, _p, _p]),
    "spx_iterate": (ctypes.c_int, [_p, _i64, _p, _p]),
    "spx_price": (ctypes.c_int, [_p, _p, _p, _p]),
    "spx_pivot": (ctypes.c_int, [_p, _p, _p]),
    "spx_dispatch_stats": (ctypes.c_int, [_p, _p]),
    "spx_prepare": (ctypes.c_int, [_p]),
    "spx_get_trace": (ctypes.c_int, [_p, _p, _p, _i64, _p]),
    "spx_get_weights": (ctypes.c_int, [_p, _p]),
    "spx_get_state": (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _p, _p]),
    "spx_reduced_costs": (ctypes.c_int, [_p, _p]),
    "spx_objective": (ctypes.c_int, [_p, _p]),
    "spx_kernel_times": (ctypes.c_int, [_p, _p, _p, _p, _p]),
    "spx_pass_times": (ctypes.c_int, [_p, _p, _p]),
    "spx_info": (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _p]),
    "spx_config": (ctypes.c_int, [_p, _p]),
    "spx_phase_times": (ctypes.c_int, [_p, _p]),
    "spx_wg_times": (ctypes.c_int, [_p, _p, _i64, _p]),
    "spx_fold_times": (ctypes.c_int, [_p, _p, _i64, _p]),
    "spx_loop_times": (ctypes.c_int, [_p, _p, _p]),
    "spx_shard_range": (ctypes.c_int, [_i64, _i64, _i32, _i32, _p]),
    "spx_minloc_merge": (ctypes.c_int, [_p, _p, _i32, _p, _p]),
    "spx_last_error": (ctypes.c_char_p, []),
    "spx_status_string": (ctypes.c_char_p, [_i32]),
    "spx_abi_version": (ctypes.c_int, []),
}

_lib = None


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} not found: build the HIP extension first (`make` or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


class SimplexError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libsimplex error {code}: {msg}")
        self.code = code


def check(rc: int) -> None:
    if rc != 0:
        raise SimplexError(rc, load().spx_last_error().decode(errors="replace"))
