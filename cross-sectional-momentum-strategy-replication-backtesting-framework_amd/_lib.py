"""ctypes binding of libcsmom.so (the C ABI declared in include/csmom.h).

The library is built in-tree (``python -c "import __graft_entry__ as g; g.build()"`` or
``make -C <pkg>/csrc``).  There is no fallback: if the shared object is missing or cannot
be loaded, every compute entry point raises ``CsmUnavailable``.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

LIB_NAME = "libcsmom.so"
PKG_DIR = Path(__file__).resolve().parent
CSM_OK = 0
CSM_E_INVAL = -1
CSM_E_HIP = -2
CSM_E_RCCL = -3
CSM_E_TIMEOUT = -4
UNIQUE_ID_BYTES = 128
ABSENT_BITS = 0x7FF4000000000001

class CsmUnavailable(RuntimeError):
    """libcsmom.so is missing or failed to load (the engine has no CPU fallback)."""


class CsmError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"csmom status {status}: {msg}")
        self.status = status


def lib_path() -> Path:
    return Path(os.environ.get("CSMOM_LIB", PKG_DIR / LIB_NAME))


_LIB = None

_p = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_f64 = ctypes.c_double


# ctypes prototypes of every entry point include/csmom.h declares (tests/test_abi_boundary.py
# checks them against the header's parameter lists)
SIGNATURES = {
    "csm_abi_version": (ctypes.c_int, []),
    "csm_tune": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int]),
    "csm_tune_ptr": (ctypes.c_int, [ctypes.c_char_p, _p]),
    "csm_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "csm_destroy": (ctypes.c_int, [_p]),
    "csm_last_error": (ctypes.c_char_p, [_p]),
    "csm_set_stream": (ctypes.c_int, [_p, _p]),
    "csm_sync": (ctypes.c_int, [_p]),
    "csm_month_end": (ctypes.c_int, [_p, _p, _p, _i64, _i64, _p, _i32, _p, _p]),
    "csm_momentum": (ctypes.c_int, [_p, _p, _i32, _i64, _i32, _i32, _p, _p, _p, _p, _p, _p]),
    "csm_momentum_multi": (ctypes.c_int, [_p, _p, _i32, _i64, _p, _i32, _i32, _p, _p]),
    "csm_momentum_multi_ids": (ctypes.c_int, [_p, _p, _i32, _i64, _p, _i32, _i32, _p, _p, _p]),
    "csm_signal": (ctypes.c_int, [_p, _p, _i64, _i64, _p, _i32, _i32, _i32, _i32, _p, _p, _p, _p,
                                  _p, _p, _p]),
    "csm_portfolio_workspace": (ctypes.c_int64, [_i32, _i32, _i64, _i32, _i32]),
    "csm_portfolio": (ctypes.c_int, [_p, _p, _p, _p, _i32, _i32, _i64, _i32, _i32, _f64, _f64,
                                     _f64, _p, _p, _p, _p, _p, _p, _p, _p]),
    "csm_cohort_sums": (ctypes.c_int, [_p, _p, _p, _p, _i32, _i32, _i64, _i32, _i32, _p]),
    "csm_portfolio_from_cohorts": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _i64, _i32, _i32,
                                                  _i32, _f64, _f64, _f64, _p, _p, _p, _p,
                                                  _p, _p, _p, _p]),
    "csm_turnover_features": (ctypes.c_int, [_p, _p, _p, _p, _p, _i32, _i64, _i32, _p, _p, _p,
                                             _p]),
    "csm_double_sort_labels": (ctypes.c_int, [_p, _p, _p, _p, _p, _i32, _i64, _i32, _p, _p]),
    "csm_portfolio_from_cohorts_multi": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _i64, _i32,
                                                        _i32, _i32, _p, _f64, _f64, _f64, _p,
                                                        _p, _p, _p, _p, _p, _p, _p]),
    "csm_cohort_sums_legs": (ctypes.c_int, [_p, _p, _p, _p, _i32, _i32, _i64, _i32, _i32, _p]),
    "csm_cohort_sums_js": (ctypes.c_int, [_p, _i32, _p, _p, _i32, _i32, _i64, _i32, _i32, _i32,
                                          _p]),
    "csm_portfolio_from_cohorts_legs": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _i64, _i32,
                                                       _i32, _i32, _p, _f64, _f64, _f64, _p,
                                                       _p, _p, _p, _p, _p, _p, _p, _p]),
    "csm_cohort_sums_grouped": (ctypes.c_int, [_p, _i32, _p, _p, _p, _i32, _i32, _i64, _i32,
                                               _i32, _i32, _p]),
    "csm_cohort_sums_js_grouped": (ctypes.c_int, [_p, _i32, _p, _p, _i32, _i32, _i64, _i32,
                                                  _i32, _i32, _p]),
    "csm_portfolio_plan": (ctypes.c_int64, [_i32, _i32, _i64, _i32, _i32]),
    "csm_portfolio_from_cohorts_grouped": (ctypes.c_int, [_p, _i32, _p, _p, _i32, _i32, _i64,
                                                          _i32, _i32, _i32, _p, _f64, _f64, _f64,
                                                          _p, _p, _p, _p, _p, _p, _p, _p, _i32,
                                                          _p]),
    "csm_summary": (ctypes.c_int, [_p, _p, _p, _p, _p, _i32, _i32, _i32, _f64, _p]),
    "csm_bootstrap": (ctypes.c_int, [_p, _p, _i32, _i64, _i32, _i64, ctypes.c_uint64, _f64,
                                     _f64, _p, _p]),
    "csm_boot_scan": (ctypes.c_int, [_p, _p, _i32, _i64, _i32, _i64, ctypes.c_uint64, _f64, _f64,
                                     _p, _i32, _i32, _p, _p, _p, _p, _p]),
    "csm_momentum_chunked": (ctypes.c_int, [_p, _p, _i32, _i64, _i32, _i32, _i32, _p, _p, _p,
                                            _p, _p]),
    "csm_signal_chunked_workspace": (ctypes.c_int64, [_i32, _i64, _i32, _i32, _i32]),
    "csm_signal_chunked": (ctypes.c_int, [_p, _p, _i64, _i64, _p, _i32, _i32, _i32, _i32, _i32,
                                          _p, _p, _p, _p, _p]),
    "csm_signal_chunked_status": (ctypes.c_int, [_p, _p]),
    "csm_momentum_chunked_workspace": (ctypes.c_int64, [_i32, _i64, _i32, _i32, _i32]),
    "csm_momentum_multi_chunked_workspace": (ctypes.c_int64, [_i32, _i64, _i32, _i32, _i32]),
    "csm_momentum_multi_chunked": (ctypes.c_int, [_p, _p, _i32, _i64, _p, _i32, _i32, _i32, _p,
                                                  _p, _p, _p]),
    "csm_momentum_chunked_ids": (ctypes.c_int, [_p, _p, _i32, _i64, _i32, _i32, _i32, _p, _p,
                                                _p, _p, _p, _p]),
    "csm_deciles": (ctypes.c_int, [_p, _p, _p, _i32, _i64, _i32, _p, _p, _p, _p, _p]),
    "csm_long_short": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _p]),
    "csm_shard_summary": (ctypes.c_int, [_p, _p, _i32, _i64, _i32, _i32, _p]),
    "csm_fold_carry": (ctypes.c_int, [_p, _p, _i32, _i32, _i64, _i32, _i32, _p, _p]),
    "csm_shard_repair": (ctypes.c_int, [_p, _p, _p, _p, _i32, _i64, _i32, _i32, _p, _p, _p,
                                        _p, _p, _p]),
    "csm_signal_shard": (ctypes.c_int, [_p, _p, _i64, _i64, _p, _i32, _i32, _i32, _i32, _p,
                                        _p, _p, _p, _p]),
    "csm_signal_shard_ids": (ctypes.c_int, [_p, _p, _i64, _i64, _p, _i32, _i32, _i32, _i32,
                                            _p, _p, _p, _p, _p, _p]),
    "csm_shard_repair_ids": (ctypes.c_int, [_p, _p, _p, _p, _i32, _i64, _i32, _i32, _p, _p,
                                            _p, _p, _p, _p, _p]),
    "csm_shard_summary_state": (ctypes.c_int, [_p, _p, _p, _p, _i32, _i64, _i32, _i32, _p,
                                               _p]),
    "csm_shard_halo": (ctypes.c_int, [_p, _p, _i64, _i64, _p, _i32, _i32, _i32, _i32, _i32, _i32,
                                      _i32, _p, _p, _p, _p]),
    "csm_signal_shard_halo": (ctypes.c_int, [_p, _p, _i64, _i64, _p, _i32, _i32, _i32, _i32, _p,
                                             _p, _p, _p, _p, _p, _p, _p]),
    "csm_shard_need": (ctypes.c_int, [_p, _p, _p, _i64, _i32, _i32, _p]),
    "csm_shard_union": (ctypes.c_int, [_p, _p, _i32, _i64, _i64, _p, _p]),
    "csm_shard_summary_cols": (ctypes.c_int, [_p, _p, _p, _p, _i32, _i64, _i32, _i32, _p, _p,
                                              _p, _i64, _p]),
    "csm_shard_repair_cols": (ctypes.c_int, [_p, _p, _p, _p, _i32, _i64, _i32, _i32, _p, _p, _p,
                                             _p, _p, _p, _i64, _p, _p, _p, _p]),
    "csm_signal_halo": (ctypes.c_int, [_p, _p, _i64, _i64, _p, _i32, _i32, _i32, _i32, _i32, _i32,
                                       _i32, _i32, _p, _p, _p, _p, _p, _p, _p]),
    "csm_shard_fix_cols": (ctypes.c_int, [_p, _p, _p, _p, _i32, _i64, _i32, _i32, _p, _i32, _i32,
                                          _p, _p, _i64, _p, _p, _p, _p]),
    "csm_signal_ids": (ctypes.c_int, [_p, _p, _i64, _i64, _p, _i32, _i32, _i32, _i32, _i32, _p,
                                      _p, _p, _p, _p]),
    "csm_deciles_ids": (ctypes.c_int, [_p, _p, _p, _p, _i32, _i64, _i32, _p, _p, _p, _p, _p]),
    "csm_deciles_ids_ls": (ctypes.c_int, [_p, _p, _p, _p, _i32, _i64, _i32, _p, _p, _p, _p, _p,
                                          _p]),
    "csm_deciles_ids_legs": (ctypes.c_int, [_p, _p, _p, _i32, _i64, _i32, _p, _p, _p]),
    "csm_pipeline": (ctypes.c_int, [_p, _p, _i64, _i64, _p, _i32, _i32, _i32, _i32, _i32, _i32,
                                    _p, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "csm_comm_unique_id": (ctypes.c_int, [_p]),
    "csm_allgather_init": (ctypes.c_int, [_p, _p, _i32, _i32]),
    "csm_allgather": (ctypes.c_int, [_p, _p, _p, _i64]),
    "csm_allgather_free": (ctypes.c_int, [_p]),
}


def _declare(lib):
    for name, (res, args) in SIGNATURES.items():
        if not hasattr(lib, name):   # (CSMOM_AB_BASE: an older build in a same-box A/B)
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


EXPORTS = tuple(SIGNATURES)


def load_library():
    """Load (once) and return the ctypes handle; raises CsmUnavailable."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = lib_path()
    if not path.exists():
        raise CsmUnavailable(
            f"{path} not found: build the HIP engine first (__graft_entry__.build()); "
            "csmom has no CPU fallback")
    try:
        lib = ctypes.CDLL(str(path))
    except OSError as e:  # pragma: no cover - depends on the host
        raise CsmUnavailable(f"cannot load {path}: {e}") from e
    missing = [n for n in EXPORTS if not hasattr(lib, n)]
    if missing and not os.environ.get("CSMOM_AB_BASE"):
        raise CsmUnavailable(f"{path} lacks exports {missing}")
    _LIB = _declare(lib)
    return _LIB


def check(lib, ctx, status: int, what: str):
    if status != CSM_OK:
        msg = lib.csm_last_error(ctx)
        raise CsmError(status, f"{what}: {msg.decode() if msg else '?'}")
