"""The C ABI library builds for gfx950, loads here (no GPU) and exports what include/csmom.h
declares; argument validation and GPU-less failure paths return status codes."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def header_symbols():
    txt = (ROOT / "include" / "csmom.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(csm_\w+)\(", txt, re.M)))


def test_header_declares_expected_api():
    syms = header_symbols()
    for s in ("csm_create", "csm_month_end", "csm_momentum", "csm_signal", "csm_deciles",
              "csm_long_short",
              "csm_shard_summary", "csm_fold_carry", "csm_last_error"):
        assert s in syms


def test_library_exports_every_header_symbol():
    import csmom
    lib = csmom.load_library()
    raw = ctypes.CDLL(str(csmom.lib_path()))
    for s in header_symbols():
        assert hasattr(raw, s), s
    assert lib.csm_abi_version() == 2


def test_null_context_is_inval():
    import csmom
    lib = csmom.load_library()
    assert lib.csm_month_end(None, None, None, 0, 0, None, 0, None, None) == -1
    assert lib.csm_momentum(None, None, 0, 0, 12, 1, None, None, None, None, None, None) == -1
    assert lib.csm_signal(None, None, 0, 0, None, 0, 23, 12, 1, None, None, None, None, None,
                          None, None) == -1
    assert lib.csm_deciles(None, None, None, 0, 0, 10, None, None, None, None, None) == -1
    assert lib.csm_momentum_multi(None, None, 0, 0, None, 0, 1, None, None) == -1
    assert lib.csm_sync(None) == -1
    assert lib.csm_last_error(None) == b"null context"


def test_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import csmom
    lib = csmom.load_library()
    h = ctypes.c_void_p()
    assert lib.csm_create(0, ctypes.byref(h)) != 0
    assert not h.value


def test_engine_requires_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import csmom
    with pytest.raises(RuntimeError):
        csmom.Engine(0)


def test_tune_keys_documented_in_header_are_accepted():
    """csm_tune only sets process-wide knobs (no GPU call): every key include/csmom.h lists
    takes its documented values and restores its default; unknown keys / values are rejected."""
    import csmom
    lib = csmom.load_library()
    cases = {b"signal_vec": ([1, 2], 2), b"signal_nbuf": ([2, 3, 4], 4), b"dec_ablate": ([0, 1], 0),
             b"signal_bwf": ([0, 1, 2, 3, 4], 0),
             b"dec_ids": ([0, 1], 0), b"dec_reg": ([0, 1, 2], 0),
             b"dec_narrow_max": ([0, 16384], 16384), b"mj_reg": ([0, 1, 2], 2),
             b"signal_store": ([0, 1, 2, 3, 4], 0), b"signal_rr": ([0, 1], 0),
             b"signal_bl": ([0, 1], 1), b"cohort_lds": ([0, 1], 1), b"cohort_seg": ([0, 1], 1),
             b"turn_list": ([0, 1, 2], 1), b"sort_wave": ([0, 1], 1),
             b"turn_want": ([1, 65536], 4096), b"overlap_rows": ([0, 1], 1),
             b"seg_stage2": ([0, 1], 1), b"turn_gen_grid": ([1, 2048], 8192),
             b"turn_prep": ([0, 1], 1)}
    for key, (vals, default) in cases.items():
        for v in vals:
            assert lib.csm_tune(key, v) == 0, (key, v)
        assert lib.csm_tune(key, default) == 0
    assert lib.csm_tune(b"dec_reg", 3) != 0
    assert lib.csm_tune(b"signal_vec", 3) != 0
    assert lib.csm_tune(b"overlap_rows", 2) != 0
    assert lib.csm_tune(b"turn_want", 0) != 0
    assert lib.csm_tune(b"no_such_knob", 1) != 0
    assert lib.csm_tune(None, 1) != 0
