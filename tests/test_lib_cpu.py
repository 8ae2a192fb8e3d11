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
    assert lib.csm_abi_version() == 3


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
    takes its documented values and restores its default; unknown keys / values are rejected,
    including the profiling ablations and the measured-and-dropped variants of earlier rounds
    (none of them is in the library any more)."""
    import csmom
    lib = csmom.load_library()
    cases = {b"signal_vec": ([1, 2], 2), b"signal_bwf": ([0, 1, 4], 0),
             b"dec_merge": ([0, 1], 1), b"dec_narrow_max": ([0, 16384], 16384),
             b"mj_reg": ([0, 1, 2], 2), b"cohort_lds": ([0, 1], 1), b"cohort_seg": ([0, 1], 1),
             b"turn_want": ([1, 65536], 4096), b"overlap_rows": ([0, 1], 1),
             b"turn_gen_grid": ([1, 2048], 8192), b"gen_reset": ([0, 1], 1), b"turn_vwg": ([0, 1], 1),
             b"dec_split": ([0, 1, 2], 2), b"dec_split_cells": ([8192, 65536], 32768),
             b"dec_split_pf": ([0, 1, 2], 0), b"tc_spins": ([0, 100], 1 << 21),
             b"turn_mask": ([0, 1], 1), b"ls_opt": ([0, 1], 1),
             b"signal_j12": ([0, 1], 1), b"cols_wg": ([0, 1], 1)}
    for key, (vals, default) in cases.items():
        for v in vals:
            assert lib.csm_tune(key, v) == 0, (key, v)
        assert lib.csm_tune(key, default) == 0
    for key, v in ((b"signal_vec", 3), (b"signal_bwf", 2), (b"dec_merge", 2), (b"overlap_rows", 2),
                   (b"turn_want", 0), (b"gen_reset", 2), (b"signal_j12", 2), (b"cols_wg", 2), (b"dec_split", 3), (b"dec_split_cells", 1000),
                   (b"dec_split_cells", 4096), (b"dec_split_pf", 3), (b"tc_spins", -1), (b"no_such_knob", 1)):
        assert lib.csm_tune(key, v) != 0, (key, v)
    # result-corrupting profiling knobs and negative-result variants are gone
    for key in (b"dec_ablate", b"signal_store", b"signal_rr", b"signal_db", b"signal_mw",
                b"dec_reg", b"dec_nreg", b"dec_wave_max", b"dec_ids", b"month_end_rows",
                b"signal_nbuf", b"signal_bw", b"signal_bl", b"turn_list", b"sort_wave",
                b"seg_stage2", b"turn_prep", b"dec_chunked"):
        assert lib.csm_tune(key, 0) != 0 and lib.csm_tune(key, 1) != 0, key
    assert lib.csm_tune(None, 1) != 0


def test_collective_entry_points_without_gpu():
    """The C-ABI all-gather validates its arguments before touching RCCL or the GPU."""
    import csmom
    lib = csmom.load_library()
    assert lib.csm_allgather_init(None, None, 0, 1) == -1
    assert lib.csm_allgather(None, None, None, 8) == -1
    assert lib.csm_allgather_free(None) == -1
    assert lib.csm_comm_unique_id(None) == -1


def test_signal_default_chunks():
    """csm_signal_chunked's default chunk count: the grid (chunks x ceil(N / 256)) within one
    workgroup per CU, chunks no shorter than one window, at least ceil(T_m / 32) chunks."""
    from csmom import Engine
    f = Engine.signal_default_chunks
    assert f(310, 5_000, 12, 1, 256) == 12          # C2: 20 column blocks -> 240 workgroups
    assert f(310, 1_000, 12, 1, 256) == 22          # narrow: one window per chunk binds
    assert f(310, 5_000, 12, 1, 304) == 15
    assert f(2_000, 60_000, 12, 1, 256) == 63       # wide: the 32-month limit binds
    assert f(0, 5_000) == 1 and f(10, 512, 12, 1) == 1
    for T_m in (1, 31, 32, 33, 700, 2_048):
        for N in (2, 256, 5_000, 100_000):
            C = f(T_m, N, 12, 1, 256)
            assert 1 <= C <= 64 and -(-T_m // C) <= 32
