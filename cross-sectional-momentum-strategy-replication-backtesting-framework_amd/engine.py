"""Device engine: the momentum hot path on dense HBM-resident panels.

`Engine` owns one csm context per device and launches on torch's current HIP stream, so
torch events, graphs and allocations compose with it.  Tensors are torch ROCm tensors:
  P[T_d][N] f64 daily prices (ABSENT payload = no row, NaN = missing price),
  month_start[T_m+1] int64, everything else as in include/csmom.h.

Reference mapping (file:line):
  month_end   -> src/features.py:34-39      momentum   -> src/features.py:44-52, run_demo.py:48
  deciles     -> run_demo.py:18-29,46,49-55  long_short -> run_demo.py:57-67
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from ._lib import ABSENT_BITS, check, load_library

QTABLE_CACHE: dict[int, np.ndarray] = {}
FUSED_MIN_N = 32768  # below this the fused kernel has too few waves to fill 256 CUs
DEC_NARROW_MAX = 16384   # widest row of the narrow-row decile kernels (libcsmom's default)
LEGS_MAX_N = 7168        # widest row of the legs-only portfolio accounting (SEG_MAXN)


def quantile_table(n_bins: int) -> np.ndarray:
    """qcut's quantile grid as NumPy's percentile sees it ((linspace*100)/100)."""
    q = QTABLE_CACHE.get(n_bins)
    if q is None:
        q = np.ascontiguousarray((np.linspace(0.0, 1.0, n_bins + 1) * 100.0) / 100.0)
        QTABLE_CACHE[n_bins] = q
    return q


def absent_tensor(shape, device) -> torch.Tensor:
    return torch.full(shape, ABSENT_BITS, dtype=torch.int64, device=device).view(torch.float64)


def is_absent(x: torch.Tensor) -> torch.Tensor:
    b = x.contiguous().view(torch.int64)
    return (b & 0x7FF7FFFFFFFFFFFF) == ABSENT_BITS


def _ptr(t: torch.Tensor | None):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _need(t: torch.Tensor, name: str, dtype, shape, device):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if t.device != device:
        raise ValueError(f"{name} must live on {device}, got {t.device}")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} must have shape {tuple(shape)}, got {tuple(t.shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


@dataclass
class PipelineOut:
    PM: torch.Tensor
    M: torch.Tensor
    NR: torch.Tensor
    L: torch.Tensor
    EW: torch.Tensor
    CNT: torch.Tensor
    LS: torch.Tensor
    R: torch.Tensor | None = None
    VOL: torch.Tensor | None = None
    NV: torch.Tensor | None = None


@dataclass
class PortfolioOut:
    PR: torch.Tensor                 # [T_m][B][n_bins] overlapped decile returns
    LS: torch.Tensor                 # [T_m][B] long-short (NaN = dropped month)
    TURN: torch.Tensor | None = None  # [T_m][B] long-short turnover
    COST: torch.Tensor | None = None  # [T_m][B] transaction cost
    NET: torch.Tensor | None = None   # [T_m][B] LS - COST
    legs_only: bool = False           # PR holds deciles 0 and n_bins - 1 only (NaN elsewhere)


@dataclass
class ShardState:
    """signal_shard's end-state record [5][N] (present months, pending ranked row, its
    subset-ffilled price, first / last present month) with the daily panel it came from
    (shard_summary / shard_repair re-derive months PM does not keep from it)."""
    t: torch.Tensor
    P: torch.Tensor
    month_start: torch.Tensor


class Engine:
    """Signal (J, skip) -> per-date n_bins labels -> equal-weight long-short, on one GPU."""

    shard_ids = True   # the fused date-shard pass writes bucket ids and ranks from them

    def __init__(self, device: int | str | torch.device = 0):
        if not torch.cuda.is_available():
            raise RuntimeError("csmom.Engine needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.device = torch.device(device) if not isinstance(device, int) else torch.device("cuda", device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.lib = load_library()
        self.cus = int(torch.cuda.get_device_properties(self.device).multi_processor_count)
        h = ctypes.c_void_p()
        st = self.lib.csm_create(self.device.index, ctypes.byref(h))
        if st != 0:
            raise RuntimeError(f"csm_create(device={self.device.index}) failed with {st}")
        self.ctx = h

    def __del__(self):
        lib = getattr(self, "lib", None)
        if lib is not None and getattr(self, "ctx", None):
            lib.csm_destroy(self.ctx)
            self.ctx = None

    # ------------------------------------------------------------------ plumbing
    def _bind_stream(self):
        s = torch.cuda.current_stream(self.device).cuda_stream
        if s != getattr(self, "_bound_stream", None):   # one ctypes call per stream change
            self.lib.csm_set_stream(self.ctx, ctypes.c_void_p(s))
            self._bound_stream = s

    def _call(self, name, *args):
        self._bind_stream()
        check(self.lib, self.ctx, getattr(self.lib, name)(self.ctx, *args), name)

    def empty(self, shape, dtype=torch.float64):
        return torch.empty(shape, dtype=dtype, device=self.device)

    # ------------------------------------------------------------------ stages
    def month_end(self, P, month_start, V=None, PM=None, VOL=None):
        T_d, N = P.shape
        T_m = month_start.numel() - 1
        _need(P, "P", torch.float64, (T_d, N), self.device)
        _need(month_start, "month_start", torch.int64, (T_m + 1,), self.device)
        PM = self.empty((T_m, N)) if PM is None else PM
        _need(PM, "PM", torch.float64, (T_m, N), self.device)
        if V is not None:
            _need(V, "V", torch.float64, (T_d, N), self.device)
            VOL = self.empty((T_m, N)) if VOL is None else VOL
            _need(VOL, "VOL", torch.float64, (T_m, N), self.device)
        else:
            VOL = None
        self._call("csm_month_end", _ptr(P), _ptr(V), T_d, N, _ptr(month_start), T_m,
                   _ptr(PM), _ptr(VOL))
        return PM, VOL

    def momentum(self, PM, J=12, skip=1, with_ret=False, carry=None, next_pm=None,
                 carry_out=None, out=None, chunked="auto"):
        """csm_momentum.  chunked="auto": panels too narrow to fill the chip (few assets)
        take the time-chunked scan (csm_momentum_chunked, the same bits) when no carry is
        involved."""
        T_m, N = PM.shape
        if (chunked == "auto" and carry is None and next_pm is None and carry_out is None
                and self.default_chunks(T_m, N, J, skip) > 1):
            return self.momentum_chunked(PM, J, skip, with_ret=with_ret, out=out)
        _need(PM, "PM", torch.float64, (T_m, N), self.device)
        W = J + skip
        if carry is not None:
            _need(carry, "carry", torch.float64, (W + 2, N), self.device)
        if next_pm is not None:
            _need(next_pm, "next_pm", torch.float64, (N,), self.device)
        if carry_out is not None:
            _need(carry_out, "carry_out", torch.float64, (W + 2, N), self.device)
        if out is None:
            R = self.empty((T_m, N)) if with_ret else None
            M = self.empty((T_m, N))
            NR = self.empty((T_m, N))
        else:
            R, M, NR = out
        self._call("csm_momentum", _ptr(PM), T_m, N, int(J), int(skip), _ptr(R), _ptr(M),
                   _ptr(NR), _ptr(carry), _ptr(next_pm), _ptr(carry_out))
        return R, M, NR

    def momentum_multi(self, PM, Js, skip=1, with_ids=False, chunks=1, stacked=False):
        """csm_momentum_multi: one scan for several look-backs (up to 4 per launch).  Returns
        [(M, NR)] in the order of Js, each equal bit for bit to momentum(PM, J, skip).
        with_ids (csm_momentum_multi_ids): [(M, NR, IDS)], IDS the fixed-map bucket id of
        every mom_J (uint16 [T_m][N], read by deciles_ids on rows of any width).  chunks > 1
        (narrow panels; max(J) + skip <= 16, even N): the time-chunked multi-J scan
        (csm_momentum_multi_chunked), the same bits.  stacked: each launch group's M / NR / IDS
        are consecutive [T_m][N] blocks of one allocation (the joined sweep reads them as one
        [nJ][T_m][N] tensor, no copy); otherwise one allocation per output, freed one by one."""
        T_m, N = PM.shape
        _need(PM, "PM", torch.float64, (T_m, N), self.device)
        Js = [int(J) for J in Js]
        outs = []
        for q0 in range(0, len(Js), 4):
            grp = Js[q0:q0 + 4]
            if stacked:
                Ms = list(self.empty((len(grp), T_m, N)))
                NRs = list(self.empty((len(grp), T_m, N)))
            else:
                Ms = [self.empty((T_m, N)) for _ in grp]
                NRs = [self.empty((T_m, N)) for _ in grp]
            new_ids = ((lambda: list(self.empty((len(grp), T_m, N), torch.int16))) if stacked
                       else (lambda: [self.empty((T_m, N), torch.int16) for _ in grp]))
            jarr = (ctypes.c_int32 * len(grp))(*grp)
            marr = (ctypes.c_void_p * len(grp))(*[t.data_ptr() for t in Ms])
            narr = (ctypes.c_void_p * len(grp))(*[t.data_ptr() for t in NRs])
            if chunks > 1:
                IDs = new_ids() if with_ids else None
                iarr = ((ctypes.c_void_p * len(grp))(*[t.data_ptr() for t in IDs])
                        if with_ids else None)
                nbytes = int(self.lib.csm_momentum_multi_chunked_workspace(
                    T_m, N, max(grp), int(skip), int(chunks)))
                ws = torch.empty(max(nbytes, 8), dtype=torch.uint8, device=self.device)
                self._call("csm_momentum_multi_chunked", _ptr(PM), T_m, N, jarr, len(grp),
                           int(skip), int(chunks), marr, narr, iarr, _ptr(ws))
                outs.extend(zip(Ms, NRs, IDs) if with_ids else zip(Ms, NRs))
            elif with_ids:
                IDs = new_ids()
                iarr = (ctypes.c_void_p * len(grp))(*[t.data_ptr() for t in IDs])
                self._call("csm_momentum_multi_ids", _ptr(PM), T_m, N, jarr, len(grp), int(skip),
                           marr, narr, iarr)
                outs.extend(zip(Ms, NRs, IDs))
            else:
                self._call("csm_momentum_multi", _ptr(PM), T_m, N, jarr, len(grp), int(skip),
                           marr, narr)
                outs.extend(zip(Ms, NRs))
        return outs

    @staticmethod
    def default_chunks(T_m, N, J=12, skip=1):
        """Chunks for the time-chunked scan: enough (chunk, asset) lanes to fill the chip
        (~2^17), chunks no shorter than one window (C2, 300 months: 20 chunks, scan 0.078 ->
        0.068 ms against 10 chunks of two windows; the fold chains through any number of
        earlier chunks, so the outputs are the same bits)."""
        if T_m <= 0:
            return 1
        want = max(1, -(-131072 // max(N, 1)))
        return int(max(1, min(want, T_m // max(J + skip + 1, 1), 256)))

    def momentum_chunked(self, PM, J=12, skip=1, chunks=None, with_ret=False, next_pm=None,
                         out=None, workspace=None, ids=None):
        """csm_momentum_chunked: the scan split into `chunks` concurrent month ranges.  ids
        (int16 [T_m][N], N % 4 == 0): also each mom_J's fixed-map bucket id
        (csm_momentum_chunked_ids, for deciles_ids)."""
        T_m, N = PM.shape
        _need(PM, "PM", torch.float64, (T_m, N), self.device)
        C = self.default_chunks(T_m, N, J, skip) if chunks is None else int(chunks)
        if next_pm is not None:
            _need(next_pm, "next_pm", torch.float64, (N,), self.device)
        if out is None:
            R = self.empty((T_m, N)) if with_ret else None
            M, NR = self.empty((T_m, N)), self.empty((T_m, N))
        else:
            R, M, NR = out
        nbytes = int(self.lib.csm_momentum_chunked_workspace(T_m, N, int(J), int(skip), C))
        if workspace is None or workspace.numel() * workspace.element_size() < nbytes:
            workspace = torch.empty(max(nbytes, 8), dtype=torch.uint8, device=self.device)
        if ids is not None:
            _need(ids, "ids", torch.int16, (T_m, N), self.device)
            self._call("csm_momentum_chunked_ids", _ptr(PM), T_m, N, int(J), int(skip), C, _ptr(R),
                       _ptr(M), _ptr(NR), _ptr(next_pm), _ptr(ids), _ptr(workspace))
        else:
            self._call("csm_momentum_chunked", _ptr(PM), T_m, N, int(J), int(skip), C, _ptr(R),
                       _ptr(M), _ptr(NR), _ptr(next_pm), _ptr(workspace))
        return R, M, NR

    @staticmethod
    def signal_default_chunks(T_m, N, J=12, skip=1, cus=256):
        """Chunks for csm_signal_chunked: as many as keep the grid (chunks x ceil(N / 256)
        workgroups) within one workgroup per CU, chunks no shorter than one window, and never
        fewer than the 32-months-per-chunk limit needs.  A second workgroup on a CU waits for
        the first to leave (each holds ~80 KB of LDS and its month-end stream saturates the
        CU), so the grid beyond the CU count serialises: C2 (20 column blocks) at 12 / 13 / 21
        chunks 0.130 / 0.152 / 0.140 ms per step (profiles/r05/experiments/tc_chunks/)."""
        if T_m <= 0:
            return 1
        nbx = max(1, -(-N // 256))
        c = min(max(1, cus // nbx), max(1, T_m // max(J + skip + 1, 1)), 64)
        return int(min(max(c, -(-T_m // 32)), 64))

    def signal_chunked(self, P, month_start, max_month_days, J=12, skip=1, chunks=None,
                       with_ret=False, with_ids=True, out=None, workspace=None, check=True):
        """csm_signal_chunked: month-end + time-chunked scan in one launch (narrow panels, C2):
        the same R / M / NR / ids bits as month_end -> momentum_chunked(_ids).  Even N, months
        of <= 23 day rows.  workspace: a zero-filled uint8 buffer of
        csm_signal_chunked_workspace bytes (kept by the caller across calls: each launch leaves
        its sync words zero).  check (default): unless the stream is capturing, read the
        launch's give-up mark (csm_signal_chunked_status; synchronises) and raise CsmError
        (CSM_E_TIMEOUT) if a workgroup gave up a wait.  check=False (timed loops, graph capture):
        the caller calls signal_chunked_status(workspace) itself afterwards.
        Returns (R, M, NR, IDS, workspace)."""
        T_d, N = P.shape
        T_m = month_start.numel() - 1
        _need(P, "P", torch.float64, (T_d, N), self.device)
        _need(month_start, "month_start", torch.int64, (T_m + 1,), self.device)
        C = (self.signal_default_chunks(T_m, N, J, skip, self.cus) if chunks is None
             else int(chunks))
        C = max(1, min(C, 64, max(T_m, 1)))
        if out is None:
            R = self.empty((T_m, N)) if with_ret else None
            M, NR = self.empty((T_m, N)), self.empty((T_m, N))
            IDS = self.empty((T_m, N), torch.int16) if with_ids else None
        else:
            R, M, NR, IDS = out
        if IDS is not None:
            _need(IDS, "IDS", torch.int16, (T_m, N), self.device)
        nbytes = int(self.lib.csm_signal_chunked_workspace(T_m, N, int(J), int(skip), C))
        if workspace is None or workspace.numel() * workspace.element_size() < nbytes:
            workspace = torch.zeros(max(nbytes, 256), dtype=torch.uint8, device=self.device)
        if R is not None:
            _need(R, "R", torch.float64, (T_m, N), self.device)
        _need(M, "M", torch.float64, (T_m, N), self.device)
        _need(NR, "NR", torch.float64, (T_m, N), self.device)
        self._call("csm_signal_chunked", _ptr(P), T_d, N, _ptr(month_start), T_m,
                   int(max_month_days), int(J), int(skip), C, _ptr(R), _ptr(M), _ptr(NR),
                   _ptr(IDS), _ptr(workspace))
        if check and not torch.cuda.is_current_stream_capturing():
            self.signal_chunked_status(workspace)
        return R, M, NR, IDS, workspace

    def signal_chunked_status(self, workspace):
        """csm_signal_chunked_status: synchronise, raise CsmError (CSM_E_TIMEOUT) if a
        csm_signal_chunked launch on this workspace gave up a wait since the last check (its
        outputs are invalid; the mark is cleared)."""
        self._call("csm_signal_chunked_status", _ptr(workspace))

    @staticmethod
    def signal_chunked_timed_out(workspace):
        """Whether the workspace holds an unreported give-up mark (sync word 2; never set by a
        correct launch).  Synchronises; does not clear it."""
        return bool(workspace[8:12].view(torch.int32).item() != 0)

    def signal(self, P, month_start, max_month_days, J=12, skip=1, with_pm=False,
               with_ret=False, carry=None, next_pm=None, carry_out=None, out=None):
        """Fused month-end + scan (csm_signal): one pass over the daily panel, no PM round
        trip.  Needs even N and months of <= 32 days."""
        T_d, N = P.shape
        T_m = month_start.numel() - 1
        _need(P, "P", torch.float64, (T_d, N), self.device)
        _need(month_start, "month_start", torch.int64, (T_m + 1,), self.device)
        W = J + skip
        for t, nm, shp in ((carry, "carry", (W + 2, N)), (next_pm, "next_pm", (N,)),
                           (carry_out, "carry_out", (W + 2, N))):
            if t is not None:
                _need(t, nm, torch.float64, shp, self.device)
        if out is None:
            PM = self.empty((T_m, N)) if with_pm else None
            R = self.empty((T_m, N)) if with_ret else None
            M, NR = self.empty((T_m, N)), self.empty((T_m, N))
        else:
            PM, R, M, NR = out
        self._call("csm_signal", _ptr(P), T_d, N, _ptr(month_start), T_m, int(max_month_days),
                   int(J), int(skip), _ptr(PM), _ptr(R), _ptr(M), _ptr(NR), _ptr(carry),
                   _ptr(next_pm), _ptr(carry_out))
        return PM, R, M, NR

    def signal_ids(self, P, month_start, max_month_days, J=12, skip=1, with_pm=False,
                   with_ret=False, out=None, min_month_days=0):
        """csm_signal_ids: csm_signal (no carry) that also writes the fixed-map bucket id of
        every mom_J (uint16 [T_m][N], read by deciles_ids).  N % 4 == 0.
        Returns (PM, R, M, NR, IDS)."""
        T_d, N = P.shape
        T_m = month_start.numel() - 1
        _need(P, "P", torch.float64, (T_d, N), self.device)
        _need(month_start, "month_start", torch.int64, (T_m + 1,), self.device)
        if out is None:
            PM = self.empty((T_m, N)) if with_pm else None
            R = self.empty((T_m, N)) if with_ret else None
            M, NR = self.empty((T_m, N)), self.empty((T_m, N))
            IDS = self.empty((T_m, N), torch.int16)
        else:
            PM, R, M, NR, IDS = out
        _need(IDS, "IDS", torch.int16, (T_m, N), self.device)
        self._call("csm_signal_ids", _ptr(P), T_d, N, _ptr(month_start), T_m, int(max_month_days),
                   int(min_month_days), int(J), int(skip), _ptr(PM), _ptr(R), _ptr(M), _ptr(NR),
                   _ptr(IDS))
        return PM, R, M, NR, IDS

    def deciles_ids(self, M, NR, IDS, n_bins=10, out=None, with_nv=False, LS=None, legs=False):
        """csm_deciles_ids: deciles() from the ids of signal_ids / momentum_multi(with_ids=True)
        (same labels / counts).  Rows of <= 16384 assets take the narrow kernel (2048 buckets:
        the fixed map's ids >> 2), wider rows the 8192-bucket merged pass; needs N % 4 == 0.
        LS (float64 [T_m], needs NR): also the long-short of every date, in the same launch
        (csm_deciles_ids_ls; equal to long_short(EW, CNT) bit for bit).
        legs=True (NR None; for legs-only accounting): csm_deciles_ids_legs -- labels 0,
        n_bins - 1 and NaN exact, every other ranked cell SOME label in [1, n_bins - 2]."""
        T_m, N = M.shape
        _need(M, "M", torch.float64, (T_m, N), self.device)
        _need(IDS, "IDS", torch.int16, (T_m, N), self.device)
        if NR is not None:
            _need(NR, "NR", torch.float64, (T_m, N), self.device)
        if out is None:
            L = self.empty((T_m, N), torch.int8)
            EW = self.empty((T_m, n_bins)) if NR is not None else None
            CNT = self.empty((T_m, n_bins), torch.int32) if NR is not None else None
            NV = self.empty((T_m,), torch.int32) if with_nv else None
        else:
            L, EW, CNT, NV = out
        q = quantile_table(n_bins)
        if LS is not None:
            if NR is None:
                raise ValueError("deciles_ids(LS=...) needs NR")
            _need(LS, "LS", torch.float64, (T_m,), self.device)
            self._call("csm_deciles_ids_ls", _ptr(M), _ptr(NR), _ptr(IDS), T_m, N, int(n_bins),
                       q.ctypes.data_as(ctypes.c_void_p), _ptr(L), _ptr(EW), _ptr(CNT), _ptr(NV),
                       _ptr(LS))
            return L, EW, CNT, NV
        if legs:
            if NR is not None:
                raise ValueError("deciles_ids(legs=True) takes no NR (labels only)")
            self._call("csm_deciles_ids_legs", _ptr(M), _ptr(IDS), T_m, N, int(n_bins),
                       q.ctypes.data_as(ctypes.c_void_p), _ptr(L), _ptr(NV))
            return L, EW, CNT, NV
        self._call("csm_deciles_ids", _ptr(M), _ptr(NR), _ptr(IDS), T_m, N, int(n_bins),
                   q.ctypes.data_as(ctypes.c_void_p), _ptr(L), _ptr(EW), _ptr(CNT), _ptr(NV))
        return L, EW, CNT, NV

    @staticmethod
    def month_days(month_start):
        """(longest month, shortest interior month) in days, one device sync; the first and
        the last month may be partial (csm_signal_ids' min_month_days excepts them)."""
        if month_start.numel() < 2:
            return 1, 0
        d = month_start[1:] - month_start[:-1]
        inner = d[1:-1] if d.numel() > 2 else d[:0]
        mn = inner.min() if inner.numel() else torch.full_like(d[0], 1 << 30)
        mx, mn = torch.stack([d.max(), mn]).tolist()
        return int(mx), int(mn)

    def pipeline(self, P, month_start, J=12, skip=1, n_bins=10, max_month_days=None,
                 with_pm=True, with_ret=False, out=None, min_month_days=None) -> PipelineOut:
        """csm_pipeline: the whole K = 1 pass in one C call (fused signal with bucket ids,
        labels + decile means, long-short)."""
        T_d, N = P.shape
        T_m = month_start.numel() - 1
        _need(P, "P", torch.float64, (T_d, N), self.device)
        _need(month_start, "month_start", torch.int64, (T_m + 1,), self.device)
        if max_month_days is None or min_month_days is None:
            mx, mn = self.month_days(month_start)
            max_month_days = mx if max_month_days is None else max_month_days
            min_month_days = mn if min_month_days is None else min_month_days
        if out is None:
            PM = self.empty((T_m, N)) if with_pm else None
            R = self.empty((T_m, N)) if with_ret else None
            M, NR = self.empty((T_m, N)), self.empty((T_m, N))
            L = self.empty((T_m, N), torch.int8)
            EW, CNT = self.empty((T_m, n_bins)), self.empty((T_m, n_bins), torch.int32)
            NV, LS = self.empty((T_m,), torch.int32), self.empty((T_m,))
        else:
            PM, R, M, NR, L, EW, CNT, NV, LS = out
        q = quantile_table(n_bins)
        self._call("csm_pipeline", _ptr(P), T_d, N, _ptr(month_start), T_m, int(max_month_days),
                   int(min_month_days), int(J), int(skip), int(n_bins),
                   q.ctypes.data_as(ctypes.c_void_p), _ptr(PM),
                   _ptr(R), _ptr(M), _ptr(NR), _ptr(L), _ptr(EW), _ptr(CNT), _ptr(NV), _ptr(LS))
        return PipelineOut(PM=PM, M=M, NR=NR, L=L, EW=EW, CNT=CNT, LS=LS, R=R, NV=NV)

    def deciles(self, M, NR=None, n_bins=10, out=None, with_nv=False):
        T_m, N = M.shape
        _need(M, "M", torch.float64, (T_m, N), self.device)
        if NR is not None:
            _need(NR, "NR", torch.float64, (T_m, N), self.device)
        if out is None:
            L = self.empty((T_m, N), torch.int8)
            EW = self.empty((T_m, n_bins)) if NR is not None else None
            CNT = self.empty((T_m, n_bins), torch.int32) if NR is not None else None
            NV = self.empty((T_m,), torch.int32) if with_nv else None
        else:
            L, EW, CNT, NV = out
        q = quantile_table(n_bins)
        self._call("csm_deciles", _ptr(M), _ptr(NR), T_m, N, int(n_bins),
                   q.ctypes.data_as(ctypes.c_void_p), _ptr(L), _ptr(EW), _ptr(CNT), _ptr(NV))
        return L, EW, CNT, NV

    def long_short(self, EW, CNT, LS=None):
        T_m, nb = EW.shape
        _need(EW, "EW", torch.float64, (T_m, nb), self.device)
        _need(CNT, "CNT", torch.int32, (T_m, nb), self.device)
        LS = self.empty((T_m,)) if LS is None else LS
        self._call("csm_long_short", _ptr(EW), _ptr(CNT), T_m, nb, _ptr(LS))
        return LS

    def portfolio(self, L, NR, n_bins=10, K=1, W=None, B=1, half_spread=0.0005, k_impact=0.1,
                  aum=0.0, ADV=None, SIG=None, with_costs=True, out=None, workspace=None):
        """csm_portfolio: K-overlapping cohorts, equal (W None) or value weights, long-short
        turnover and costs (rules E1..E5).  L/NR/W/ADV/SIG are [T_m][B*N] (B panels side by
        side, the sweep layout) or [T_m][N] with B = 1.  Returns a PortfolioOut."""
        T_m, BN = L.shape
        if B < 1 or BN % B:
            raise ValueError(f"row width {BN} is not B={B} panels")
        N = BN // B
        _need(L, "L", torch.int8, (T_m, BN), self.device)
        _need(NR, "NR", torch.float64, (T_m, BN), self.device)
        for t, nm in ((W, "W"), (ADV, "ADV"), (SIG, "SIG")):
            if t is not None:
                _need(t, nm, torch.float64, (T_m, BN), self.device)
        if out is None:
            PR = self.empty((T_m, B, n_bins))
            LS = self.empty((T_m, B))
            TURN = self.empty((T_m, B)) if with_costs else None
            COST = self.empty((T_m, B)) if with_costs else None
            NET = self.empty((T_m, B)) if with_costs else None
        else:
            PR, LS, TURN, COST, NET = out
        nbytes = int(self.lib.csm_portfolio_workspace(T_m, B, N, int(n_bins), int(K)))
        if workspace is None or workspace.numel() * workspace.element_size() < nbytes:
            workspace = torch.empty(max(nbytes, 8), dtype=torch.uint8, device=self.device)
        self._call("csm_portfolio", _ptr(L), _ptr(NR), _ptr(W), T_m, int(B), N, int(n_bins),
                   int(K), float(half_spread), float(k_impact), float(aum), _ptr(ADV), _ptr(SIG),
                   _ptr(PR), _ptr(LS), _ptr(TURN), _ptr(COST), _ptr(NET), _ptr(workspace))
        return PortfolioOut(PR=PR, LS=LS, TURN=TURN, COST=COST, NET=NET)

    def portfolio_multi(self, L, NR, n_bins=10, Ks=(1,), W=None, B=1, half_spread=0.0005,
                        k_impact=0.1, aum=0.0, ADV=None, SIG=None, with_costs=True,
                        workspace=None, return_stacked=False, legs_only=False, need_full=None):
        """One cohort-sum pass (csm_cohort_sums, Kmax = max(Ks)) shared by the accounting of
        every holding period K in Ks (csm_portfolio_from_cohorts).  Returns {K: PortfolioOut}.
        legs_only (rows of <= 7168 assets): sort and sum only deciles 0 and n_bins - 1
        (csm_cohort_sums_legs / csm_portfolio_from_cohorts_legs): LS / TURN / COST / NET bit for
        bit the full path's, PR NaN outside the legs.  When a panel lacks one leg's column (the
        long-short rule then needs every decile) the full path is rerun (one device sync); with
        need_full (device int32 [1], caller-zeroed) the flag is left there instead, no sync, and
        the caller reruns with legs_only=False when it is set."""
        T_m, BN = L.shape
        if B < 1 or BN % B:
            raise ValueError(f"row width {BN} is not B={B} panels")
        N = BN // B
        _need(L, "L", torch.int8, (T_m, BN), self.device)
        _need(NR, "NR", torch.float64, (T_m, BN), self.device)
        for t, nm in ((W, "W"), (ADV, "ADV"), (SIG, "SIG")):
            if t is not None:
                _need(t, nm, torch.float64, (T_m, BN), self.device)
        Ks = [int(k) for k in Ks]
        Kmax = max(Ks)
        legs_only = bool(legs_only) and N <= LEGS_MAX_N   # wider rows: every decile
        nbytes = int(self.lib.csm_portfolio_workspace(T_m, B, N, int(n_bins), Kmax))
        if workspace is None or workspace.numel() * workspace.element_size() < nbytes:
            workspace = torch.empty(max(nbytes, 8), dtype=torch.uint8, device=self.device)
        self._call("csm_cohort_sums_legs" if legs_only else "csm_cohort_sums", _ptr(L), _ptr(NR),
                   _ptr(W), T_m, int(B), N, int(n_bins), Kmax, _ptr(workspace))
        flag = need_full
        if legs_only and need_full is None:
            flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        res, stacked = self._from_cohorts(L, W, T_m, B, N, n_bins, Ks, half_spread, k_impact,
                                          aum, ADV, SIG, with_costs, workspace, legs_only, flag)
        if legs_only and need_full is None and int(flag.item()):   # a panel lacks a leg's column
            return self.portfolio_multi(L, NR, n_bins, Ks, W, B, half_spread, k_impact, aum,
                                        ADV, SIG, with_costs, workspace, return_stacked)
        if return_stacked:
            return res, stacked
        return res

    def portfolio_multi_js(self, Ls, NR, n_bins=10, Ks=(1,), B=1, half_spread=0.0005,
                           k_impact=0.1, aum=0.0, with_costs=True, legs_only=False, need_full=None):
        """portfolio_multi (equal weights) for several label panels Ls that share ONE next_ret
        panel NR (the bootstrap sweep's, boot_scan): one cohort pass for every J
        (csm_cohort_sums_js: each month's return row read once), then each J's accounting.
        Returns [(res, stacked)] per J, each equal bit for bit to portfolio_multi(L, NR, ...,
        return_stacked=True)."""
        T_m, BN = NR.shape
        if B < 1 or BN % B:
            raise ValueError(f"row width {BN} is not B={B} panels")
        N = BN // B
        _need(NR, "NR", torch.float64, (T_m, BN), self.device)
        for L in Ls:
            _need(L, "L", torch.int8, (T_m, BN), self.device)
        Ks = [int(k) for k in Ks]
        Kmax = max(Ks)
        legs_only = bool(legs_only) and N <= LEGS_MAX_N
        nbytes = int(self.lib.csm_portfolio_workspace(T_m, B, N, int(n_bins), Kmax))
        wss = [torch.empty(max(nbytes, 8), dtype=torch.uint8, device=self.device) for _ in Ls]
        nJ = len(Ls)
        self._call("csm_cohort_sums_js", nJ, (ctypes.c_void_p * nJ)(*[L.data_ptr() for L in Ls]),
                   _ptr(NR), T_m, int(B), N, int(n_bins), Kmax, 1 if legs_only else 0,
                   (ctypes.c_void_p * nJ)(*[w.data_ptr() for w in wss]))
        flag = need_full
        if legs_only and need_full is None:
            flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        outs = [self._from_cohorts(L, None, T_m, B, N, n_bins, Ks, half_spread, k_impact, aum,
                                   None, None, with_costs, ws, legs_only, flag)
                for L, ws in zip(Ls, wss)]
        if legs_only and need_full is None and int(flag.item()):   # a panel lacks a leg's column
            return self.portfolio_multi_js(Ls, NR, n_bins, Ks, B, half_spread, k_impact, aum,
                                           with_costs, legs_only=False)
        return outs

    def portfolio_plan(self, T_m, B, N, n_bins=10, K=1):
        """csm_portfolio_plan: (cohort chunks, turnover chunks) of a portfolio call; calls with
        the same plan give each panel the same bits."""
        v = int(self.lib.csm_portfolio_plan(int(T_m), int(B), int(N), int(n_bins), int(K)))
        if v < 0:
            raise ValueError("csm_portfolio_plan: bad arguments")
        return v & 0xFFFFFFFF, v >> 32

    def portfolio_multi_js_grouped(self, Lg, NR, n_bins=10, Ks=(1,), B=1, half_spread=0.0005,
                                   k_impact=0.1, aum=0.0, with_costs=True, legs_only=False,
                                   need_full=None, return_stacked=False):
        """portfolio_multi_js with the look-backs' label panels stored group-major, Lg int8
        [nJ][T_m][B * N] (as one stacked decile pass writes them): one cohort pass over the shared
        next_ret NR [T_m][B * N] into one workspace of nJ * B panels (csm_cohort_sums_js_grouped),
        then ONE accounting launch set for every J (csm_portfolio_from_cohorts_grouped: panel
        q * B + b = J q's panel b).  Where portfolio_plan(T_m, B) == portfolio_plan(T_m, nJ * B),
        each J's outputs equal portfolio_multi_js's bit for bit."""
        if Lg.dim() != 3:
            raise ValueError("Lg must be [nJ][T_m][B * N]")
        nJ, T_m, BN = Lg.shape
        if B < 1 or BN % B:
            raise ValueError(f"row width {BN} is not B={B} panels")
        N = BN // B
        _need(Lg, "Lg", torch.int8, (nJ, T_m, BN), self.device)
        _need(NR, "NR", torch.float64, (T_m, BN), self.device)
        Ks = [int(k) for k in Ks]
        Kmax = max(Ks)
        legs_only = bool(legs_only) and N <= LEGS_MAX_N
        nbytes = int(self.lib.csm_portfolio_workspace(T_m, nJ * B, N, int(n_bins), Kmax))
        ws = torch.empty(max(nbytes, 8), dtype=torch.uint8, device=self.device)
        self._call("csm_cohort_sums_js_grouped", nJ, _ptr(Lg), _ptr(NR), T_m, int(B), N,
                   int(n_bins), Kmax, 1 if legs_only else 0, _ptr(ws))
        flag = need_full
        if legs_only and need_full is None:
            flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        res, stacked = self._from_cohorts(Lg, None, T_m, nJ * B, N, n_bins, Ks, half_spread,
                                          k_impact, aum, None, None, with_costs, ws, legs_only,
                                          flag, groups=(nJ, B))
        if legs_only and need_full is None and int(flag.item()):   # a panel lacks a leg's column
            return self.portfolio_multi_js_grouped(Lg, NR, n_bins, Ks, B, half_spread, k_impact,
                                                   aum, with_costs, False, None, return_stacked)
        return (res, stacked) if return_stacked else res

    def portfolio_multi_grouped(self, Lg, NRg, n_bins=10, Ks=(1,), W=None, Bg=1,
                                half_spread=0.0005, k_impact=0.1, aum=0.0, ADV=None, SIG=None,
                                with_costs=True, workspace=None, return_stacked=False,
                                legs_only=False, need_full=None):
        """portfolio_multi of B = G * Bg panels stored group-major (csm_cohort_sums_grouped ->
        csm_portfolio_from_cohorts_grouped): Lg int8 / NRg f64 [G][T_m][Bg * N] (G blocks, e.g.
        the look-backs' label panels as one stacked decile pass writes them) and W / ADV / SIG
        [T_m][Bg * N] shared by the groups.  Outputs (panel g * Bg + p = group g's panel p) equal
        portfolio_multi(cat(Lg, 1), cat(NRg, 1), ..., W.repeat(1, G), B=G * Bg) bit for bit,
        without building those side-by-side copies."""
        if Lg.dim() != 3:
            raise ValueError("Lg must be [G][T_m][Bg * N]")
        G, T_m, BgN = Lg.shape
        if Bg < 1 or BgN % Bg:
            raise ValueError(f"row width {BgN} is not Bg={Bg} panels")
        N = BgN // Bg
        B = G * Bg
        _need(Lg, "Lg", torch.int8, (G, T_m, BgN), self.device)
        _need(NRg, "NRg", torch.float64, (G, T_m, BgN), self.device)
        for t, nm in ((W, "W"), (ADV, "ADV"), (SIG, "SIG")):
            if t is not None:
                _need(t, nm, torch.float64, (T_m, BgN), self.device)
        Ks = [int(k) for k in Ks]
        Kmax = max(Ks)
        legs_only = bool(legs_only) and N <= LEGS_MAX_N
        nbytes = int(self.lib.csm_portfolio_workspace(T_m, B, N, int(n_bins), Kmax))
        if workspace is None or workspace.numel() * workspace.element_size() < nbytes:
            workspace = torch.empty(max(nbytes, 8), dtype=torch.uint8, device=self.device)
        self._call("csm_cohort_sums_grouped", G, _ptr(Lg), _ptr(NRg), _ptr(W), T_m, int(Bg), N,
                   int(n_bins), Kmax, 1 if legs_only else 0, _ptr(workspace))
        flag = need_full
        if legs_only and need_full is None:
            flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        res, stacked = self._from_cohorts(Lg, W, T_m, B, N, n_bins, Ks, half_spread, k_impact,
                                          aum, ADV, SIG, with_costs, workspace, legs_only, flag,
                                          groups=(G, Bg))
        if legs_only and need_full is None and int(flag.item()):   # a panel lacks a leg's column
            return self.portfolio_multi_grouped(Lg, NRg, n_bins, Ks, W, Bg, half_spread, k_impact,
                                                aum, ADV, SIG, with_costs, workspace,
                                                return_stacked)
        if return_stacked:
            return res, stacked
        return res

    def _from_cohorts(self, L, W, T_m, B, N, n_bins, Ks, half_spread, k_impact, aum, ADV, SIG,
                      with_costs, workspace, legs_only, need_full, groups=None):
        """The accounting half of portfolio_multi on a workspace holding the cohort sums ->
        (res {K: PortfolioOut}, stacked PortfolioOut).  groups=(G, Bg): the group-major layout
        of portfolio_multi_grouped."""
        nK = len(Ks)
        Kmax = max(Ks)
        PR, LS = self.empty((nK, T_m, B, n_bins)), self.empty((nK, T_m, B))
        TURN = self.empty((nK, T_m, B)) if with_costs else None
        COST = self.empty((nK, T_m, B)) if with_costs else None
        NET = self.empty((nK, T_m, B)) if with_costs else None
        ks = (ctypes.c_int32 * nK)(*Ks)
        args = (_ptr(L), _ptr(W), T_m, int(B), N, int(n_bins), Kmax, nK,
                ctypes.cast(ks, ctypes.c_void_p), float(half_spread), float(k_impact), float(aum),
                _ptr(ADV), _ptr(SIG), _ptr(PR), _ptr(LS), _ptr(TURN), _ptr(COST), _ptr(NET),
                _ptr(workspace))
        if groups is not None:
            G, Bg = groups
            gargs = (_ptr(L), _ptr(W), T_m, int(Bg)) + args[4:]
            self._call("csm_portfolio_from_cohorts_grouped", int(G), *gargs,
                       1 if legs_only else 0, _ptr(need_full) if legs_only else None)
        elif legs_only:
            self._call("csm_portfolio_from_cohorts_legs", *args, _ptr(need_full))
        else:
            self._call("csm_portfolio_from_cohorts_multi", *args)
        pick = lambda x, q: None if x is None else x[q]
        res = {K: PortfolioOut(PR=PR[q], LS=LS[q], TURN=pick(TURN, q), COST=pick(COST, q),
                               NET=pick(NET, q), legs_only=legs_only) for q, K in enumerate(Ks)}
        return res, PortfolioOut(PR=PR, LS=LS, TURN=TURN, COST=COST, NET=NET, legs_only=legs_only)

    def summary(self, LS, TURN=None, COST=None, NET=None, freq=12.0):
        """csm_summary: [nS][B][7] (months, mean, Sharpe, turnover, cost, net mean, net
        Sharpe) from stacked [nS][T_m][B] series (or one [T_m][B] series: nS = 1)."""
        if LS.dim() == 2:
            LS = LS.unsqueeze(0)
            TURN, COST, NET = (None if x is None else x.unsqueeze(0) for x in (TURN, COST, NET))
        nS, T_m, B = LS.shape
        for t, nm in ((LS, "LS"), (TURN, "TURN"), (COST, "COST"), (NET, "NET")):
            if t is not None:
                _need(t, nm, torch.float64, (nS, T_m, B), self.device)
        out = self.empty((nS, B, 7))
        self._call("csm_summary", _ptr(LS), _ptr(TURN), _ptr(COST), _ptr(NET), nS, T_m, B,
                   float(freq), _ptr(out))
        return out

    def turnover_features(self, PM, VOL, so, mcap, lookback=3):
        """csm_turnover_features (src/features.py:60-107, rule T1): (ADV, SH, TURN, TAVG)."""
        T_m, N = PM.shape
        _need(PM, "PM", torch.float64, (T_m, N), self.device)
        _need(VOL, "VOL", torch.float64, (T_m, N), self.device)
        _need(so, "so", torch.float64, (N,), self.device)
        _need(mcap, "mcap", torch.float64, (N,), self.device)
        outs = [self.empty((T_m, N)) for _ in range(4)]
        self._call("csm_turnover_features", _ptr(PM), _ptr(VOL), _ptr(so), _ptr(mcap), T_m, N,
                   int(lookback), *[_ptr(o) for o in outs])
        return tuple(outs)

    def mask_by(self, M, X):
        """X where M is valid, NaN elsewhere (csm_double_sort_labels)."""
        T_m, N = M.shape
        _need(X, "X", torch.float64, (T_m, N), self.device)
        Xm = self.empty((T_m, N))
        self._call("csm_double_sort_labels", _ptr(M), _ptr(X), None, None, T_m, N, 1, _ptr(Xm),
                   None)
        return Xm

    def combine_labels(self, Lm, Lv, n_vol):
        """n_vol * Lm + Lv where both are valid, else -1 (csm_double_sort_labels)."""
        T_m, N = Lm.shape
        _need(Lv, "Lv", torch.int8, (T_m, N), self.device)
        Lc = self.empty((T_m, N), torch.int8)
        dummy = self.empty((1,))
        self._call("csm_double_sort_labels", _ptr(dummy), None, _ptr(Lm), _ptr(Lv), T_m, N,
                   int(n_vol), None, _ptr(Lc))
        return Lc

    def bootstrap(self, R, B, b0=0, seed=5000, mean_block=6.0, p0=100.0, out=None):
        """csm_bootstrap: B stationary-bootstrap month panels of the base month-return panel
        R[T_m][N] (rule E6) -> (src [B][T_m] int32, PMb [T_m][B*N] month prices)."""
        T_m, N = R.shape
        _need(R, "R", torch.float64, (T_m, N), self.device)
        if out is None:
            src = self.empty((B, T_m), torch.int32)
            PMb = self.empty((T_m, B * N))
        else:
            src, PMb = out
        self._call("csm_bootstrap", _ptr(R), T_m, N, int(B), int(b0), ctypes.c_uint64(int(seed)),
                   float(mean_block), float(p0), _ptr(src), _ptr(PMb))
        return src, PMb

    def boot_scan(self, R, B, Js, skip=1, b0=0, seed=5000, mean_block=6.0, p0=100.0,
                  with_ids=True):
        """csm_boot_scan: bootstrap(R, B, ...) and momentum_multi(with_ids) in one pass, the panel
        never written -> (src [B][T_m], [(M, IDS)] per J (IDS None without ids), NR [T_m][B*N]
        next_ret shared by every J, bad [1] int32).  M / IDS equal momentum_multi's on
        bootstrap's panel bit for bit; NR equals each J's next_ret on every row J ranks unless
        bad is set (include/csmom.h)."""
        T_m, N = R.shape
        _need(R, "R", torch.float64, (T_m, N), self.device)
        Js = [int(J) for J in Js]
        nJ = len(Js)
        BN = B * N
        src = self.empty((B, T_m), torch.int32)
        # (the Js' panels back to back: a caller may rank them as one stacked decile pass)
        Ms = list(self.empty((len(Js), T_m, BN)))
        IDS = list(self.empty((len(Js), T_m, BN), torch.int16)) if with_ids else None
        NR = self.empty((T_m, BN))
        bad = torch.empty(1, dtype=torch.int32, device=self.device)
        arr = lambda ts: (ctypes.c_void_p * nJ)(*[t.data_ptr() for t in ts])
        self._call("csm_boot_scan", _ptr(R), T_m, N, int(B), int(b0), ctypes.c_uint64(int(seed)),
                   float(mean_block), float(p0), (ctypes.c_int32 * nJ)(*Js), nJ, int(skip),
                   _ptr(src), arr(Ms), arr(IDS) if with_ids else None, _ptr(NR), _ptr(bad))
        return src, list(zip(Ms, IDS if with_ids else [None] * nJ)), NR, bad

    def shard_summary(self, PM, J, skip, out=None, state=None):
        """csm_shard_summary (one pass over PM), or csm_shard_summary_state (short walks,
        the same record) when `state` from signal_shard is given."""
        T_m, N = PM.shape
        _need(PM, "PM", torch.float64, (T_m, N), self.device)
        S = 6 + J + skip + 1
        out = self.empty((S, N)) if out is None else out
        _need(out, "summary", torch.float64, (S, N), self.device)
        if state is not None:
            _need(state.t, "state", torch.float64, (5, N), self.device)
            self._call("csm_shard_summary_state", _ptr(state.P), _ptr(state.month_start),
                       _ptr(PM), T_m, N, int(J), int(skip), _ptr(state.t), _ptr(out))
        else:
            self._call("csm_shard_summary", _ptr(PM), T_m, N, int(J), int(skip), _ptr(out))
        return out

    def fold_carry(self, summaries, g, J, skip, carry=None, next_pm=None):
        G, S, N = summaries.shape
        if S != 6 + J + skip + 1:
            raise ValueError(f"summaries have {S} rows, expected {6 + J + skip + 1}")
        _need(summaries, "summaries", torch.float64, (G, S, N), self.device)
        carry = self.empty((J + skip + 2, N)) if carry is None else carry
        next_pm = self.empty((N,)) if next_pm is None else next_pm
        self._call("csm_fold_carry", _ptr(summaries), G, int(g), N, int(J), int(skip),
                   _ptr(carry), _ptr(next_pm))
        return carry, next_pm

    def signal_shard(self, P, month_start, max_month_days, J=12, skip=1, with_ret=False,
                     out=None, ids=None):
        """csm_signal_shard: the fused pass over this date shard from an empty scan state
        (speculative; shard_repair fixes it once the carry is known).  Returns
        (PM, R, M, NR, ShardState); PM holds only the shard's first / last J + skip + 8
        months (the rest are re-derived from P where needed).  ids (int16 [T_m][N], N % 4 ==
        0): also the fixed-map bucket id of every mom_J (csm_signal_shard_ids)."""
        T_d, N = P.shape
        T_m = month_start.numel() - 1
        _need(P, "P", torch.float64, (T_d, N), self.device)
        _need(month_start, "month_start", torch.int64, (T_m + 1,), self.device)
        if out is None:
            PM, M, NR = self.empty((T_m, N)), self.empty((T_m, N)), self.empty((T_m, N))
            R = self.empty((T_m, N)) if with_ret else None
            state = self.empty((5, N))
        else:
            PM, R, M, NR, state = out
        if ids is not None:
            _need(ids, "ids", torch.int16, (T_m, N), self.device)
            self._call("csm_signal_shard_ids", _ptr(P), T_d, N, _ptr(month_start), T_m,
                       int(max_month_days), int(J), int(skip), _ptr(PM), _ptr(R), _ptr(M),
                       _ptr(NR), _ptr(state), _ptr(ids))
        else:
            self._call("csm_signal_shard", _ptr(P), T_d, N, _ptr(month_start), T_m,
                       int(max_month_days), int(J), int(skip), _ptr(PM), _ptr(R), _ptr(M),
                       _ptr(NR), _ptr(state))
        return PM, R, M, NR, ShardState(state, P, month_start)

    def shard_repair(self, PM, carry, next_pm, state, M, NR, J, skip, R=None, ids=None):
        """csm_shard_repair: turn the outputs of signal_shard (M, NR, R rewritten in place)
        into those of the scan from `carry`, and finish the pending rows with `next_pm` (both
        from fold_carry)."""
        T_m, N = PM.shape
        W = J + skip
        _need(PM, "PM", torch.float64, (T_m, N), self.device)
        _need(carry, "carry", torch.float64, (W + 2, N), self.device)
        _need(next_pm, "next_pm", torch.float64, (N,), self.device)
        _need(state.t, "state", torch.float64, (5, N), self.device)
        for t, nm in ((M, "M"), (NR, "NR"), (R, "R")):
            if t is not None:
                _need(t, nm, torch.float64, (T_m, N), self.device)
        if ids is not None:   # rewrite the ids of the rewritten cells too
            _need(ids, "ids", torch.int16, (T_m, N), self.device)
            self._call("csm_shard_repair_ids", _ptr(state.P), _ptr(state.month_start), _ptr(PM),
                       T_m, N, int(J), int(skip), _ptr(carry), _ptr(next_pm), _ptr(state.t),
                       _ptr(R), _ptr(M), _ptr(NR), _ptr(ids))
        else:
            self._call("csm_shard_repair", _ptr(state.P), _ptr(state.month_start), _ptr(PM),
                       T_m, N, int(J), int(skip), _ptr(carry), _ptr(next_pm), _ptr(state.t),
                       _ptr(R), _ptr(M), _ptr(NR))
        return M, NR

    # ------------------------------------------------------------ halo date shards
    def shard_halo(self, P, month_start, H, F, J=12, skip=1, before=True, after=True, out=None):
        """csm_shard_halo: P holds H halo months, the shard and F (0..8) forward months
        (month_start [H + T_m + F + 1], day offsets into P); before / after: the panel has
        months before the halo / after the forward months.  Returns (carry [J+skip+2][N],
        next_pm [N], flags uint8 [N]; bit 0 carry uncertain, bit 1 next_pm uncertain)."""
        T_d, N = P.shape
        T_m = month_start.numel() - 1 - H - F
        _need(P, "P", torch.float64, (T_d, N), self.device)
        _need(month_start, "month_start", torch.int64, (H + T_m + F + 1,), self.device)
        if out is None:
            carry, npm = self.empty((J + skip + 2, N)), self.empty((N,))
            flags = self.empty((N,), torch.uint8)
        else:
            carry, npm, flags = out
        hpm = self.empty((max(H + F, 1), N))
        self._call("csm_shard_halo", _ptr(P), T_d, N, _ptr(month_start), int(H), int(T_m),
                   int(F), int(bool(before)), int(bool(after)), int(J), int(skip), _ptr(hpm),
                   _ptr(carry), _ptr(npm), _ptr(flags))
        return carry, npm, flags

    def signal_shard_halo(self, P, month_start, max_month_days, J, skip, carry, next_pm,
                          with_ret=False, out=None, ids=None):
        """csm_signal_shard_halo: signal_shard from the halo's carry / next_pm (month_start =
        the shard's T_m + 1 offsets into P).  Returns (PM, R, M, NR, ShardState)."""
        T_d, N = P.shape
        T_m = month_start.numel() - 1
        W = J + skip
        _need(P, "P", torch.float64, (T_d, N), self.device)
        _need(month_start, "month_start", torch.int64, (T_m + 1,), self.device)
        _need(carry, "carry", torch.float64, (W + 2, N), self.device)
        _need(next_pm, "next_pm", torch.float64, (N,), self.device)
        if out is None:
            PM, M, NR = self.empty((T_m, N)), self.empty((T_m, N)), self.empty((T_m, N))
            R = self.empty((T_m, N)) if with_ret else None
            state = self.empty((5, N))
        else:
            PM, R, M, NR, state = out
        if ids is not None:
            _need(ids, "ids", torch.int16, (T_m, N), self.device)
        self._call("csm_signal_shard_halo", _ptr(P), T_d, N, _ptr(month_start), T_m,
                   int(max_month_days), int(J), int(skip), _ptr(carry), _ptr(next_pm), _ptr(PM),
                   _ptr(R), _ptr(M), _ptr(NR), _ptr(state), _ptr(ids))
        return PM, R, M, NR, ShardState(state, P, month_start)

    @staticmethod
    def halo_fused_ok(N, max_month_days):
        """Whether csm_signal_halo (the halo prologue inside the wide shard kernel) takes this
        panel: even N >= 92160 (the four-wave blocks), months of <= 23 day rows."""
        return N % 2 == 0 and 92160 <= N < (1 << 31) // 256 and max_month_days <= 23

    def signal_halo(self, P, month_start, H, F, max_month_days, J, skip, before=True, after=True,
                    with_ret=False, ids=None):
        """csm_signal_halo: shard_halo + signal_shard_halo in one launch (halo_fused_ok
        panels).  month_start [H + T_m + F + 1] as shard_halo's.  Returns (PM, R, M, NR,
        ShardState, flags) -- ShardState on the shard's month offsets, flags shard_halo's."""
        T_d, N = P.shape
        T_m = month_start.numel() - 1 - H - F
        _need(P, "P", torch.float64, (T_d, N), self.device)
        _need(month_start, "month_start", torch.int64, (H + T_m + F + 1,), self.device)
        PM, M, NR = self.empty((T_m, N)), self.empty((T_m, N)), self.empty((T_m, N))
        R = self.empty((T_m, N)) if with_ret else None
        state = self.empty((5, N))
        flags = self.empty((N,), torch.uint8)
        if ids is not None:
            _need(ids, "ids", torch.int16, (T_m, N), self.device)
        self._call("csm_signal_halo", _ptr(P), T_d, N, _ptr(month_start), int(H), int(T_m), int(F),
                   int(bool(before)), int(bool(after)), int(max_month_days), int(J), int(skip),
                   _ptr(PM), _ptr(R), _ptr(M), _ptr(NR), _ptr(state), _ptr(ids), _ptr(flags))
        return PM, R, M, NR, ShardState(state, P, month_start[H:H + T_m + 1]), flags

    def shard_need(self, flags, state, H, out=None):
        """csm_shard_need -> int64 [4][ceil(N / 64)]: this rank's exchange bits (H = the halo
        length the next rank holds)."""
        N = flags.numel()
        T_m = state.month_start.numel() - 1
        mask = self.empty((4, (N + 63) // 64), torch.int64) if out is None else out
        self._call("csm_shard_need", _ptr(flags), _ptr(state.t), N, T_m, int(H), _ptr(mask))
        return mask

    def shard_union(self, masks, N, cap, out=None):
        """csm_shard_union over the gathered bits [G][4][ceil(N / 64)] -> (idx int32 [cap],
        count int32 [1]) on the device (no sync)."""
        G = masks.shape[0]
        _need(masks, "masks", torch.int64, (G, 4, (N + 63) // 64), self.device)
        idx, cnt = ((self.empty((cap,), torch.int32), self.empty((1,), torch.int32))
                    if out is None else out)
        self._call("csm_shard_union", _ptr(masks), G, N, int(cap), _ptr(idx), _ptr(cnt))
        return idx, cnt

    def shard_summary_cols(self, PM, state, idx, cnt, J, skip, out=None):
        """csm_shard_summary_cols: the exchange record [S][cap] of the listed assets."""
        T_m, N = PM.shape
        cap = idx.numel()
        S = 6 + J + skip + 1
        out = self.empty((S, cap)) if out is None else out
        _need(out, "summary", torch.float64, (S, cap), self.device)
        self._call("csm_shard_summary_cols", _ptr(state.P), _ptr(state.month_start), _ptr(PM),
                   T_m, N, int(J), int(skip), _ptr(state.t), _ptr(idx), _ptr(cnt), cap,
                   _ptr(out))
        return out

    def shard_repair_cols(self, PM, carry, next_pm, fcarry, state, idx, cnt, M, NR, J, skip,
                          R=None, ids=None):
        """csm_shard_repair_cols: repair the listed assets from their folded carry / next_pm
        columns ([.][cap]); fcarry = the halo carry the pass started from."""
        T_m, N = PM.shape
        cap = idx.numel()
        W = J + skip
        _need(carry, "carry", torch.float64, (W + 2, cap), self.device)
        _need(next_pm, "next_pm", torch.float64, (cap,), self.device)
        _need(fcarry, "fcarry", torch.float64, (W + 2, N), self.device)
        self._call("csm_shard_repair_cols", _ptr(state.P), _ptr(state.month_start), _ptr(PM),
                   T_m, N, int(J), int(skip), _ptr(carry), _ptr(next_pm), _ptr(fcarry),
                   _ptr(state.t), _ptr(idx), _ptr(cnt), cap, _ptr(R), _ptr(M), _ptr(NR),
                   _ptr(ids))
        return M, NR

    def shard_fix_cols(self, PM, records, g, state, idx, cnt, M, NR, J, skip, R=None, ids=None):
        """csm_shard_fix_cols: fold the listed columns' all-gathered records [G][S][cap] (this
        rank g) and replay every month of each listed column from its true carry, in one launch
        (the halo pass's fold_carry + shard_repair_cols)."""
        T_m, N = PM.shape
        G, S, cap = records.shape
        if S != 6 + J + skip + 1:
            raise ValueError(f"records have {S} rows, expected {6 + J + skip + 1}")
        _need(records, "records", torch.float64, (G, S, cap), self.device)
        _need(idx, "idx", torch.int32, (cap,), self.device)
        _need(M, "M", torch.float64, (T_m, N), self.device)
        _need(NR, "NR", torch.float64, (T_m, N), self.device)
        if ids is not None:
            _need(ids, "ids", torch.int16, (T_m, N), self.device)
        self._call("csm_shard_fix_cols", _ptr(state.P), _ptr(state.month_start), _ptr(PM),
                   T_m, N, int(J), int(skip), _ptr(records), G, int(g), _ptr(idx), _ptr(cnt), cap,
                   _ptr(R), _ptr(M), _ptr(NR), _ptr(ids))
        return M, NR

    def sync(self):
        self._call("csm_sync")

    # ------------------------------------------------------------------ pipeline
    def use_fused(self, P, V=None, max_month_days=None) -> bool:
        T_d, N = P.shape
        return (V is None and N >= FUSED_MIN_N and max_month_days is not None
                and max_month_days <= 32)

    def run(self, P, month_start, J=12, skip=1, n_bins=10, V=None, with_ret=False,
            max_month_days=None, fused=None):
        """One full pass: month-end -> signal -> labels + EW decile means -> long-short.
        Large panels take the fused month-end + scan kernel (no PM round trip)."""
        T_m, N = month_start.numel() - 1, P.shape[1]
        min_month_days = None
        if max_month_days is None and T_m > 0:
            max_month_days, min_month_days = self.month_days(month_start)
        if fused is None:
            fused = self.use_fused(P, V, max_month_days)
        if fused:   # one C call: signal (+ bucket ids for wide rows) -> deciles -> long-short
            return self.pipeline(P, month_start, J, skip, n_bins, max_month_days, with_pm=True,
                                 with_ret=with_ret, min_month_days=min_month_days)
        else:
            PM, VOL = self.month_end(P, month_start, V)
            if self.default_chunks(T_m, N, J, skip) > 1:
                R, M, NR = self.momentum_chunked(PM, J, skip, with_ret=with_ret)
            else:
                R, M, NR = self.momentum(PM, J, skip, with_ret=with_ret)
        L, EW, CNT, NV = self.deciles(M, NR, n_bins, with_nv=True)
        LS = self.long_short(EW, CNT)
        return PipelineOut(PM=PM, M=M, NR=NR, L=L, EW=EW, CNT=CNT, LS=LS, R=R, VOL=VOL, NV=NV)
