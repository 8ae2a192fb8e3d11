"""Date-sharded multi-GPU pipeline: one process per GPU, torch.distributed over RCCL/xGMI.

Each rank owns a contiguous range of whole calendar months of the daily panel (month-end
aggregation is month-local, so no daily halo is exchanged).  The per-asset scan needs the
state the earlier months leave behind (ret window, ffilled price, subset-ffilled price) and
the first month price after the shard (next_ret of the shard's last ranked row).  Both are
rebuilt exactly from one all-gather of prefix-independent per-asset shard summaries
([S][N] f64, S = 6 + J + skip + 1).  After ranking and the per-date decile means, a second
all-gather of the per-date [T_m_local][n_bins] mean/count rows gives every rank the full
series; the long-short needs panel-wide column existence (run_demo.py:60-65).

Two collectives per pass; no collective touches daily data.  The default sharded pass
(run_halo) gives each rank a lookback halo of daily rows instead, so the exchange shrinks to the
few assets the halo does not settle (collective 1 then moves N / 8 bytes of need bits and a
fixed-width record of the listed assets).  The stage implementation is
injected: `Engine` on the GPU (the product), anything with the same methods elsewhere (the
CPU tests drive this orchestration with gloo and the oracle).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


def month_partition(T_m: int, G: int):
    """Contiguous month ranges, earlier ranks take the remainder."""
    base, rem = divmod(T_m, G)
    out, m0 = [], 0
    for g in range(G):
        m1 = m0 + base + (1 if g < rem else 0)
        out.append((m0, m1))
        m0 = m1
    return out


def all_gather_stack(x: torch.Tensor, group=None) -> torch.Tensor:
    """[G, *x.shape] all-gather; RCCL gets the single-buffer form, gloo the list form (device
    tensors staged through host memory: gloo's all-gather is host-only)."""
    G = dist.get_world_size(group)
    if G == 1:
        return x.unsqueeze(0)
    if dist.get_backend(group) == "nccl":
        out = torch.empty((G,) + tuple(x.shape), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out.view(-1), x.contiguous().view(-1), group=group)
        return out
    xs = x.detach().contiguous().cpu()
    out = torch.empty((G,) + tuple(x.shape), dtype=x.dtype)
    dist.all_gather(list(out.unbind(0)), xs, group=group)
    return out.to(x.device)


class CsmCollective:
    """The date-shard all-gathers through libcsmom.so's own RCCL communicator (csm_comm_unique_id
    / csm_allgather_init / csm_allgather, include/csmom.h) -- the collectives a non-Python host
    makes.  The 128-byte unique id travels over an existing process group (any backend); the
    gathers run on the engine's current HIP stream.  Drop-in for all_gather_stack in
    DateShardPipeline(collective=...)."""

    def __init__(self, engine, group=None):
        import ctypes
        self.eng = engine
        self.G = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        uid = (ctypes.c_ubyte * 128)()
        if self.rank == 0:
            st = engine.lib.csm_comm_unique_id(ctypes.cast(uid, ctypes.c_void_p))
            if st != 0:
                raise RuntimeError(f"csm_comm_unique_id failed ({st})")
        if self.G > 1:
            box = [bytes(uid)]
            dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group else 0,
                                       group=group)
            uid = (ctypes.c_ubyte * 128).from_buffer_copy(box[0])
        engine._call("csm_allgather_init", ctypes.cast(uid, ctypes.c_void_p), self.rank, self.G)

    def all_gather_stack(self, x: torch.Tensor) -> torch.Tensor:
        import ctypes
        x = x.contiguous()
        out = torch.empty((self.G,) + tuple(x.shape), dtype=x.dtype, device=x.device)
        self.eng._call("csm_allgather", ctypes.c_void_p(x.data_ptr()),
                       ctypes.c_void_p(out.data_ptr()), x.numel() * x.element_size())
        return out

    def close(self):
        self.eng._call("csm_allgather_free")


@dataclass
class ShardResult:
    M: torch.Tensor      # [T_m_local][N] mom_J of this rank's months
    NR: torch.Tensor     # [T_m_local][N] next_ret
    L: torch.Tensor      # [T_m_local][N] labels
    EW: torch.Tensor     # [T_m_total][n_bins] all ranks' decile means (rank order)
    CNT: torch.Tensor    # [T_m_total][n_bins]
    LS: torch.Tensor     # [T_m_total] long-short, NaN = dropped


class DateShardPipeline:
    """Runs one pass of the hot path on this rank's month range.

    stages: object with month_end, shard_summary, fold_carry, momentum, deciles, long_short
    (the `Engine` method signatures); with fused=True also signal and shard_repair.
    months_per_rank: local month counts of all ranks (fixed for a run, so no size exchange
    happens per pass).

    fused=False: month-end, summary, collective 1, carry, scan from the carry (the carry is
    needed before the scan starts, so month-end and scan are separate passes).
    fused=True (speculative): the fused signal pass runs from an empty state at once (one
    read of the daily panel; PM and a small end-state record written for the exchange), the
    summary comes from short walks at both ends, collective 1 follows, and shard_repair
    rewrites the outputs of the first months where the true carry changes them --
    bit-identical to fused=False (tests/test_gpu_shards_api.py).
    """

    def __init__(self, stages, months_per_rank, J=12, skip=1, n_bins=10, group=None,
                 fused=False, collective=None, halo=None, fwd=None):
        self.st = stages
        # collective: None = torch.distributed (all_gather_stack), or a CsmCollective
        self.gather = (collective.all_gather_stack if collective is not None
                       else (lambda x: all_gather_stack(x, group)))
        self.months = list(months_per_rank)
        self.J, self.skip, self.n_bins = J, skip, n_bins
        self.group = group
        self.fused = fused
        self.G = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if len(self.months) != self.G:
            raise ValueError(f"months_per_rank has {len(self.months)} entries for {self.G} ranks")
        self.Tmax = max(self.months)
        # run_halo: the lookback months every rank holds (rank r: min(halo, its first month))
        self.halo = halo_months(J, skip) if halo is None else int(halo)
        # ... and the forward months after it (the next rank's first ones)
        self.fwd = FWD_MONTHS if fwd is None else int(fwd)
        self._rows = {}   # collective 2's row index (every rank's months in order), per device

    def _check_months(self, T_m):
        if T_m != self.months[self.rank]:
            raise ValueError(f"rank {self.rank}: {T_m} months, partition says {self.months[self.rank]}")

    def run(self, P_local, month_start_local, max_month_days=None) -> ShardResult:
        st, J, s = self.st, self.J, self.skip
        if self.fused:
            if max_month_days is None:
                raise ValueError("the fused shard pass needs max_month_days")
            T_m = month_start_local.numel() - 1
            self._check_months(T_m)
            if self.G == 1:
                if _wants_ids(st, P_local):                                   # = csm_pipeline
                    _, _, M, NR, ids = st.signal_ids(P_local, month_start_local, max_month_days,
                                                     J, s)
                    return self._rank_and_gather(M, NR, ids)
                _, _, M, NR = st.signal(P_local, month_start_local, max_month_days, J, s)
                return self._rank_and_gather(M, NR)
            ids = _shard_ids(st, P_local, month_start_local)
            PM, _, M, NR, state = st.signal_shard(P_local, month_start_local, max_month_days,
                                                  J, s, **({} if ids is None else {"ids": ids}))
            summary = st.shard_summary(PM, J, s, state=state)
            summaries = self.gather(summary)                           # collective 1
            carry, next_pm = st.fold_carry(summaries, self.rank, J, s)
            st.shard_repair(PM, carry, next_pm, state, M, NR, J, s,
                            **({} if ids is None else {"ids": ids}))
            return self._rank_and_gather(M, NR, ids)
        PM, _ = st.month_end(P_local, month_start_local)
        self._check_months(PM.shape[0])
        summary = st.shard_summary(PM, J, s)
        if self.G > 1:
            summaries = self.gather(summary)                           # collective 1
            carry, next_pm = st.fold_carry(summaries, self.rank, J, s)
        else:
            carry, next_pm = None, None
        _, M, NR = st.momentum(PM, J, s, carry=carry, next_pm=next_pm)
        return self._rank_and_gather(M, NR)

    def fallback_cap(self, N):
        """Columns of the halo pass's fallback exchange: a fixed width per panel (no size
        exchange, no host sync), so collective 1b moves S x cap f64 per rank whatever G is."""
        return fallback_cap(N)

    def run_halo(self, P, month_start, H, F, max_month_days, check=True):
        """The halo date-shard pass (the default sharded path; north_star's "J + skip lookback
        halo").  P holds this rank's H halo months, its shard and F forward months;
        month_start [H + T_m + F + 1] are day offsets into P.

        1. shard_halo: the halo's scan state and the forward month's price (flags where either
           may differ from the whole history's);
        2. signal_shard_halo: the fused pass from that state -- final for unflagged assets;
        3. shard_need -> collective 1a (all-gather of N / 2 bytes: four bits per asset) ->
           shard_union:
           the ascending list of the assets any rank needs (the same on every rank);
        4. shard_summary_cols: the exchange record of the listed assets only -> collective 1b
           (all-gather of [S][cap] f64) -> fold_carry -> shard_repair_cols.
        Bit for bit the all-gather pass (tests/test_gpu_shards_api.py, the gloo tests).
        check=True: one sync to confirm the list fit its fixed width (else the pass reruns on
        the all-gather path); check=False leaves that to the caller (self.last_count)."""
        st, J, s = self.st, self.J, self.skip
        T_m = month_start.numel() - 1 - H - F
        self._check_months(T_m)
        N = P.shape[1]
        m0 = sum(self.months[:self.rank])
        rest = sum(self.months) - m0 - T_m   # months after this shard
        if H != min(self.halo, m0) or F != min(self.fwd, rest):
            raise ValueError(f"rank {self.rank}: P holds {H} halo / {F} forward months, the "
                             f"pipeline expects {min(self.halo, m0)} / {min(self.fwd, rest)}")
        msh = month_start[H:H + T_m + 1]
        ids = _shard_ids(st, P, msh)
        kw = {} if ids is None else {"ids": ids}
        if _halo_fused(st, P, max_month_days):   # one launch: halo prologue + shard
            carry_h = None
            PM, _, M, NR, state, flags = st.signal_halo(P, month_start, H, F, max_month_days, J,
                                                        s, before=m0 > H, after=rest > F, **kw)
        else:
            carry_h, npm_h, flags = st.shard_halo(P, month_start, H, F, J, s, before=m0 > H,
                                                  after=rest > F)
            PM, _, M, NR, state = st.signal_shard_halo(P, msh, max_month_days, J, s, carry_h,
                                                       npm_h, **kw)
        self.last_count = None
        if self.G > 1:
            cap = self.fallback_cap(N)
            # (row 3: rows before the part of this shard the NEXT rank's halo covers)
            Hn = min(self.halo, m0 + T_m)
            mask = st.shard_need(flags, state, Hn)
            masks = self.gather(mask)                                  # collective 1a
            idx, cnt = st.shard_union(masks, N, cap)
            rec = st.shard_summary_cols(PM, state, idx, cnt, J, s)
            recs = self.gather(rec)                                    # collective 1b
            self._fix_cols(PM, recs, carry_h, state, idx, cnt, M, NR, ids)
            self.last_count = (cnt, cap)
            if check and int(cnt.max().item()) > cap:   # every rank sees the same list
                return self._run_allgather_fallback(P, month_start, H, F, max_month_days)
        return self._rank_and_gather(M, NR, ids)

    def _fix_cols(self, PM, recs, carry_h, state, idx, cnt, M, NR, ids):
        """The listed columns from the all-gathered records: fold + replay in one launch
        (shard_fix_cols), or -- stages without it (the CPU oracle stages) -- fold_carry then
        shard_repair_cols."""
        st, J, s = self.st, self.J, self.skip
        kw = {} if ids is None else {"ids": ids}
        if hasattr(st, "shard_fix_cols"):
            st.shard_fix_cols(PM, recs, self.rank, state, idx, cnt, M, NR, J, s, **kw)
        else:
            carry_u, npm_u = st.fold_carry(recs, self.rank, J, s)
            st.shard_repair_cols(PM, carry_u, npm_u, carry_h, state, idx, cnt, M, NR, J, s, **kw)

    def _run_allgather_fallback(self, P, month_start, H, F, max_month_days):
        """The halo pass's list overflowed its width: the speculative all-gather pass on the
        shard's own rows (rare: more flagged assets than cap)."""
        T_m = month_start.numel() - 1 - H - F
        d0 = int(month_start[H].item())
        d1 = int(month_start[H + T_m].item())
        Ps = P[d0:d1].contiguous()
        msl = (month_start[H:H + T_m + 1] - d0).contiguous()
        fused = self.fused
        self.fused = True
        try:
            return self.run(Ps, msl, max_month_days)
        finally:
            self.fused = fused

    def _rank_and_gather(self, M, NR, ids=None) -> ShardResult:
        st, nb = self.st, self.n_bins
        T_m = M.shape[0]
        if ids is not None:   # rank from the bucket ids the shard pass wrote
            L, EW, CNT, _ = st.deciles_ids(M, NR, ids, nb)
        else:
            L, EW, CNT, _ = st.deciles(M, NR, nb)
        if self.G > 1:
            # one collective for both: counts ride as exact float64; the padding rows past a
            # rank's months are never read, so they stay unwritten
            packed = torch.empty((self.Tmax, 2 * nb), dtype=EW.dtype, device=EW.device)
            packed[:T_m, :nb] = EW
            packed[:T_m, nb:] = CNT
            allp = self.gather(packed)                                  # collective 2
            # every rank's months in order: one row gather over the stacked blocks
            key = (str(EW.device), nb)
            idx = self._rows.get(key)
            if idx is None:
                idx = torch.cat([torch.arange(m, dtype=torch.int64) + g * self.Tmax
                                 for g, m in enumerate(self.months)]).to(EW.device)
                self._rows[key] = idx
            flat = allp.reshape(self.G * self.Tmax, 2 * nb).index_select(0, idx)
            EW = flat[:, :nb].contiguous()
            CNT = flat[:, nb:].to(torch.int32)
        LS = st.long_short(EW, CNT)
        return ShardResult(M=M, NR=NR, L=L, EW=EW, CNT=CNT, LS=LS)


def _wants_ids(stages, P):
    """Whether the fused shard pass ranks from bucket ids: the engine, on the rows csm_pipeline
    ranks from ids too (N % 4 == 0, wider than the narrow-row decile kernels), so a sharded run's
    decile means are the one-GPU pipeline's bit for bit."""
    from .engine import DEC_NARROW_MAX
    N = P.shape[1]
    return bool(getattr(stages, "shard_ids", False)) and N % 4 == 0 and N > DEC_NARROW_MAX


def _shard_ids(stages, P, month_start):
    """An id buffer for the fused shard pass when _wants_ids; None: rank from mom_J."""
    if not _wants_ids(stages, P):
        return None
    return torch.empty((month_start.numel() - 1, P.shape[1]), dtype=torch.int16, device=P.device)


FWD_MONTHS = 3   # forward months a halo rank holds: next_pm is exact unless all three lack a row


def fallback_cap(N):
    """Width of the halo pass's fallback list: N / 32 columns (at least 2,048, at most N)."""
    return int(max(1, min(N, max(2048, N // 32))))


def halo_months(J, skip):
    """Calendar months of halo a rank holds before its shard: the window's J + skip present
    months plus three, so up to three absent / price-less months in the halo still leave the
    carry exact (k_shard_halo's test: two valid prices J + skip present months apart)."""
    return int(J) + int(skip) + 3


def halo_slices(month_start_host, G, H, fwd=None):
    """Per shard g of a G-way whole-month split: (d0, d1, hm, F, h0, m0, m1) -- the day range
    of its halo months, shard and forward months, the halo's month count, the forward month
    count F (fewer at the panel's end), and the first halo month, first shard month and end
    month."""
    import numpy as np
    ms = np.asarray(month_start_host, dtype=np.int64)
    T_m = len(ms) - 1
    out = []
    for (m0, m1) in month_partition(T_m, G):
        h0 = max(0, m0 - H)
        F = min(FWD_MONTHS if fwd is None else fwd, T_m - m1)
        out.append((int(ms[h0]), int(ms[m1 + F]), m0 - h0, F, h0, m0, m1))
    return out


# csm_signal_halo (the halo prologue inside the shard kernel) is bit for bit the two-launch
# csm_shard_halo + csm_signal_shard_halo, but its main loop runs slower on long shards (C4
# ranks, ms: 2-way 0.976 vs 0.086 + 0.873, 4-way 0.527 vs 0.079 + 0.443, 8-way 0.315 vs
# 0.091 + 0.232), so it is taken for shards of at most HALO_FUSED_MAX_DAYS days (halo and
# forward months included; CSM_HALO_FUSED_MAX_DAYS, 0 never);
# profiles/r06/experiments/negative_results.txt
HALO_FUSED_MAX_DAYS = int(os.environ.get("CSM_HALO_FUSED_MAX_DAYS", "2048"))


def _halo_fused(stages, P, max_month_days):
    """Whether the halo pass takes csm_signal_halo (halo prologue in the shard kernel)."""
    return (P.shape[0] <= HALO_FUSED_MAX_DAYS and hasattr(stages, "signal_halo")
            and stages.halo_fused_ok(P.shape[1], max_month_days))


def virtual_shards_halo(stages, P, month_start_host, G, J=12, skip=1, n_bins=10, H=None,
                        cap=None, fold_repair=False, fused_halo=None):
    """The halo pass's G-shard decomposition run sequentially on ONE device (the collectives
    replaced by stacks): every shard's halo state, fused pass, need mask, the union list, the
    listed records, fold and repair -- for single-GPU verification that a G-GPU halo run equals
    the 1-GPU run bit for bit.  Returns (M, NR, L, EW, CNT, LS, count) with count the union
    list's length.  fold_repair: the listed columns by fold_carry + shard_repair_cols (the
    convergence-tested repair) instead of the one-launch shard_fix_cols.  fused_halo: True
    takes csm_signal_halo where it applies, False shard_halo + signal_shard_halo, None the
    run_halo choice (shards of at most HALO_FUSED_MAX_DAYS days)."""
    import numpy as np
    H = halo_months(J, skip) if H is None else int(H)
    ms = np.asarray(month_start_host, dtype=np.int64)
    dev = P.device
    N = P.shape[1]
    cap = fallback_cap(N) if cap is None else int(cap)
    sh = []
    for (d0, d1, hm, F, h0, m0, m1) in halo_slices(ms, G, H):
        Pg = P[d0:d1].contiguous()
        msg = torch.from_numpy(ms[h0:m1 + F + 1] - d0).to(dev)
        msh = msg[hm:hm + (m1 - m0) + 1]
        maxd = int(np.diff(ms[m0:m1 + 1]).max()) if m1 > m0 else 1
        ids = _shard_ids(stages, Pg, msh)
        kw = {} if ids is None else {"ids": ids}
        if fused_halo is None:
            fh = _halo_fused(stages, Pg, maxd)
        else:
            fh = fused_halo and stages.halo_fused_ok(N, maxd)
        if fh and not fold_repair:
            carry_h = None
            PM, _, M, NR, state, flags = stages.signal_halo(Pg, msg, hm, F, maxd, J, skip,
                                                            before=h0 > 0,
                                                            after=m1 + F < len(ms) - 1, **kw)
        else:
            carry_h, npm_h, flags = stages.shard_halo(Pg, msg, hm, F, J, skip, before=h0 > 0,
                                                      after=m1 + F < len(ms) - 1)
            PM, _, M, NR, state = stages.signal_shard_halo(Pg, msh, maxd, J, skip, carry_h,
                                                           npm_h, **kw)
        sh.append((PM, M, NR, state, ids, carry_h, flags))
    masks = torch.stack([stages.shard_need(x[6], x[3], min(H, m1))
                         for x, (_, _, _, _, _, _, m1) in zip(sh, halo_slices(ms, G, H))])
    idx, cnt = stages.shard_union(masks, N, cap)
    if int(cnt.item()) > cap:   # (one sync: this helper verifies; a wider list, same columns)
        cap = int(cnt.item())
        idx, cnt = stages.shard_union(masks, N, cap)
    recs = torch.stack([stages.shard_summary_cols(x[0], x[3], idx, cnt, J, skip) for x in sh])
    Ms, NRs, Ls, EWs, CNTs = [], [], [], [], []
    for g, (PM, M, NR, state, ids, carry_h, _) in enumerate(sh):
        kw = {} if ids is None else {"ids": ids}
        if hasattr(stages, "shard_fix_cols") and not fold_repair:
            stages.shard_fix_cols(PM, recs, g, state, idx, cnt, M, NR, J, skip, **kw)
        else:
            carry_u, npm_u = stages.fold_carry(recs, g, J, skip)
            stages.shard_repair_cols(PM, carry_u, npm_u, carry_h, state, idx, cnt, M, NR, J, skip,
                                     **kw)
        if ids is not None:
            L, EW, CNT, _ = stages.deciles_ids(M, NR, ids, n_bins)
        else:
            L, EW, CNT, _ = stages.deciles(M, NR, n_bins)
        Ms.append(M); NRs.append(NR); Ls.append(L); EWs.append(EW); CNTs.append(CNT)
    EW = torch.cat(EWs).contiguous()
    CNT = torch.cat(CNTs).contiguous()
    LS = stages.long_short(EW, CNT)
    return torch.cat(Ms), torch.cat(NRs), torch.cat(Ls), EW, CNT, LS, int(cnt.max().item())


def virtual_shards(stages, P, month_start_host, G, J=12, skip=1, n_bins=10, fused=False):
    """Run the G-shard decomposition sequentially on ONE device (no collectives): the same
    summary / fold / scan kernels as DateShardPipeline (fused=True: the speculative signal +
    shard_repair path), for single-GPU verification that a G-GPU run equals the 1-GPU run bit
    for bit.  Returns concatenated (M, NR, L, EW, CNT, LS)."""
    import numpy as np

    ms = np.asarray(month_start_host, dtype=np.int64)
    T_m = len(ms) - 1
    dev = P.device
    parts = month_partition(T_m, G)
    PMs, outs = [], []
    for (m0, m1) in parts:
        d0, d1 = ms[m0], ms[m1]
        msl = torch.from_numpy(ms[m0:m1 + 1] - d0).to(dev)
        if fused:
            maxd = int(np.diff(ms[m0:m1 + 1]).max()) if m1 > m0 else 1
            Pg = P[d0:d1].contiguous()
            ids = _shard_ids(stages, Pg, msl)
            PM, _, M, NR, state = stages.signal_shard(Pg, msl, maxd, J, skip,
                                                      **({} if ids is None else {"ids": ids}))
            outs.append((M, NR, state, ids))
        else:
            PM, _ = stages.month_end(P[d0:d1].contiguous(), msl)
            outs.append((None, None, None, None))
        PMs.append(PM)
    summaries = torch.stack([stages.shard_summary(PM, J, skip, state=outs[g][2])
                             for g, PM in enumerate(PMs)])
    Ms, NRs, Ls, EWs, CNTs = [], [], [], [], []
    for g, PM in enumerate(PMs):
        carry, next_pm = stages.fold_carry(summaries, g, J, skip)
        ids = None
        if fused:
            M, NR, state, ids = outs[g]
            stages.shard_repair(PM, carry, next_pm, state, M, NR, J, skip,
                                **({} if ids is None else {"ids": ids}))
        else:
            _, M, NR = stages.momentum(PM, J, skip, carry=carry, next_pm=next_pm)
        if ids is not None:
            L, EW, CNT, _ = stages.deciles_ids(M, NR, ids, n_bins)
        else:
            L, EW, CNT, _ = stages.deciles(M, NR, n_bins)
        Ms.append(M); NRs.append(NR); Ls.append(L); EWs.append(EW); CNTs.append(CNT)
    EW = torch.cat(EWs).contiguous()
    CNT = torch.cat(CNTs).contiguous()
    LS = stages.long_short(EW, CNT)
    return torch.cat(Ms), torch.cat(NRs), torch.cat(Ls), EW, CNT, LS
