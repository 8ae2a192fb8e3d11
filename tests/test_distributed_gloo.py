"""Multi-process date sharding on CPU: DateShardPipeline (the orchestration the GPU ranks run
over RCCL) driven with gloo, world_size 2 and 3, with oracle-backed stages.  The sharded
result must equal the unsharded oracle bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import csmom_oracle as O


class OracleStages:
    """Engine-shaped stage adapter over the CPU oracle (test-only)."""

    def month_end(self, P, ms, V=None):
        PM, _ = O.month_end(P.numpy(), ms.numpy())
        return torch.from_numpy(PM), None

    def shard_summary(self, PM, J, skip, state=None):
        return torch.from_numpy(O.shard_summary(PM.numpy(), J, skip))

    def fold_carry(self, summaries, g, J, skip):
        return O.fold_carry(summaries.numpy(), g, J, skip)

    def momentum(self, PM, J=12, skip=1, carry=None, next_pm=None, **kw):
        R, M, NR, _ = O.momentum_scan(PM.numpy(), J, skip, state=carry, next_pm=next_pm)
        return torch.from_numpy(R), torch.from_numpy(M), torch.from_numpy(NR)

    def deciles(self, M, NR, n_bins=10, **kw):
        L = O.assign_deciles(M.numpy(), n_bins)
        EW, CNT, _ = O.portfolio_ew(L, NR.numpy(), n_bins)
        return (torch.from_numpy(L), torch.from_numpy(EW),
                torch.from_numpy(CNT.astype(np.int32)), None)

    def long_short(self, EW, CNT):
        return torch.from_numpy(O.long_short(EW.numpy(), CNT.numpy()))

    # fused (speculative) mode: the signal pass runs from an empty state; the repair stage
    # stands in for csm_shard_repair by rescanning from the carry (orchestration test only --
    # the kernel itself is checked on the GPU, tests/test_gpu_shards_api.py)
    def signal(self, P, ms, max_month_days, J=12, skip=1, with_pm=False, **kw):
        PM, _ = O.month_end(P.numpy(), ms.numpy())
        R, M, NR, _ = O.momentum_scan(PM, J, skip)
        return (torch.from_numpy(PM) if with_pm else None), torch.from_numpy(R), \
            torch.from_numpy(M), torch.from_numpy(NR)

    def signal_shard(self, P, ms, max_month_days, J=12, skip=1, **kw):
        PM, R, M, NR = self.signal(P, ms, max_month_days, J, skip, with_pm=True)
        return PM, R, M, NR, None

    def shard_repair(self, PM, carry, next_pm, state, M, NR, J, skip, R=None):
        _, M2, NR2, _ = O.momentum_scan(PM.numpy(), J, skip, state=carry, next_pm=next_pm)
        M.copy_(torch.from_numpy(M2))
        NR.copy_(torch.from_numpy(NR2))
        return M, NR

    # halo mode (DateShardPipeline.run_halo): the halo's state from an empty scan over its
    # month prices, flags by k_shard_halo's rule (two valid prices J + skip present months
    # apart), the listed assets' records, fold and rescan
    def shard_halo(self, P, ms, H, F, J=12, skip=1, before=True, after=True):
        P_, ms_ = P.numpy(), ms.numpy()
        T_m = len(ms_) - 1 - H - F
        N = P_.shape[1]
        flags = np.zeros(N, dtype=np.uint8)
        if H > 0:
            PMh, _ = O.month_end(P_[:ms_[H]], ms_[:H + 1])
            _, _, _, carry = O.momentum_scan(PMh, J, skip)
        else:
            PMh, carry = O.absent_like((0, N)), O.ScanState(N, J, skip)
        for a in range(N):
            pres = ~O.is_absent(PMh[:, a])
            vi = np.nonzero(~np.isnan(PMh[pres, a]))[0]
            if before and not (len(vi) and vi[-1] - vi[0] >= J + skip):
                flags[a] |= 1
        npm = O.absent_like(N)
        if F > 0:
            d0, d1 = ms_[H + T_m], ms_[H + T_m + F]
            pmf, _ = O.month_end(P_[d0:d1], ms_[H + T_m:H + T_m + F + 1] - d0)
            for f in range(F - 1, -1, -1):   # the first forward month with a row
                npm = np.where(O.is_absent(pmf[f]), npm, pmf[f])
        if after:
            flags[O.is_absent(npm)] |= 2
        return carry, torch.from_numpy(npm), torch.from_numpy(flags)

    def signal_shard_halo(self, P, msh, max_month_days, J, skip, carry, next_pm, **kw):
        P_, ms_ = P.numpy(), msh.numpy()
        PM, _ = O.month_end(P_[ms_[0]:ms_[-1]], ms_ - ms_[0])
        self._last_T_m = PM.shape[0]
        R, M, NR, _ = O.momentum_scan(PM, J, skip, state=carry, next_pm=next_pm.numpy())
        pres = ~O.is_absent(PM)
        # end state: present months, the pending ranked row, the first present month
        # (k_signal<SH>'s record)
        pend = np.full(PM.shape[1], -1.0)
        fm = np.full(PM.shape[1], -1.0)
        for a in range(PM.shape[1]):
            pr = np.nonzero(pres[:, a])[0]
            rows = np.nonzero(pres[:, a] & ~np.isnan(M[:, a]))[0]
            if len(rows) and rows[-1] == pr[-1]:
                pend[a] = rows[-1]
            if len(pr):
                fm[a] = pr[0]
        state = np.stack([pres.sum(0).astype(np.float64), pend, fm])
        return (torch.from_numpy(PM), torch.from_numpy(R), torch.from_numpy(M),
                torch.from_numpy(NR), torch.from_numpy(state))

    def shard_need(self, flags, state, H):
        f, st = flags.numpy(), state.numpy()
        N = len(f)
        rows = [((f & 1).astype(bool) & (st[0] > 0)), ((f & 2).astype(bool) & (st[1] >= 0)),
                st[0] > 0, None]
        T_m = self._last_T_m
        rows[3] = (st[2] >= 0) & (st[2] < T_m - H)
        words = np.zeros((4, (N + 63) // 64), dtype=np.uint64)
        for r, bits in enumerate(rows):
            for a in np.nonzero(bits)[0]:
                words[r, a >> 6] |= np.uint64(1) << np.uint64(a & 63)
        return torch.from_numpy(words.view(np.int64))

    def shard_union(self, masks, N, cap):
        m = masks.numpy().view(np.uint64)
        G = m.shape[0]
        bit = lambda g, r, a: bool((int(m[g, r, a >> 6]) >> (a & 63)) & 1)
        lst = []
        for a in range(N):
            need = False
            for g in range(G):
                hist = any(bit(h, 2, a) for h in range(g - 1)) or (g >= 1 and bit(g - 1, 3, a))
                later = any(bit(h, 2, a) for h in range(g + 1, G))
                need |= (bit(g, 0, a) and hist) or (bit(g, 1, a) and later)
            if need:
                lst.append(a)
        idx = np.zeros(cap, dtype=np.int32)
        idx[:min(cap, len(lst))] = lst[:cap]
        return torch.from_numpy(idx), torch.tensor([len(lst)], dtype=torch.int32)

    def shard_summary_cols(self, PM, state, idx, cnt, J, skip):
        cap, c = idx.numel(), min(int(cnt.item()), idx.numel())
        cols = O.absent_like((PM.shape[0], cap))
        cols[:, :c] = PM.numpy()[:, idx.numpy()[:c]]
        return torch.from_numpy(O.shard_summary(cols, J, skip))

    def shard_repair_cols(self, PM, carry, next_pm, fcarry, state, idx, cnt, M, NR, J, skip,
                          **kw):
        c = min(int(cnt.item()), idx.numel())
        if c == 0:
            return M, NR
        cols = idx.numpy()[:c]
        st = O.ScanState.__new__(O.ScanState)
        st.ring, st.pff, st.psff = carry.ring[:, :c], carry.pff[:c], carry.psff[:c]
        _, M2, NR2, _ = O.momentum_scan(PM.numpy()[:, cols], J, skip, state=st,
                                        next_pm=next_pm[:c])
        M[:, torch.from_numpy(cols.astype(np.int64))] = torch.from_numpy(M2)
        NR[:, torch.from_numpy(cols.astype(np.int64))] = torch.from_numpy(NR2)
        return M, NR


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, J, skip, q, fused=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import csmom  # noqa: F401
        from csmom.distributed import DateShardPipeline, month_partition
        from conftest import load_golden
        z = load_golden("edge")
        ms = z["month_start"].astype(np.int64)
        parts = month_partition(len(ms) - 1, world)
        m0, m1 = parts[rank]
        d0, d1 = ms[m0], ms[m1]
        P = torch.from_numpy(np.ascontiguousarray(z["P"][d0:d1]))
        msl = torch.from_numpy(ms[m0:m1 + 1] - d0)
        pipe = DateShardPipeline(OracleStages(), [b - a for a, b in parts], J, skip, 10,
                                 fused=fused)
        r = pipe.run(P, msl, int(np.diff(ms).max()))
        q.put((rank, r.M.numpy(), r.NR.numpy(), r.L.numpy(), r.EW.numpy(), r.CNT.numpy(),
               r.LS.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,J,skip,fused", [(2, 12, 1, False), (3, 3, 0, False),
                                                (2, 9, 2, False), (2, 12, 1, True),
                                                (3, 9, 2, True)])
def test_date_shards_gloo(world, J, skip, fused):
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    from conftest import bits_equal, load_golden
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, J, skip, q, fused)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    z = load_golden("edge")
    ref = O.pipeline(z["P"], z["month_start"], J, skip, 10)
    assert bits_equal(np.concatenate([r[1] for r in res]), ref["M"])
    assert bits_equal(np.concatenate([r[2] for r in res]), ref["NR"])
    assert np.array_equal(np.concatenate([r[3] for r in res]), ref["L"])
    for r in res:  # every rank holds the full per-date series
        assert bits_equal(r[4], ref["EW"])
        assert np.array_equal(r[5], ref["CNT"])
        assert bits_equal(r[6], ref["LS"])


def _worker_halo(rank, world, port, J, skip, H, cap, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import csmom  # noqa: F401
        from csmom.distributed import DateShardPipeline, halo_slices, month_partition
        from conftest import load_golden
        z = load_golden("edge")
        ms = z["month_start"].astype(np.int64)
        parts = month_partition(len(ms) - 1, world)
        d0, d1, hm, F, h0, m0, m1 = halo_slices(ms, world, H)[rank]
        P = torch.from_numpy(np.ascontiguousarray(z["P"][d0:d1]))
        msl = torch.from_numpy(ms[h0:m1 + F + 1] - d0)
        pipe = DateShardPipeline(OracleStages(), [b - a for a, b in parts], J, skip, 10,
                                 fused=False, halo=H)
        if cap is not None:
            pipe.fallback_cap = lambda N: cap
        r = pipe.run_halo(P, msl, hm, F, int(np.diff(ms).max()))
        cnt = int(pipe.last_count[0].item())
        q.put((rank, r.M.numpy(), r.NR.numpy(), r.L.numpy(), r.EW.numpy(), r.CNT.numpy(),
               r.LS.numpy(), cnt))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,J,skip,H,cap", [(2, 12, 1, 16, None), (3, 3, 0, 6, None),
                                                (3, 9, 2, 14, None), (2, 12, 1, 0, None),
                                                (3, 12, 1, 16, 1)])
def test_date_shards_halo_gloo(world, J, skip, H, cap):
    """The halo pass (run_halo: each rank's halo state, the need bits' all-gather, the listed
    assets' records all-gathered, fold and rescan) over gloo equals the unsharded oracle bit
    for bit -- with no halo (H = 0: every asset with history is listed) and with a list that
    overflows its width (cap = 1: the all-gather pass takes over)."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    from conftest import bits_equal, load_golden
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_halo, args=(r, world, port, J, skip, H, cap, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    z = load_golden("edge")
    ref = O.pipeline(z["P"], z["month_start"], J, skip, 10)
    assert bits_equal(np.concatenate([r[1] for r in res]), ref["M"])
    assert bits_equal(np.concatenate([r[2] for r in res]), ref["NR"])
    assert np.array_equal(np.concatenate([r[3] for r in res]), ref["L"])
    for r in res:
        assert bits_equal(r[4], ref["EW"])
        assert np.array_equal(r[5], ref["CNT"])
        assert bits_equal(r[6], ref["LS"])
    assert len({r[7] for r in res}) == 1          # one union list on every rank
    if H == 0:
        assert res[0][7] > 0


def test_shard_id_buffer_shape():
    """The fused shard pass's id buffer: [T_m][N] int16 exactly where csm_pipeline ranks from
    ids (N % 4 == 0, rows wider than the narrow kernels), None elsewhere (host tensors suffice:
    the helper only allocates)."""
    from csmom.distributed import _shard_ids, _wants_ids
    from csmom.engine import DEC_NARROW_MAX

    class S:
        shard_ids = True

    ms = torch.arange(0, 13 * 21, 21, dtype=torch.int64)    # 12 months
    wide = torch.zeros((1, DEC_NARROW_MAX + 4), dtype=torch.float64)
    ids = _shard_ids(S(), wide, ms)
    assert ids.shape == (12, DEC_NARROW_MAX + 4) and ids.dtype == torch.int16
    assert _shard_ids(S(), torch.zeros((1, DEC_NARROW_MAX), dtype=torch.float64), ms) is None
    assert _shard_ids(S(), torch.zeros((1, DEC_NARROW_MAX + 2), dtype=torch.float64), ms) is None
    assert not _wants_ids(OracleStages(), wide)
