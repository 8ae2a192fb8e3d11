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
