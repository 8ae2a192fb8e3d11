"""The HIP shard kernels composed with a real process group: 2 worker processes (spawn: each
initialises the GPU itself; nothing re-executes a process that has touched the GPU), both on
cuda:0, gloo (CUDA tensors staged through host memory by all_gather_stack).

Date shards: DateShardPipeline(Engine, fused=True) -- k_signal<SH>, k_shard_summary_state,
collective 1, k_fold_carry, k_shard_repair, k_deciles, collective 2, k_long_short -- must equal
the one-process fused pass bit for bit (and the oracle).  Sweep shards: SweepRunner over the
bootstrap panels split across the 2 ranks equals the one-process run.  The RCCL ("nccl")
branch of all_gather_stack is the same call sequence; it needs one GPU per rank, so it runs
only on a multi-GPU node (bench.py --gpus N), never in this one-GPU suite.
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

sys.path.insert(0, str(Path(__file__).resolve().parent))
from conftest import bits_equal  # noqa: E402
from oracle import csmom_oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu
N_ASSETS, N_DAYS, SEED = 3000, 2600, 29


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _panel(n=N_ASSETS, days=N_DAYS):
    from oracle.synth_np import make_panel
    return make_panel(n, days, seed=SEED, start="1990-01-01", with_volume=False,
                      nan_day=0.02, absent_month=0.01, nan_month=0.005, cents=True)


def _date_worker(rank, world, port, J, skip, n, days, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import csmom
        from csmom.distributed import DateShardPipeline, month_partition
        eng = csmom.Engine(0)
        pan = _panel(n, days)
        ms = pan["month_start"].astype(np.int64)
        parts = month_partition(len(ms) - 1, world)
        m0, m1 = parts[rank]
        d0, d1 = ms[m0], ms[m1]
        P = torch.from_numpy(np.ascontiguousarray(pan["P"][d0:d1])).to(eng.device)
        msl = torch.from_numpy(ms[m0:m1 + 1] - d0).to(eng.device)
        pipe = DateShardPipeline(eng, [b - a for a, b in parts], J, skip, 10, fused=True)
        maxd = int(np.diff(ms[m0:m1 + 1]).max())
        r = pipe.run(P, msl, maxd)
        torch.cuda.synchronize()
        q.put((rank, r.M.cpu().numpy(), r.NR.cpu().numpy(), r.L.cpu().numpy(),
               r.EW.cpu().numpy(), r.CNT.cpu().numpy(), r.LS.cpu().numpy()))
    except Exception as e:   # surface the worker's failure in the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=150) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [r for r in res if isinstance(r[1], str)]
    assert not errs, errs
    for p in procs:
        assert p.exitcode == 0
    return sorted(res, key=lambda t: t[0])


@pytest.mark.parametrize("J,skip,n,days", [(12, 1, N_ASSETS, N_DAYS), (3, 0, N_ASSETS, N_DAYS),
                                           (12, 1, 20_000, 1_400)])
def test_date_shards_two_processes_equal_one_process(engine, J, skip, n, days):
    """2 ranks (gloo, both on cuda:0) run the fused shard pass, collectives included; equal to
    one process bit for bit.  The 20,000-asset case ranks from bucket ids on every rank and is
    compared with the one-GPU csm_pipeline (ids too)."""
    res = _spawn(_date_worker, 2, J, skip, n, days)
    pan = _panel(n, days)
    ms_h = pan["month_start"].astype(np.int64)
    Pd = torch.from_numpy(pan["P"]).to(engine.device)
    msd = torch.from_numpy(ms_h).to(engine.device)
    if n > 16384:
        one = engine.pipeline(Pd, msd, J, skip, 10)
    else:
        one = engine.run(Pd, msd, J, skip, 10, max_month_days=int(np.diff(ms_h).max()), fused=True)
    M = np.concatenate([r[1] for r in res])
    NR = np.concatenate([r[2] for r in res])
    L = np.concatenate([r[3] for r in res])
    assert bits_equal(M, one.M.cpu().numpy()) and bits_equal(NR, one.NR.cpu().numpy())
    assert np.array_equal(L, one.L.cpu().numpy())
    for r in res:   # every rank holds the full per-date series
        assert bits_equal(r[4], one.EW.cpu().numpy())
        assert np.array_equal(r[5], one.CNT.cpu().numpy())
        assert bits_equal(r[6], one.LS.cpu().numpy())
    ref = O.pipeline(pan["P"], ms_h, J, skip, 10)
    assert bits_equal(M, ref["M"]) and np.array_equal(L, ref["L"])


def _sweep_cfg():
    import csmom
    return csmom.SweepConfig(Js=(3, 12), Ks=(1, 6), skip=1, aum=1e8)


def _base_R(eng):
    pan = _panel()
    P = torch.from_numpy(pan["P"]).to(eng.device)
    ms = torch.from_numpy(pan["month_start"].astype(np.int64)).to(eng.device)
    PM, _ = eng.month_end(P, ms)
    R, _, _ = eng.momentum(PM, 12, 1, with_ret=True)
    return R


def _sweep_worker(rank, world, port, n_panels, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import csmom
        eng = csmom.Engine(0)
        R = _base_R(eng)
        out = csmom.SweepRunner(eng, _sweep_cfg()).run_bootstrap(R, n_panels, seed=5000,
                                                                 mean_block=6.0, batch=4)
        torch.cuda.synchronize()
        q.put((rank, out.cpu().numpy()))
    except Exception as e:
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_sweep_shards_two_processes_equal_one_process(engine):
    import csmom
    n_panels = 7
    res = _spawn(_sweep_worker, 2, n_panels)
    one = csmom.SweepRunner(engine, _sweep_cfg()).run_bootstrap(
        _base_R(engine), n_panels, seed=5000, mean_block=6.0, batch=4).cpu().numpy()
    for _, tab in res:       # every rank holds the whole [panels][strategies][fields] table
        assert tab.shape == one.shape
        assert np.array_equal(np.isnan(tab), np.isnan(one))
        assert np.array_equal(tab[..., 0], one[..., 0])
        m = ~np.isnan(one)
        assert np.allclose(tab[m], one[m], rtol=1e-12, atol=1e-15)


def test_csm_allgather_single_rank(engine):
    """The C-ABI collective (csm_comm_unique_id / csm_allgather_init / csm_allgather over RCCL)
    on a one-rank communicator: the gather returns the rank's buffer, on the engine's stream;
    the date-shard pass driven through it equals the torch.distributed one (G = 1: no gather
    runs, the construction and the call sequence are exercised).  Two ranks need two GPUs
    (RCCL rejects two ranks on one device): bench.py --collective csm on the driver's node."""
    from csmom.distributed import CsmCollective
    coll = CsmCollective(engine)
    try:
        x = torch.arange(1000, dtype=torch.float64, device=engine.device) * 0.5
        y = coll.all_gather_stack(x)
        torch.cuda.synchronize()
        assert tuple(y.shape) == (1, 1000) and torch.equal(y[0], x)
        ids = torch.randint(0, 1 << 15, (7, 33), dtype=torch.int16, device=engine.device)
        assert torch.equal(coll.all_gather_stack(ids)[0], ids)
    finally:
        coll.close()
    assert engine.lib.csm_allgather(engine.ctx, None, None, 8) != 0   # freed: no communicator
