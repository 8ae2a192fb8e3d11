"""bench.py's multi-rank path, rehearsed on ONE GPU: 2 spawned worker processes (each
initialises the GPU itself; nothing re-executes a process that has touched the GPU), both on
cuda:0, torchrun's environment (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*), `--backend gloo`.
Every rank runs the same collectives the RCCL run makes (the date-shard pass with its two
all-gathers, the barriers, the max-over-ranks timing, the rank-summed decile match), so a
rank-0-only collective would hang here (bounded by the queue timeout) instead of on the
driver's 8-GPU node.

C4 (custom size): the two date shards of ONE global panel; rank 0's line must report a 100 %
decile match over both ranks' dates, and its long-short series must equal, bit for bit, the
1-GPU csm_pipeline over the concatenated panel.  C5 (8 panels, batches of 4): the panels split
over the ranks; the gathered summary table equals the 1-process SweepRunner's.
"""
import json
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(Path(__file__).resolve().parent))
from conftest import bits_equal  # noqa: E402

pytestmark = pytest.mark.gpu
WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench_worker(rank, world, port, argv, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0", LOCAL_WORLD_SIZE=str(world))
    try:
        import bench
        out = bench.main(argv)
        q.put((rank, json.dumps(out) if out is not None else None))
    except BaseException as e:   # surface the worker's failure in the parent
        q.put((rank, "ERROR " + repr(e)))
        raise


def _spawn_bench(argv, timeout=200):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, WORLD, port, argv, q))
             for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=timeout) for _ in range(WORLD)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [r for r in res if isinstance(r[1], str) and r[1].startswith("ERROR")]
    assert not errs, errs
    for p in procs:
        assert p.exitcode == 0
    res = dict(res)
    assert res[1] is None            # only rank 0 prints / returns the line
    return json.loads(res[0])


def test_bench_c4_two_ranks_gloo(engine, tmp_path):
    from csmom.synth import make_device_panel, shard_calendar
    # wide enough for the fused shard pass with bucket ids (N >= 32768, N % 4 == 0): each rank
    # ranks its months exactly as the one-GPU csm_pipeline does, so the means are bit-identical
    N, DAYS, SEED = 40_000, 1_100, 4
    dump = tmp_path / "c4.npz"
    line = _spawn_bench(["--gpus", "2", "--backend", "gloo", "--assets", str(N), "--days",
                         str(DAYS), "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                         "--seed", str(SEED), "--dump", str(dump)])
    assert line["n_gpus"] == 2 and line["decile_match_pct"] == 100.0
    assert "all 2 ranks" in line["decile_check"]
    assert line["engine_path"].startswith("speculative fused")
    # the same global panel on one GPU: both shards, concatenated along the days
    total = DAYS * WORLD
    parts = []
    for r in range(WORLD):
        days, ms, _, _ = shard_calendar("1985-01-01", total, WORLD, r)
        parts.append(make_device_panel(N, days, ms, seed=SEED * 1000 + r, device=engine.device,
                                       shard=(r, WORLD, SEED, total / WORLD)))
    P = torch.cat([p.P for p in parts], 0).contiguous()
    ms_all, off = [0], 0
    for p in parts:
        ms_all.extend((p.month_start_host[1:] + off).tolist())
        off += p.P.shape[0]
    msd = torch.tensor(ms_all, dtype=torch.int64, device=engine.device)
    one = engine.pipeline(P, msd, 12, 1, 10)
    got = np.load(dump)
    assert bits_equal(got["LS"], one.LS.cpu().numpy())
    assert bits_equal(got["EW"], one.EW.cpu().numpy())
    assert np.array_equal(got["CNT"], one.CNT.cpu().numpy())


def test_bench_c5_two_ranks_gloo(engine, tmp_path):
    import csmom
    from csmom.synth import bday_calendar, make_device_panel
    dump = tmp_path / "c5.npz"
    line = _spawn_bench(["--gpus", "2", "--backend", "gloo", "--config", "c5", "--panels", "8",
                         "--batch", "4", "--steps", "1", "--warmup", "1", "--no-cpu-baseline",
                         "--dump", str(dump)])
    assert line["n_gpus"] == 2 and line["config"]["panels"] == 8
    # the 1-process run of the same sweep (bench.py's C5 base panel and runner settings)
    days, ms, _ = bday_calendar("2000-01-03", 6_522)
    panel = make_device_panel(5_000, days, ms, seed=4 * 1000 + 5, device=engine.device)
    PM0, _ = engine.month_end(panel.P, panel.month_start)
    R0, _, _ = engine.momentum(PM0, 12, 1, with_ret=True)
    cfg = csmom.SweepConfig(Js=(3, 6, 9, 12), Ks=(3, 6, 9, 12), skip=1, aum=1e8)
    one = csmom.SweepRunner(engine, cfg).run_bootstrap(R0, 8, seed=5000, mean_block=6.0,
                                                      batch=4).cpu().numpy()
    tab = np.load(dump)["table"]
    assert tab.shape == one.shape
    assert np.array_equal(np.isnan(tab), np.isnan(one))
    assert np.array_equal(tab[..., 0], one[..., 0])          # months per (panel, strategy)
    m = ~np.isnan(one)
    assert np.allclose(tab[m], one[m], rtol=1e-12, atol=1e-15)
