"""bench.py's multi-rank path, rehearsed on ONE GPU with 2 ranks on cuda:0 and `--backend gloo`.

Two launch forms:
  * the driver's own: `python bench.py --gpus 2 ...` with no torchrun environment -- bench.py
    starts the two worker processes itself (spawn_workers: each initialises the GPU itself, the
    parent never touches it), rank 0 prints the line;
  * torchrun's environment set by the test (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*), the
    workers spawned with multiprocessing.
Every rank runs the same collectives the RCCL run makes (the date-shard pass with its two
all-gathers, the strategy-shard all-gather, the barriers, the max-over-ranks timing, the
rank-summed decile match), so a rank-0-only collective would hang here (bounded by a timeout)
instead of on the driver's 8-GPU node.

C4 (custom size, strong scaling = BASELINE C4's form: ONE global panel date-sharded over the
ranks): rank 0's line must report a 100 % decile match over both ranks' dates, and its
long-short series must equal, bit for bit, the 1-GPU csm_pipeline over the concatenated panel.
C3: the (J, K) grid split over the ranks; the gathered table equals the 1-process run_batch
bit for bit.  C5 (8 panels, batches of 4): the panels split over the ranks; the gathered summary
table equals the 1-process SweepRunner's.
"""
import json
import os
import socket
import subprocess
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


def _self_launch(argv, timeout=300):
    """`python bench.py <argv>` exactly as the driver runs it (no torchrun environment)."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                        "MASTER_PORT")}
    r = subprocess.run([sys.executable, "-u", str(ROOT / "bench.py"), *argv], env=env,
                       capture_output=True, text=True, timeout=timeout, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]            # rank 0 only
    return json.loads(lines[0])


def _c4_one_gpu(engine, N, total, seed):
    """The global panel of a 2-rank C4 run on one GPU: both date shards, concatenated."""
    from csmom.synth import make_device_panel, shard_calendar
    parts = []
    for r in range(WORLD):
        days, ms, _, _ = shard_calendar("1985-01-01", total, WORLD, r)
        parts.append(make_device_panel(N, days, ms, seed=seed * 1000 + r, device=engine.device,
                                       shard=(r, WORLD, seed, total / WORLD)))
    P = torch.cat([p.P for p in parts], 0).contiguous()
    ms_all, off = [0], 0
    for p in parts:
        ms_all.extend((p.month_start_host[1:] + off).tolist())
        off += p.P.shape[0]
    msd = torch.tensor(ms_all, dtype=torch.int64, device=engine.device)
    return engine.pipeline(P, msd, 12, 1, 10)


def test_bench_c4_self_launch_strong_scaling(engine, tmp_path):
    """`bench.py --gpus 2` as the driver invokes it: the fixed panel (strong scaling, the
    default) date-sharded over 2 self-launched ranks; LS / EW / CNT equal the 1-GPU pipeline."""
    # wide enough for the fused shard pass with bucket ids (N >= 32768, N % 4 == 0): each rank
    # ranks its months exactly as the one-GPU csm_pipeline does, so the means are bit-identical
    N, DAYS, SEED = 40_000, 2_200, 4
    dump = tmp_path / "c4s.npz"
    line = _self_launch(["--gpus", "2", "--backend", "gloo", "--assets", str(N), "--days",
                         str(DAYS), "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                         "--seed", str(SEED), "--dump", str(dump)])
    assert line["n_gpus"] == 2 and line["decile_match_pct"] == 100.0
    assert line["scaling"] == "strong" and line["config"]["bdays"] == DAYS
    assert line["engine_path"].startswith("halo date shards")     # the default sharded pass
    assert 0 <= line["halo"]["listed_assets"] <= line["halo"]["list_width"]
    assert line["config"]["parallelism"] == "date-shard x2"
    assert abs(line["value"] - N * DAYS * line["steps"] / (line["ms_per_step"] * 1e-3 * line["steps"])) \
        <= 1e-6 * line["value"]
    one = _c4_one_gpu(engine, N, DAYS, SEED)
    got = np.load(dump)
    assert bits_equal(got["LS"], one.LS.cpu().numpy())
    assert bits_equal(got["EW"], one.EW.cpu().numpy())
    assert np.array_equal(got["CNT"], one.CNT.cpu().numpy())


def test_bench_c4_two_ranks_gloo(engine, tmp_path):
    """torchrun's environment, weak scaling: every rank a DAYS-long month range; the
    speculative all-gather pass (--shard-mode fused)."""
    N, DAYS, SEED = 40_000, 1_100, 4
    dump = tmp_path / "c4.npz"
    line = _spawn_bench(["--gpus", "2", "--backend", "gloo", "--assets", str(N), "--days",
                         str(DAYS), "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                         "--seed", str(SEED), "--dump", str(dump), "--scaling", "weak",
                         "--shard-mode", "fused"])
    assert line["n_gpus"] == 2 and line["decile_match_pct"] == 100.0
    assert "all 2 ranks" in line["decile_check"]
    assert line["engine_path"].startswith("speculative fused")
    one = _c4_one_gpu(engine, N, DAYS * WORLD, SEED)   # both shards of the global panel
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


def test_bench_c5_self_launch(engine, tmp_path):
    dump = tmp_path / "c5s.npz"
    line = _self_launch(["--gpus", "2", "--backend", "gloo", "--config", "c5", "--panels", "8",
                         "--batch", "4", "--steps", "1", "--warmup", "1", "--no-cpu-baseline",
                         "--dump", str(dump)])
    assert line["n_gpus"] == 2 and line["config"]["panels"] == 8
    assert line["config"]["parallelism"] == "panel-shard x2"
    assert np.load(dump)["table"].shape == (8, 16, 7)


def test_bench_c3_strategy_shards_self_launch(engine, tmp_path):
    """C3 at N = 2: the 16 strategies split over the ranks (SweepRunner.run_batch_sharded), one
    all-gather; the table equals the 1-process run_batch on the same panel bit for bit."""
    import csmom
    from csmom.synth import bday_calendar, make_device_panel
    N, T_d = 1_000, 2_600
    dump = tmp_path / "c3s.npz"
    line = _self_launch(["--gpus", "2", "--backend", "gloo", "--config", "c3", "--assets", str(N),
                         "--days", str(T_d), "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                         "--dump", str(dump)])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "strategy-shard x2"
    assert line["scaling"] == "strong"
    seed = 4 * 1000 + 3
    days, ms, _ = bday_calendar("2000-01-03", T_d)
    panel = make_device_panel(N, days, ms, seed=seed, device=engine.device)
    g = torch.Generator(device=engine.device)
    g.manual_seed(seed)
    shares = torch.exp(torch.randn(N, generator=g, device=engine.device, dtype=torch.float64) + 16.0)
    rate = torch.rand(N, generator=g, device=engine.device, dtype=torch.float64) * 0.018 + 0.002
    PM, _ = engine.month_end(panel.P, panel.month_start)
    W = PM.abs() * shares
    cfg = csmom.SweepConfig(Js=(3, 6, 9, 12), Ks=(3, 6, 9, 12), skip=1, aum=1e8)
    one, _ = csmom.SweepRunner(engine, cfg).run_batch(PM, 1, W=W, ADV=W * rate)
    assert bits_equal(np.load(dump)["table"], one.cpu().numpy())
