#!/usr/bin/env python3
"""Benchmark: asset-days backtested per second on the fused signal -> rank -> portfolio pass.

Workload (BASELINE.json north_star / configs[3]): C4 = 100,000 assets x 10,000 business days
(bdate_range('1985-01-01'), 461 months), J=12 skip=1 K=1 equal-weight deciles, long-short.
N GPUs = one process per GPU over RCCL: `python bench.py --gpus N` starts the N worker
processes itself (or run it under torchrun).  C4 at N > 1 date-shards the FIXED 100k x 10k
panel in whole months (--scaling strong, the default); --scaling weak gives every rank a
C4-sized month range of an N x 10,000-day panel.

A step = one full pass over the resident panel: month-end aggregation, [summary all-gather +
carry fold when N>1], ret/mom/next_ret scan, per-date qcut labels fused with decile means,
[per-date row all-gather when N>1], long-short.  Inputs are in HBM before timing starts.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path
from types import SimpleNamespace

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
SWEEP_CONFIGS = {
    "c3": dict(N=5_000, days=6_522, start="2000-01-03", panels=1,
               name="C3: J x K grid J,K in {3,6,9,12}, K-overlapping value-weighted portfolios "
                    "with turnover + spread/sqrt-impact costs, 5k assets x 25y bdays (6522)"),
    "c5": dict(N=5_000, days=6_522, start="2000-01-03", panels=1000,
               name="C5: 1000 stationary-bootstrap month panels x 16 (J,K) strategies with "
                    "turnover + costs, base panel 5k assets x 25y bdays, panel-sharded"),
}
CONFIGS = {
    "c4": dict(N=100_000, days=10_000, start="1985-01-01",
               name="C4: 100k assets x 10k bdays, J=12 skip=1 K=1 EW decile long-short"),
    "c2": dict(N=5_000, days=6_522, start="2000-01-03",
               name="C2: 5k assets x 25y bdays (6522), J=12 skip=1 K=1 EW decile long-short"),
}


# The reference's pandas path (features.py:5-107, run_demo.py:41-67), timed in the survey
# container on a 10,000 x 10,000-day proxy of C4: context for the line, not
# measured by bench.py (the reference does not travel to the GPU box).
REFERENCE_PANDAS = {"value": 1.41e6, "unit": "asset-days/s", "cores": 1, "kind": "reference",
                    "value_excluding_turnover": 2.65e6,
                    "c4_seconds_extrapolated": 720.0, "c4_seconds_excluding_turnover": 380.0,
                    "where": "survey container, 8-core Xeon VM, pandas 2.3.3 (1 core); "
                             "BASELINE.md, C4 proxy 1e8 asset-days, extrapolated linearly"}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS) + sorted(SWEEP_CONFIGS))
    ap.add_argument("--panels", type=int, default=None, help="C5: bootstrap panels (total)")
    ap.add_argument("--batch", type=int, default=200, help="C5: panels per device batch (200: 56.2-57.1 vs 59.1-59.4 ms/step at 100, 60.4 at 250, same box; profiles/r04/experiments/batch/)")
    ap.add_argument("--assets", type=int, default=None)
    ap.add_argument("--days", type=int, default=None)
    ap.add_argument("--scaling", default="strong", choices=["weak", "strong"],
                    help="C4 / C2 at N > 1: strong = the fixed panel date-sharded over the ranks "
                         "(BASELINE C4), weak = every rank a full-size month range")
    ap.add_argument("--shard-mode", default="halo", choices=["halo", "fused", "unfused"],
                    help="N>1 date shards: halo (each rank holds J + skip + 3 lookback months of "
                         "daily rows; only the assets the halo leaves uncertain are exchanged), "
                         "speculative fused signal + all-gather + repair, or month-end + carried "
                         "scan")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-assets", type=int, default=150000)   # ~10-15 s of oracle time
    ap.add_argument("--seed", type=int, default=4)
    ap.add_argument("--no-ids", action="store_true",
                    help="C4 / C2: decile pass streams mom_J (k_deciles) instead of the bucket ids "
                         "the signal kernel (C4: csm_signal_ids) or the time-chunked scan (C2: "
                         "csm_momentum_chunked_ids) writes")
    ap.add_argument("--no-fused-ls", action="store_true",
                    help="C4 / C2 on ids: the long-short as its own launch (csm_long_short) "
                         "instead of the decile pass's last workgroup (csm_deciles_ids_ls)")
    ap.add_argument("--chunks", type=int, default=0,
                    help="C2 / C3: month chunks of the time-chunked scan (0 = Engine.default_chunks)")
    ap.add_argument("--c2-unfused", action="store_true",
                    help="C2 A/B: k_month_end + the three-launch chunked scan (summary, fold, scan) "
                         "instead of the one-launch month-end + chunked scan (csm_signal_chunked)")
    ap.add_argument("--no-oracle-mom", action="store_true",
                    help="N = 1 decile check: qcut the engine's mom_J instead of the oracle's own "
                         "month-end + scan of the panel (that pass adds ~10-20 s at C4)")
    ap.add_argument("--match-dates", type=int, default=0,
                    help="decile-match check on this many evenly spaced dates (0 = every date)")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="replay the step as one captured hipGraph (auto: the unfused narrow "
                         "panels, C2, where launch gaps are a large share of the step; C3 on one "
                         "GPU with 'on')")
    ap.add_argument("--tune", action="append", default=[],
                    help="csm_tune key=value applied before the run (kernel A/B), repeatable")
    ap.add_argument("--full-deciles", action="store_true",
                    help="sweeps: overlapped returns of every decile (default: the two legs, "
                         "all the summary table needs)")
    ap.add_argument("--no-decile-ids", action="store_true",
                    help="sweeps: rank from mom_J (streaming decile kernel) instead of the bucket "
                         "ids the multi-J scan writes (csm_momentum_multi_ids -> csm_deciles_ids)")
    ap.add_argument("--per-j-scan", action="store_true",
                    help="C5: one scan per J instead of every J of a wide batch from one scan "
                         "(csm_momentum_multi, the default)")
    ap.add_argument("--no-boot-scan", action="store_true",
                    help="C5: csm_bootstrap -> multi-J scan on materialised panels instead of "
                         "csm_boot_scan (the panel generated in registers, one shared next_ret)")
    ap.add_argument("--no-grouped", action="store_true",
                    help="C3 A/B: the joined look-backs' panels as side-by-side copies instead of "
                         "the group-major portfolio calls (same bits)")
    ap.add_argument("--no-legs-labels", action="store_true",
                    help="C3/C5 A/B: exact interior deciles in the decile pass instead of the legs "
                         "mode before legs-only accounting (same table bit for bit)")
    ap.add_argument("--no-share-nr", action="store_true",
                    help="C5: each J's cohort pass reads the shared next_ret itself instead of one "
                         "pass staging each month's row for every J (csm_cohort_sums_js)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="N>1 process group: nccl (= RCCL over xGMI, one GPU per rank) or gloo "
                         "(device tensors staged through host memory; the 1-GPU rehearsal of the "
                         "multi-rank path, tests/test_gpu_bench_ranks.py)")
    ap.add_argument("--collective", default="torch", choices=["torch", "csm"],
                    help="N>1 date shards: the all-gathers through torch.distributed, or through "
                         "libcsmom.so's own RCCL communicator (csm_allgather, the C-ABI path)")
    ap.add_argument("--dump", default=None,
                    help="rank 0 saves the pass's results (.npz: LS / EW / CNT, or the sweep's "
                         "summary table) for comparison with a 1-GPU run")
    return ap.parse_args(argv)


def apply_tunes(eng, tunes):
    for kv in tunes:
        k, v = kv.split("=")
        if eng.lib.csm_tune(k.encode(), int(v)) != 0:
            raise SystemExit(f"csm_tune({k}, {v}) rejected")


def cpu_baseline(n_assets: int, days: int, start: str):
    """The CPU oracle (NumPy port of the reference path) on a bounded sample of the same
    workload shape: n_assets x days, one pass, 1 host thread."""
    from oracle import csmom_oracle as O
    from oracle.synth_np import make_panel

    pan = make_panel(n_assets, days, seed=4, start=start, with_volume=False)
    t0 = time.perf_counter()
    PM, _ = O.month_end(pan["P"], pan["month_start"])
    _, M, NR, _ = O.momentum_scan(PM, 12, 1)
    L = O.assign_deciles(M, 10)
    O.portfolio_ew(L, NR, 10)
    dt = time.perf_counter() - t0
    return dict(value=n_assets * days / dt, unit="asset-days/s", cores=1, kind="port",
                sample=f"oracle (NumPy restatement) month-end+scan+deciles+EW on "
                       f"{n_assets} assets x {days} bdays, one pass {dt:.1f} s")


def cpu_baseline_sweep(config: str, n_assets: int, days: int, start: str):
    """The CPU oracles (NumPy ports: month-end, scan, qcut, portfolio rules E1-E6) on a bounded
    sample of the sweep workload, one host thread, in the same unit as the GPU line."""
    from oracle import csmom_oracle as O
    from oracle import portfolio_oracle as PO
    from oracle.synth_np import make_panel

    pan = make_panel(n_assets, days, seed=3, start=start, with_volume=False)
    Js = Ks = (3, 6, 9, 12)
    t0 = time.perf_counter()
    PM, _ = O.month_end(pan["P"], pan["month_start"])
    T_m = PM.shape[0]
    if config == "c3":
        with np.errstate(invalid="ignore"):
            W = np.abs(PM) * 1e6
        for J in Js:
            _, M, NR, _ = O.momentum_scan(PM, J, 1)
            L = O.assign_deciles(M, 10)
            for K in Ks:
                PO.portfolio(L, NR, 10, K=K, W=W)
        dt = time.perf_counter() - t0
        return dict(value=n_assets * days * len(Js) * len(Ks) / dt, unit="asset-day-strategies/s",
                    cores=1, kind="port",
                    sample=f"oracle month-end + 4 scans + 4 qcut + 16 VW portfolios (E1-E5) on "
                           f"{n_assets} assets x {days} bdays, {dt:.1f} s")
    R, _, _, _ = O.momentum_scan(PM, 12, 1)
    t0 = time.perf_counter()
    B = 2
    pmb = PO.bootstrap_panel(R, PO.bootstrap_indices(T_m, B, 5000, 6.0)).reshape(T_m, B * n_assets)
    for J in Js:
        _, M, NR, _ = O.momentum_scan(pmb, J, 1)
        L = O.assign_deciles(M.reshape(T_m * B, n_assets), 10).reshape(T_m, B, n_assets)
        for K in Ks:
            PO.portfolio(L, NR.reshape(T_m, B, n_assets), 10, K=K)
    dt = time.perf_counter() - t0
    return dict(value=n_assets * T_m * B * len(Js) * len(Ks) / dt,
                unit="asset-month-strategies/s", cores=1, kind="port",
                sample=f"oracle bootstrap + 4 scans + 4 qcut + 16 portfolios with turnover/costs "
                       f"on {B} panels x {n_assets} assets x {T_m} months, {dt:.1f} s")


def spawn_workers(argv):
    """`bench.py --gpus N` outside torchrun: start N worker processes of this script with
    torchrun's environment (RANK = LOCAL_RANK = the GPU index, WORLD_SIZE = N, MASTER_* on
    127.0.0.1) and wait for them.  This process never touches the GPU (nothing here imports
    torch), so no process that initialised the GPU is replaced; the workers inherit stdout and
    rank 0 prints the JSON line.  If a worker fails the others are stopped and the first
    failing status is returned."""
    import signal
    import socket
    import subprocess

    args = parse(argv)
    n = args.gpus
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n))
    procs = [subprocess.Popen([sys.executable, "-u", str(Path(__file__).resolve()), *argv],
                              env=dict(base, RANK=str(r), LOCAL_RANK=str(r)))
             for r in range(n)]
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(0.2)
    finally:
        live = [p for p in procs if p.poll() is None]
        for p in live:
            p.send_signal(signal.SIGTERM)
        for p in live:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc


def dist_setup(args):
    """(world, rank, device) from the torchrun environment (set by spawn_workers or torchrun);
    the process group for N > 1 on args.backend (nccl = RCCL, one GPU per rank; gloo =
    host-staged, the 1-GPU rehearsal, where ranks beyond the visible GPUs share them)."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    ndev = torch.cuda.device_count()
    if local >= ndev:
        if args.backend != "gloo":
            raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but {ndev} visible GPUs (RCCL needs "
                             f"one GPU per rank; --backend gloo shares them)")
        local %= ndev
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 and not dist.is_initialized():
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    return world, rank, dev


def allreduce_host(vals, op, dev):
    """Reduce a few host floats over all ranks (max / sum); device tensors for RCCL, host
    tensors for gloo."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return list(vals)
    on = dev if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor(list(vals), dtype=torch.float64, device=on)
    dist.all_reduce(t, op=op)
    return [float(x) for x in t.cpu().tolist()]


def dist_close():
    import torch.distributed as dist
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def lib_sha256():
    import hashlib
    import csmom
    return hashlib.sha256(Path(csmom.lib_path()).read_bytes()).hexdigest()


def committed_profile(config, N, T_d, lib_hash):
    """The committed rocprofv3 evidence for this workload (profiles/<round>/<config>_profile.json,
    scripts/profile.sh): per-kernel average durations from --kernel-trace --stats of the bench
    command and HBM bytes per launch from separate FETCH_SIZE / WRITE_SIZE passes.  Used only
    when it was taken on THIS build of libcsmom.so (sha256) at this workload, else None."""
    for f in sorted((ROOT / "profiles").glob(f"r*/{config}_profile.json"), reverse=True):
        try:
            pj = json.loads(f.read_text())
        except Exception:
            continue
        if pj.get("N") == N and pj.get("T_d") == T_d and pj.get("lib_sha256") == lib_hash:
            pj["path"] = str(f.relative_to(ROOT))
            return pj
    return None


def main(argv=None):
    args = parse(argv)
    if args.gpus > 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        rc = spawn_workers(list(sys.argv[1:] if argv is None else argv))
        if rc:
            raise SystemExit(rc)
        return None
    if args.config in SWEEP_CONFIGS:
        return sweep_main(args)
    import torch
    import torch.distributed as dist

    import csmom
    from csmom.distributed import CsmCollective, DateShardPipeline, halo_months
    from csmom.synth import make_device_panel, make_halo_panel, shard_calendar

    world, rank, dev = dist_setup(args)
    local = dev.index

    cfg = dict(CONFIGS[args.config])
    N = args.assets or cfg["N"]
    days_per_rank = args.days or cfg["days"]
    total_days = days_per_rank * world if args.scaling == "weak" else days_per_rank
    days, ms_host, mend, months = shard_calendar(cfg["start"], total_days, world, rank)
    halo = world > 1 and args.shard_mode == "halo"
    if halo:   # this rank's shard with H lookback months and the next month (neighbours' rows)
        hp = make_halo_panel(N, cfg["start"], total_days, world, rank, halo_months(12, 1),
                             seed_of=lambda r: args.seed * 1000 + r, base_seed=args.seed,
                             device=dev)
        panel = SimpleNamespace(P=hp.P, month_start=hp.month_start)
    else:
        panel = make_device_panel(N, days, ms_host, seed=args.seed * 1000 + rank, device=dev,
                                  shard=(rank, world, args.seed, total_days / world))
    T_d, T_m = len(days), len(ms_host) - 1

    eng = csmom.Engine(local)
    apply_tunes(eng, args.tune)
    J, skip, nb = 12, 1, 10
    # preallocated outputs: the timed loop performs no allocation
    max_days = int(np.diff(ms_host).max())
    min_days = int(np.diff(ms_host)[1:-1].min()) if len(ms_host) > 3 else 1 << 30   # interior months
    fused = eng.use_fused(panel.P, None, max_days) or halo
    coll = CsmCollective(eng) if world > 1 and args.collective == "csm" else None
    pipe = (DateShardPipeline(eng, months, J, skip, nb,
                              fused=fused and args.shard_mode == "fused", collective=coll)
            if world > 1 else None)
    PM = None if fused else eng.empty((T_m, N))
    M, NR = eng.empty((T_m, N)), eng.empty((T_m, N))
    L = eng.empty((T_m, N), torch.int8)
    EW, CNT = eng.empty((T_m, nb)), eng.empty((T_m, nb), torch.int32)
    LS = eng.empty((T_m,))
    # fused + wide rows: the signal kernel writes each mom_J's fixed-map bucket id and the
    # decile pass histograms the 2-B ids instead of streaming mom_J three times
    use_ids = fused and pipe is None and not args.no_ids and N % 4 == 0 and N > 16384
    chunks = 1 if fused else (args.chunks or eng.default_chunks(T_m, N, J, skip))
    # narrow panels (C2): the time-chunked scan writes the bucket ids too and the narrow decile
    # pass ranks from them (csm_momentum_chunked_ids -> csm_deciles_ids)
    narrow_ids = (not fused and pipe is None and not args.no_ids and chunks > 1 and N % 4 == 0
                  and N <= 16384)
    IDS = eng.empty((T_m, N), torch.int16) if (use_ids or narrow_ids) else None
    # C2: month-end and the chunked scan in one launch (k_signal_tc; its workspace is zeroed
    # once here and leaves its sync words zero after every launch)
    tc = narrow_ids and not args.c2_unfused and max_days <= 23 and N % 2 == 0
    tc_ws = None
    if tc:
        chunks = args.chunks or eng.signal_default_chunks(T_m, N, J, skip, eng.cus)
        nbytes = int(eng.lib.csm_signal_chunked_workspace(T_m, N, J, skip, min(chunks, 64)))
        tc_ws = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
    ws = None
    if chunks > 1:
        nbytes = int(eng.lib.csm_momentum_chunked_workspace(T_m, N, J, skip, chunks))
        ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    scan_name = (f"scan(k_momentum_chunked x{chunks}{' +ids' if narrow_ids else ''})" if chunks > 1
                 else "scan(k_momentum)")
    # on ids the long-short is formed by the decile pass's last workgroup (csm_deciles_ids_ls)
    fused_ls = (use_ids or narrow_ids) and not args.no_fused_ls
    stage_names = (["signal(k_signal+ids)", "deciles+long_short(k_deciles<ids>)"] if use_ids and fused_ls else
                   ["signal(k_signal+ids)", "deciles(k_deciles<ids>)", "long_short"] if use_ids else
                   ["signal(k_signal)", "deciles(k_deciles)", "long_short"] if fused else
                   ["signal(k_signal_tc+ids)", "deciles+long_short(k_deciles<ids>)"]
                   if tc and fused_ls else
                   ["signal(k_signal_tc+ids)", "deciles(k_deciles<ids>)", "long_short"] if tc else
                   ["month_end(k_month_end)", scan_name,
                    "deciles+long_short(k_deciles<ids>)"] if narrow_ids and fused_ls else
                   ["month_end(k_month_end)", scan_name, "deciles(k_deciles<ids>)", "long_short"]
                   if narrow_ids else
                   ["month_end(k_month_end)", scan_name, "deciles(k_deciles)", "long_short"])
    nst = len(stage_names) + 1
    step_events = [[torch.cuda.Event(enable_timing=True) for _ in range(nst)]
                   for _ in range(args.steps)]
    scratch_events = [torch.cuda.Event(enable_timing=True) for _ in range(nst)]

    def step(ev=scratch_events):
        if pipe is not None:
            if halo:   # (the fallback list's fit is checked once, after the timed loop)
                return pipe.run_halo(hp.P, hp.month_start, hp.H, hp.F, max_days, check=False).LS
            r = pipe.run(panel.P, panel.month_start, max_days)
            return r.LS
        rec = (lambda e: e.record()) if ev is not None else (lambda e: None)
        ev = ev if ev is not None else [None] * nst
        i = 0
        rec(ev[i])
        if use_ids:
            eng.signal_ids(panel.P, panel.month_start, max_days, J, skip,
                           out=(None, None, M, NR, IDS), min_month_days=min_days)
        elif fused:
            eng.signal(panel.P, panel.month_start, max_days, J, skip, out=(None, None, M, NR))
        elif tc:
            eng.signal_chunked(panel.P, panel.month_start, max_days, J, skip, chunks=chunks,
                               out=(None, M, NR, IDS), workspace=tc_ws, check=False)
        else:
            eng.month_end(panel.P, panel.month_start, PM=PM)
            i += 1
            rec(ev[i])
            if chunks > 1:
                eng.momentum_chunked(PM, J, skip, chunks=chunks, out=(None, M, NR), workspace=ws,
                                     ids=IDS if narrow_ids else None)
            else:
                eng.momentum(PM, J, skip, out=(None, M, NR))
        i += 1
        rec(ev[i])
        if fused_ls:
            eng.deciles_ids(M, NR, IDS, nb, out=(L, EW, CNT, None), LS=LS)
        elif use_ids or narrow_ids:
            eng.deciles_ids(M, NR, IDS, nb, out=(L, EW, CNT, None))
            i += 1
            rec(ev[i])
            eng.long_short(EW, CNT, LS)
        else:
            eng.deciles(M, NR, nb, out=(L, EW, CNT, None))
            i += 1
            rec(ev[i])
            eng.long_short(EW, CNT, LS)
        rec(ev[i + 1])
        return LS

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    use_graph = (world == 1 and pipe is None and
                 (args.graph == "on" or (args.graph == "auto" and not fused)))
    graph = None
    if use_graph:   # the whole pass as one hipGraph (no host launches inside the timed loop)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step(None)
        graph.replay()
        torch.cuda.synchronize()

    stage_ms = np.zeros(len(stage_names))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        if graph is not None:
            graph.replay()
        else:
            step(step_events[k])   # HIP events on the launch stream; read after the loop
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if graph is not None:   # per-stage device times from an untimed eager pass
        for k in range(args.steps):
            step(step_events[k])
        torch.cuda.synchronize()
    elapsed = allreduce_host([elapsed], dist.ReduceOp.MAX if world > 1 else None, dev)[0]
    if tc_ws is not None and hasattr(eng.lib, "csm_signal_chunked_status"):   # (A/B base builds)
        # k_signal_tc's in-launch hand-off: a workgroup that gave up a wait marks the workspace;
        # any mark left by the timed (or staging) launches invalidates the line
        try:
            eng.signal_chunked_status(tc_ws)
        except Exception as e:
            raise SystemExit(f"C2 signal: {e}; the timed passes are invalid, no line printed")

    if world == 1:
        for ev in step_events:
            stage_ms += [ev[i].elapsed_time(ev[i + 1]) for i in range(len(stage_names))]
    else:
        stage_ms[:] = np.nan

    # decile match vs the oracle (metric: "decile match %"): the oracle's qcut on the engine's
    # mom_J for every date (or --match-dates evenly spaced ones), labels compared cell by cell.
    # N > 1: EVERY rank runs the (collective-bearing) pass and checks its own months; the
    # counts are summed over the ranks.
    from oracle import csmom_oracle as O
    halo_info = None
    if world > 1:
        if halo:   # the timed passes' list fit (every rank sees the same list); then a checked pass
            cnt, cap = pipe.last_count
            listed = int(cnt.max().item())
            if listed > cap:
                raise SystemExit(f"halo pass: {listed} listed assets exceed the list width {cap}; "
                                 "the timed passes are invalid (rerun with --shard-mode fused)")
            halo_info = dict(H=hp.H, F=hp.F, listed_assets=listed, list_width=cap,
                             rows_read_with_halo=int(hp.P.shape[0]), shard_days=hp.shard_days)
            res = pipe.run_halo(hp.P, hp.month_start, hp.H, hp.F, max_days)
        else:
            res = pipe.run(panel.P, panel.month_start, max_days)
        Mh, Lh, LSh, EWh, CNTh = res.M, res.L, res.LS, res.EW, res.CNT
    else:
        Mh, Lh, LSh, EWh, CNTh = M, L, LS, EW, CNT
    if args.match_dates > 0:
        dates = sorted({int(x) for x in np.linspace(0, T_m - 1, args.match_dates)})
    else:
        dates = list(range(T_m))
    # N = 1: the reference labels come from the ORACLE's mom_J -- the oracle's month-end and scan
    # over this very panel, in column blocks (per-asset arithmetic: a block is exact) -- and the
    # engine's mom_J is checked against it bit for bit on every cell
    Mo, mom_exact = None, None
    if world == 1 and not args.no_oracle_mom:
        Mo = np.empty((T_m, N))
        same = 0
        for c0 in range(0, N, 20_000):
            c1 = min(N, c0 + 20_000)
            PMb, _ = O.month_end(panel.P[:, c0:c1].cpu().numpy(), ms_host)
            _, Mb, _, _ = O.momentum_scan(PMb, J, skip)
            Mo[:, c0:c1] = Mb
            same += int((Mb.view(np.uint64) == Mh[:, c0:c1].cpu().numpy().view(np.uint64)).sum())
        mom_exact = 100.0 * same / (T_m * N)
    tot = ok = 0
    for t0 in range(0, len(dates), 64):
        blk = dates[t0:t0 + 64]
        mrows = Mo[blk] if Mo is not None else Mh[blk].cpu().numpy()
        lrows = Lh[blk].cpu().numpy()
        for row, got in zip(mrows, lrows):
            ref = np.full(N, -1, dtype=np.int8)
            v = ~np.isnan(row)
            if v.any():
                lab = O.qcut_labels(row[v], nb)
                ref[v] = np.where(np.isnan(lab), -1, lab).astype(np.int8)
            ok += int((got == ref).sum())
            tot += N
    ok, tot, ndates = allreduce_host([ok, tot, len(dates)],
                                     dist.ReduceOp.SUM if world > 1 else None, dev)
    tm_all = sum(pipe.months) if pipe is not None else T_m
    match = dict(pct=100.0 * ok / tot,
                 sample=f"{int(ndates)} of {tm_all} dates x {N} assets"
                        f"{f' (all {world} ranks)' if world > 1 else ''}: oracle qcut of the "
                        + ("ORACLE's mom_J (oracle month-end + scan on this panel; engine mom_J "
                           f"bit-exact on {mom_exact:.4f} % of cells)" if Mo is not None
                           else "engine's mom_J"))
    if rank == 0 and args.dump:
        np.savez(args.dump, LS=LSh.cpu().numpy(), EW=EWh.cpu().numpy(), CNT=CNTh.cpu().numpy())

    ms_per_step = 1000.0 * elapsed / args.steps
    units = N * total_days            # the whole panel (all ranks' date shards)
    value = units * args.steps / elapsed
    out = None
    if rank == 0:
        alg_pipe = 8.0 * N * T_d + 17.0 * N * T_m + 8.0 * T_m * (nb + 1)   # SURVEY 8(d), per rank
        roofline = None
        if world == 1:
            me_ms = stage_ms[0] / args.steps
            if fused or tc:
                kname = "k_signal_tc" if tc else "k_signal"
                alg_me = 8.0 * N * T_d + 16.0 * N * T_m       # read P once, write mom + next_ret
            else:
                kname = "k_month_end"
                alg_me = 8.0 * N * T_d + 8.0 * N * T_m          # read P once, write PM once
            achieved = alg_me / (me_ms * 1e-3) / 1e9
            # the committed rocprofv3 run of this exact bench command on this build (else null)
            prof = committed_profile(args.config, N, T_d, lib_sha256())
            # the profile keys kernels per template instantiation ("k_signal<23, 2, ...>"): the
            # dominant kernel is the instantiation of kname with the most device time
            kern = (prof or {}).get("kernels", {})
            pk = max((v for k, v in kern.items() if k == kname or k.startswith(kname + "<")),
                     key=lambda v: v.get("total_ns", 0.0), default={})
            traffic = pk.get("hbm_bytes_per_launch")
            roofline = dict(bound="hbm", kernel=kname, achieved=round(achieved, 1),
                            peak=HBM_PEAK_GBS, unit="GB/s", frac=round(achieved / HBM_PEAK_GBS, 4),
                            traffic=traffic, algorithmic_bytes_per_launch=alg_me,
                            avg_launch_ms=round(me_ms, 4))
            if pk.get("avg_ns"):
                # the same roofline from the committed profile's kernel average: a reader
                # recomputes it from profiles/ (alg bytes / avg_ns / peak)
                roofline["profile_frac"] = round(alg_me / (pk["avg_ns"] * 1e-9) / 1e9 / HBM_PEAK_GBS, 4)
                roofline["profile_avg_launch_ms"] = round(pk["avg_ns"] * 1e-6, 4)
                roofline["profile"] = dict(path=prof["path"], commit=prof.get("git_head"),
                                           box_note="rocprofv3 run on another box than this line")
        pipe_gbs = alg_pipe * world / (ms_per_step * 1e-3) / 1e9
        out = {
            "metric": "asset-periods backtested/sec (1/2/4/8 GPU) + % HBM peak BW; decile match %",
            "value": value,
            "unit": "asset-days/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic seeded GBM panel generated in HBM (late listings, delistings, "
                    "NaN days, absent and all-NaN months); N>1: rank r holds date shard r of "
                    "one global panel (prices continue across shards)",
            "hipgraph": graph is not None,
            "halo": halo_info,
            "engine_path": (("halo date shards: k_shard_halo state -> k_signal<SH> (+ ids) -> "
                             "need bits all-gather -> listed assets' records all-gather, fold, "
                             "column repair -> decile pass on ids" if halo else
                             "speculative fused k_signal + k_shard_repair" if pipe.fused else
                             "k_month_end + carried k_momentum") if pipe is not None else
                            "fused k_signal (+ bucket ids) -> k_deciles on ids (+ long-short, one "
                            "launch tail)" if use_ids else
                            "fused k_signal" if fused else
                            f"k_signal_tc (month-end + {min(chunks, 64)}-chunk scan + bucket ids, one "
                            f"launch) -> narrow k_deciles on ids (+ long-short in the same launch)"
                            if tc else
                            f"k_month_end + scan ({chunks} month chunks, + bucket ids) -> narrow "
                            f"k_deciles on ids (+ long-short in the same launch)" if narrow_ids else
                            f"k_month_end + scan ({chunks} month chunks)"),
            "config": {"workload": (cfg["name"] if args.assets is None and args.days is None
                                    else f"custom: {N} assets x {total_days} bdays") +
                                   (f", date-sharded across {world} GPUs" if world > 1 else "") +
                                   (" (weak scaling: 10k bdays per GPU)"
                                    if world > 1 and args.scaling == "weak" else ""),
                       "assets": N, "bdays": total_days, "bdays_rank0": T_d, "months_rank0": T_m,
                       "J": J,
                       "skip": skip, "K": 1, "n_bins": nb, "weighting": "equal",
                       "parallelism": f"date-shard x{world}"},
            "roofline": roofline,
            "pipeline_roofline": {"bound": "hbm", "achieved": round(pipe_gbs, 1),
                                  "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
                                  "frac": round(pipe_gbs / (HBM_PEAK_GBS * world), 4),
                                  "algorithmic_bytes_per_pass_per_gpu": alg_pipe},
            "stage_ms": ({k: round(v / args.steps, 4) for k, v in zip(stage_names, stage_ms)}
                         if world == 1 else None),
            "decile_match_pct": match["pct"] if match else None,
            "mom_bit_exact_pct": mom_exact,
            "decile_check": match["sample"] if match else None,
            "cpu_baseline": None,
            # context only (not measured by this run): the reference's own pandas path
            "reference_pandas": REFERENCE_PANDAS,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_assets, T_d, cfg["start"])
        print(json.dumps(out), flush=True)
    dist_close()
    return out


class TimedStages:
    """Engine proxy recording HIP events around every stage call on torch's current stream
    (the stream the engine launches on); per-stage device time is read after the timed loop."""

    def __init__(self, eng):
        self.eng = eng
        self.rec = []          # (stage, start_event, end_event, algorithmic bytes)
        self.on = False

    def _wrap(self, name, nbytes, fn, *a, **k):
        import torch
        if not self.on:
            return fn(*a, **k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = fn(*a, **k)
        e1.record()
        self.rec.append((name, e0, e1, nbytes))
        return out

    def month_end(self, P, ms, **k):
        T_d, N = P.shape
        T_m = ms.numel() - 1
        return self._wrap("month_end(k_month_end)", 8.0 * N * T_d + 8.0 * N * T_m,
                          self.eng.month_end, P, ms, **k)

    def momentum(self, PM, J=12, skip=1, **k):
        T_m, N = PM.shape
        return self._wrap("scan(k_momentum*)", 24.0 * N * T_m, self.eng.momentum, PM, J, skip, **k)

    def momentum_multi(self, PM, Js, skip=1, with_ids=False, chunks=1, stacked=False):
        T_m, N = PM.shape
        return self._wrap("scan(k_momentum*)", (8.0 + 16.0 * len(Js)) * N * T_m,
                          self.eng.momentum_multi, PM, Js, skip, with_ids=with_ids, chunks=chunks,
                          stacked=stacked)

    def default_chunks(self, *a, **k):
        return self.eng.default_chunks(*a, **k)

    def deciles(self, M, NR=None, n_bins=10, **k):
        R_, N = M.shape
        return self._wrap("deciles(k_deciles)", 9.0 * N * R_, self.eng.deciles, M, NR, n_bins, **k)

    def deciles_ids(self, M, NR, IDS, n_bins=10, **k):
        R_, N = M.shape   # algorithmic: the labels of every cell (mom_J read, label written)
        return self._wrap("deciles(k_deciles)", 9.0 * N * R_, self.eng.deciles_ids, M, NR, IDS,
                          n_bins, **k)

    def portfolio(self, L, NR, n_bins=10, **k):
        T_m, BN = L.shape
        per = 9.0 + (8.0 if k.get("W") is not None else 0.0) + \
            (8.0 if k.get("ADV") is not None else 0.0) + (8.0 if k.get("SIG") is not None else 0.0)
        return self._wrap("portfolio(k_cohort+k_turnover+k_overlap_ls)", per * T_m * BN,
                          self.eng.portfolio, L, NR, n_bins, **k)

    def portfolio_multi(self, L, NR, n_bins=10, **k):
        T_m, BN = L.shape
        per = 9.0 + (8.0 if k.get("W") is not None else 0.0) + \
            (8.0 if k.get("ADV") is not None else 0.0) + (8.0 if k.get("SIG") is not None else 0.0)
        return self._wrap("portfolio(k_cohort+k_turnover+k_overlap+k_ls)", per * T_m * BN,
                          self.eng.portfolio_multi, L, NR, n_bins, **k)

    def portfolio_multi_grouped(self, Lg, NRg, n_bins=10, **k):
        G, T_m, BgN = Lg.shape   # algorithmic: each group's labels + next_ret, the shared
        per_w = sum(8.0 for x in ("W", "ADV", "SIG") if k.get(x) is not None)   # weights once
        return self._wrap("portfolio(k_cohort+k_turnover+k_overlap+k_ls)",
                          (9.0 * G + per_w) * T_m * BgN, self.eng.portfolio_multi_grouped, Lg,
                          NRg, n_bins, **k)

    def portfolio_multi_js(self, Ls, NR, n_bins=10, **k):
        T_m, BN = NR.shape   # algorithmic: each J's labels, the shared next_ret once
        return self._wrap("portfolio(k_cohort+k_turnover+k_overlap+k_ls)",
                          (1.0 * len(Ls) + 8.0) * T_m * BN, self.eng.portfolio_multi_js, Ls, NR,
                          n_bins, **k)

    def portfolio_multi_js_grouped(self, Lg, NR, n_bins=10, **k):
        T_m, BN = NR.shape   # algorithmic: each J's labels, the shared next_ret once
        return self._wrap("portfolio(k_cohort+k_turnover+k_overlap+k_ls)",
                          (1.0 * Lg.shape[0] + 8.0) * T_m * BN, self.eng.portfolio_multi_js_grouped,
                          Lg, NR, n_bins, **k)

    def portfolio_plan(self, *a, **k):
        return self.eng.portfolio_plan(*a, **k)

    def summary(self, LS, TURN=None, COST=None, NET=None, **k):
        return self._wrap("summary(k_summary)", 8.0 * LS.numel() * (4 if TURN is not None else 1),
                          self.eng.summary, LS, TURN, COST, NET, **k)

    def bootstrap(self, R, B, **k):
        T_m, N = R.shape
        return self._wrap("bootstrap(k_bootstrap_*)", 16.0 * T_m * B * N, self.eng.bootstrap,
                          R, B, **k)

    def boot_scan(self, R, B, Js, skip=1, **k):
        T_m, N = R.shape   # algorithmic: R once, mom_J (+ ids) per J and one next_ret written
        per = (8.0 + (2.0 if k.get("with_ids", True) else 0.0)) * len(Js) + 8.0
        return self._wrap("bootscan(k_bootstrap_index+k_boot_scan)", 8.0 * T_m * N + per * T_m * B * N,
                          self.eng.boot_scan, R, B, Js, skip, **k)

    @property
    def device(self):
        return self.eng.device

    @property
    def lib(self):
        return self.eng.lib

    def stage_report(self, steps):
        agg = {}
        for name, e0, e1, nb in self.rec:
            ms, tot = agg.get(name, (0.0, 0.0))
            agg[name] = (ms + e0.elapsed_time(e1), tot + nb)
        return {k: (v[0] / steps, v[1] / steps) for k, v in agg.items()}


def sweep_traffic(config, N, T_d, stage):
    """HBM bytes per step of the dominant sweep stage from the committed PMC passes
    (profiles/<round>/<config>_profile.json, scripts/profile.sh), only when they were taken on
    THIS build of libcsmom.so at this workload and name this stage; else None."""
    pj = committed_profile(config, N, T_d, lib_sha256())
    st = (pj or {}).get("stage", {})
    if st.get("label") == stage:
        return st.get("hbm_bytes_per_step")
    return None


def sweep_profile(config, N, T_d, stage, alg_bytes):
    """profile_frac of the dominant stage from the committed rocprofv3 kernel averages (the
    stage's kernels' device time per step), with the profile's path and commit."""
    pj = committed_profile(config, N, T_d, lib_sha256())
    st = (pj or {}).get("stage", {})
    if st.get("label") != stage or not st.get("ns_per_step"):
        return {}
    ms = st["ns_per_step"] * 1e-6
    return {"profile_frac": round(alg_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "profile_avg_ms_per_step": round(ms, 4),
            "profile": {"path": pj["path"], "commit": pj.get("git_head"),
                        "box_note": "rocprofv3 run on another box than this line"}}


def sweep_decile_match(config, eng, PM=None, R0=None, J=12, n_bins=10):
    """Decile match % of a sweep line: one sampled panel (C3: the panel; C5:
    bootstrap panel 0) and one look-back J, ranked by the bench's kernels -- the chunked multi-J
    scan (C3) or csm_boot_scan (C5), then the decile pass on ids -- against the oracle's qcut of
    the ORACLE's mom_J (oracle month-end + scan; C5: the oracle's bootstrap of the same base
    returns).  Full labels (every decile) and the legs-mode labels the sweep's accounting reads
    (deciles 0 / n_bins - 1 / NaN exact, the interior ones anywhere inside)."""
    import torch
    from oracle import csmom_oracle as O
    from oracle import portfolio_oracle as PO
    if config == "c3":
        T_m, N = PM.shape
        M, _, IDS = eng.momentum_multi(PM, (J,), 1, with_ids=True,
                                       chunks=eng.default_chunks(T_m, N, J, 1))[0]
        _, Mo, _, _ = O.momentum_scan(PM.cpu().numpy(), J, 1)
        what = f"the C3 panel, J = {J}"
    else:
        T_m, N = R0.shape
        _, outs, _, _ = eng.boot_scan(R0, 1, (3, 6, 9, 12), 1, b0=0, seed=5000, mean_block=6.0)
        M, IDS = outs[(3, 6, 9, 12).index(J)]
        src = PO.bootstrap_indices(T_m, 1, 5000, 6.0, b0=0)
        pm = PO.bootstrap_panel(R0.cpu().numpy(), src).reshape(T_m, N)
        _, Mo, _, _ = O.momentum_scan(pm, J, 1)
        what = f"bootstrap panel 0 of the C5 draw, J = {J}"
    L, _, _, _ = eng.deciles_ids(M, None, IDS, n_bins)
    Lg, _, _, _ = eng.deciles_ids(M, None, IDS, n_bins, legs=True)
    torch.cuda.synchronize()
    Lo = O.assign_deciles(Mo, n_bins)
    Lh, Lgh = L.cpu().numpy(), Lg.cpu().numpy()
    mom_exact = float((M.cpu().numpy().view(np.uint64) == Mo.view(np.uint64)).mean()) * 100.0
    edge = (Lo == 0) | (Lo == n_bins - 1) | (Lo < 0)
    legs_ok = np.where(edge, Lgh == Lo, (Lgh >= 1) & (Lgh <= n_bins - 2))
    return {"decile_match_pct": round(100.0 * float((Lh == Lo).mean()), 6),
            "legs_match_pct": round(100.0 * float(legs_ok.mean()), 6),
            "mom_bit_exact_pct": round(mom_exact, 6),
            "sample": f"{what}: {T_m} dates x {N} assets, the oracle's qcut of the oracle's mom_J "
                      f"(full labels; legs: the legs-mode labels the accounting reads)"}


def sweep_main(args):
    """C3 / C5: the (J, K) sweep (SweepRunner) on one panel (C3: at N > 1 the 16 strategies are
    split across the ranks, SweepRunner.run_batch_sharded, strong scaling of the fixed grid) or
    on bootstrap panels (C5, strong scaling: the panels are split across ranks)."""
    import torch
    import torch.distributed as dist

    import csmom
    from csmom.synth import bday_calendar, make_device_panel

    world, rank, dev = dist_setup(args)
    local = dev.index
    cfg = dict(SWEEP_CONFIGS[args.config])
    N = args.assets or cfg["N"]
    T_d = args.days or cfg["days"]
    days, ms_host, _ = bday_calendar(cfg["start"], T_d)
    T_m = len(ms_host) - 1
    eng = csmom.Engine(local)
    apply_tunes(eng, args.tune)
    ts = TimedStages(eng)
    scfg = csmom.SweepConfig(Js=(3, 6, 9, 12), Ks=(3, 6, 9, 12), skip=1, aum=1e8,
                             multi_j_scan=not args.per_j_scan, decile_ids=not args.no_decile_ids,
                             legs_only=not args.full_deciles, boot_scan=not args.no_boot_scan,
                             share_nr=not args.no_share_nr, grouped=not args.no_grouped,
                             legs_labels=not args.no_legs_labels,
                             scan_chunks=args.chunks or 0)
    S = len(scfg.strategies)
    runner = csmom.SweepRunner(ts, scfg)
    if args.config == "c3":
        seed = args.seed * 1000 + 3      # the same panel on every rank (strategy shards)
        panel = make_device_panel(N, days, ms_host, seed=seed, device=dev)
        g = torch.Generator(device=dev)
        g.manual_seed(seed)
        shares = torch.exp(torch.randn(N, generator=g, device=dev, dtype=torch.float64) + 16.0)
        turn_rate = torch.rand(N, generator=g, device=dev, dtype=torch.float64) * 0.018 + 0.002
        PM = eng.empty((T_m, N))

        def step():
            ts.month_end(panel.P, panel.month_start, PM=PM)
            W = PM.abs() * shares              # market cap at formation (value weights)
            ADV = W * turn_rate                # dollar ADV for the square-root impact
            summ, _ = run_grid(PM, 1, W=W, ADV=ADV)
            return summ

        flag_acc = torch.zeros(1, dtype=torch.int32, device=dev)
        # N > 1: each rank runs its block of the (J, K) grid, one all-gather of the summary
        run_grid = runner.run_batch_sharded if world > 1 else runner.run_batch

        def step_defer():   # the same step with no device sync (hipGraph capture): the
            ts.month_end(panel.P, panel.month_start, PM=PM)   # legs flag is accumulated and
            W = PM.abs() * shares                             # read after the timed loop
            ADV = W * turn_rate
            summ, _, fl = run_grid(PM, 1, W=W, ADV=ADV, defer=True)
            if fl is not None:
                flag_acc.add_(fl)
            return summ
        units = float(N) * T_d * S
        unit = "asset-day-strategies/s"
        scaling = "strong"
        n_panels = 1
    else:
        n_panels = args.panels or cfg["panels"]
        panel = make_device_panel(N, days, ms_host, seed=args.seed * 1000 + 5, device=dev)
        PM0, _ = eng.month_end(panel.P, panel.month_start)
        R0, _, _ = eng.momentum(PM0, 12, 1, with_ret=True)     # base month returns
        del panel

        def step():
            return runner.run_bootstrap(R0, n_panels, seed=5000, mean_block=6.0, batch=args.batch)
        units = float(N) * T_m * S * n_panels
        unit = "asset-month-strategies/s"
        scaling = "strong"
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # C3 (one panel, ~40 launches a step): the step defers its legs-flag check (no device sync
    # inside the step), so the host queues step k + 1 while step k runs; the accumulated flag is
    # read after the timed loop and, if a panel ever lacked a leg's column, the loop is timed
    # again with the synchronous step (which reruns such a panel with every decile)
    defer = args.config == "c3"

    def timed(fn):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            o = fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return time.perf_counter() - t0, o

    # C3 on one GPU with --graph on: the deferred step captured as one hipGraph and replayed
    # (replay-safe, tests/test_gpu_capture.py).  Not the default: the step is device-bound, the
    # graph measured 0.675 vs 0.672 ms eager (profiles/r04/experiments).  N > 1 keeps the eager
    # step (its all-gather is a host-staged gloo call or an RCCL call outside the graph).
    graph = None
    if defer and world == 1 and args.graph == "on":
        if args.per_j_scan or args.no_decile_ids:   # never captured (sweep._refuse_capture)
            raise SystemExit("--graph on takes the default scan and decile paths only "
                             "(not --per-j-scan / --no-decile-ids; DESIGN.md 4.3)")
        s_cap = torch.cuda.Stream()
        s_cap.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s_cap):      # warm-up on a side stream (torch's capture recipe)
            step_defer()
        torch.cuda.current_stream().wait_stream(s_cap)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            g_out = step_defer()
        graph.replay()
        torch.cuda.synchronize()

        def step_graph():
            graph.replay()
            return g_out
    # the timed loop runs uninstrumented (HIP events per stage call cost host time the
    # launch-bound C3 step would pay); per-stage device times come from a second, untimed pass
    if defer:
        flag_acc.zero_()
    elapsed, out = timed(step_graph if graph is not None else step_defer if defer else step)
    if defer and allreduce_host([float(flag_acc.item())],
                                dist.ReduceOp.SUM if world > 1 else None, dev)[0]:
        defer = False   # (every rank decides alike: the rerun's barriers need them all)
        graph = None
        elapsed, out = timed(step)
    elapsed = allreduce_host([elapsed], dist.ReduceOp.MAX if world > 1 else None, dev)[0]
    ts.on = True
    for _ in range(args.steps):
        (step_defer if defer else step)()
    torch.cuda.synchronize()
    ts.on = False
    stages = ts.stage_report(args.steps)
    line = None
    if rank == 0:
        dom = max(stages.items(), key=lambda kv: kv[1][0])
        dname, (dms, dbytes) = dom
        ach = dbytes / (dms * 1e-3) / 1e9
        alg_step = sum(v[1] for v in stages.values())
        ms_step = 1000.0 * elapsed / args.steps
        res = out.cpu().numpy()
        res_summary = {f: float(np.nanmean(res[..., i])) for i, f in enumerate(csmom.SUMMARY_FIELDS)}
        line = {
            "metric": "asset-periods backtested/sec (1/2/4/8 GPU) + % HBM peak BW; decile match %",
            "value": units * args.steps / elapsed,
            "unit": unit,
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_step, "higher_is_better": True, "scaling": scaling,
            "vs_baseline": None, "dtype": "f64",
            "data": "synthetic seeded GBM panel generated in HBM" +
                    (" + stationary bootstrap of its month returns" if args.config == "c5" else
                     "; lognormal shares (value weights), uniform daily turnover (dollar ADV)"),
            "config": {"workload": cfg["name"], "assets": N, "bdays": T_d, "months": T_m,
                       "strategies": S, "panels": n_panels, "weighting": "value" if args.config == "c3" else "equal",
                       "costs": "spread/2 + 0.1*vol*sqrt(size/ADV), AUM 1e8" if args.config == "c3" else "spread/2",
                       "parallelism": f"{'panel' if args.config == 'c5' else 'strategy'}-shard x{world}"},
            "roofline": {"bound": "hbm", "kernel": dname, "achieved": round(ach, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                         "traffic": sweep_traffic(args.config, N, T_d, dname),
                         **sweep_profile(args.config, N, T_d, dname, dbytes),
                         "algorithmic_bytes_per_step": dbytes,
                         "avg_ms_per_step": round(dms, 4)},
            "pipeline_roofline": {"bound": "hbm", "achieved": round(alg_step / (ms_step * 1e-3) / 1e9, 1),
                                  "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": round(alg_step / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                  "algorithmic_bytes_per_step_rank0": alg_step},
            "stage_ms": {k: round(v[0], 4) for k, v in stages.items()},
            "hipgraph": graph is not None,
            "result_means": res_summary,
            "cpu_baseline": None,
        }
        if not args.no_oracle_mom:
            line["decile_match"] = sweep_decile_match(args.config, eng,
                                                      PM=PM if args.config == "c3" else None,
                                                      R0=R0 if args.config == "c5" else None)
            line["decile_match_pct"] = line["decile_match"]["decile_match_pct"]
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline_sweep(args.config, 1500 if args.config == "c3" else 1000,
                                                      T_d, cfg["start"])
        if args.dump:
            np.savez(args.dump, table=res)
        print(json.dumps(line), flush=True)
    dist_close()
    return line


if __name__ == "__main__":
    main()
