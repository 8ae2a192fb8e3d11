"""One-GPU rehearsal of a halo date-shard rank's pass (DateShardPipeline.run_halo) at C4 width:
rank 1 of a 3-rank whole-month split (a middle rank: halo before, forward month after), each
rank `days_per_rank` business days -- 1,250 days is an 8-way strong-scaling shard of C4.  The
collectives are replaced by stacks of this rank's own tensors (the records: G copies, the bytes a
G-rank all-gather would deliver; the need bits: the three ranks' own, so the union -- and the
listed count -- is the real one), so the numbers are the per-rank device cost without xGMI.

Times, interleaved (median of `reps`): the halo pass, the speculative all-gather pass
(signal_shard from an empty state, full summary, fold, repair) and the 1-GPU pipeline on the
shard alone; per-stage HIP events of the halo pass; |U| (the assets this rank lists).
Prints one JSON line.  Usage: exp_shard_halo.py [N] [days_per_rank] [reps] [G] [split_cells]"""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import csmom  # noqa: E402
from csmom.distributed import _halo_fused, fallback_cap, halo_months  # noqa: E402
from csmom.synth import make_halo_panel  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    dpr = int(sys.argv[2]) if len(sys.argv) > 2 else 1_250
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    G = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    cells = int(sys.argv[5]) if len(sys.argv) > 5 else 0     # split-sweep chunk (0: default)
    dev = torch.device("cuda", 0)
    eng = csmom.Engine(0)
    if cells:
        assert eng.lib.csm_tune(b"dec_split_cells", cells) == 0
    import os
    for kv in filter(None, os.environ.get("CSM_TUNE", "").split(",")):   # A/B: key=value,...
        k, v = kv.split("=")
        assert eng.lib.csm_tune(k.encode(), int(v)) == 0, kv
    split = os.environ.get("CSM_DEC_SPLIT")   # A/B: 0 = one workgroup per date row, 1 / 2 split
    if split is not None:
        assert eng.lib.csm_tune(b"dec_split", int(split)) == 0
    J, skip, nb = 12, 1, 10
    H = halo_months(J, skip)
    def panel(r):
        return make_halo_panel(N, "1980-01-01", 3 * dpr, 3, r, H, seed_of=lambda q: 1000 + q,
                               base_seed=1, device=dev)

    def bits(p, r):   # a rank's need bits (untimed), for the union the timed rank computes
        c, n, f = eng.shard_halo(p.P, p.month_start, p.H, p.F, J, skip, before=r > 0,
                                 after=r < 2)
        msr = p.shard_month_start
        _, _, _, _, s = eng.signal_shard_halo(p.P, msr, int(np.diff(p.month_start_host).max()),
                                              J, skip, c, n)
        return eng.shard_need(f, s, H)   # (the next rank's halo length)

    other = {}
    for r in (0, 2):
        p = panel(r)
        other[r] = bits(p, r)
        del p
    hp = panel(1)
    P, ms, T_m = hp.P, hp.month_start, hp.T_m
    msh = hp.shard_month_start
    mh = hp.month_start_host
    maxd = int(np.diff(mh).max())
    cap = fallback_cap(N)
    IDS = torch.empty((T_m, N), dtype=torch.int16, device=dev)
    # the shard alone, for the speculative pass and the 1-GPU reference point
    d0, d1 = int(mh[hp.H]), int(mh[hp.H + T_m])
    Ps = P[d0:d1].contiguous()
    mss = (msh - d0).contiguous()
    torch.cuda.synchronize()

    # run_halo's choice (distributed._halo_fused); CSM_HALO_FUSED=1 / 0 forces either
    force = os.environ.get("CSM_HALO_FUSED")
    fused = _halo_fused(eng, P, maxd) if force is None else force == "1"

    def halo(ev=None):
        rec = (lambda i: ev[i].record()) if ev else (lambda i: None)
        rec(0)
        if not fused:   # the two launches
            carry_h, npm_h, flags = eng.shard_halo(P, ms, hp.H, hp.F, J, skip, before=True,
                                                   after=True)
            rec(1)
            PM, _, M, NR, st = eng.signal_shard_halo(P, msh, maxd, J, skip, carry_h, npm_h,
                                                     ids=IDS)
        else:   # the halo prologue inside the shard kernel (csm_signal_halo)
            carry_h = None
            rec(1)
            PM, _, M, NR, st, flags = eng.signal_halo(P, ms, hp.H, hp.F, maxd, J, skip,
                                                      ids=IDS)
        rec(2)
        mask = eng.shard_need(flags, st, H)
        masks = torch.stack([other[0], mask, other[2]])   # the 3 ranks' bits (the union's input)
        idx, cnt = eng.shard_union(masks, N, cap)
        rec(3)
        rcd = eng.shard_summary_cols(PM, st, idx, cnt, J, skip)
        recs = torch.stack([rcd] * G)
        rec(4)
        if os.environ.get("CSM_FOLD_REPAIR") and carry_h is not None:   # A/B: round 5's repair
            carry_u, npm_u = eng.fold_carry(recs, 1, J, skip)
            eng.shard_repair_cols(PM, carry_u, npm_u, carry_h, st, idx, cnt, M, NR, J, skip,
                                  ids=IDS)
        else:
            eng.shard_fix_cols(PM, recs, 1, st, idx, cnt, M, NR, J, skip, ids=IDS)
        rec(5)
        L, EW, CNT, _ = eng.deciles_ids(M, NR, IDS, nb)
        rec(6)
        EWg = torch.cat([torch.cat([EW, CNT.to(EW.dtype)], 1)] * G)
        LS = eng.long_short(EW, CNT)
        rec(7)
        return LS, cnt, M, NR, L

    def speculative():
        PM, _, M, NR, st = eng.signal_shard(Ps, mss, maxd, J, skip, ids=IDS)
        S1 = eng.shard_summary(PM, J, skip, state=st)
        SS = torch.stack([S1] * G)
        carry, npm = eng.fold_carry(SS, 1, J, skip)
        eng.shard_repair(PM, carry, npm, st, M, NR, J, skip, ids=IDS)
        L, EW, CNT, _ = eng.deciles_ids(M, NR, IDS, nb)
        return eng.long_short(EW, CNT)

    def single():
        return eng.pipeline(Ps, mss, J, skip, nb, max_month_days=maxd, min_month_days=0).LS

    fns = dict(halo=lambda: halo()[0], speculative=speculative, single=single)
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    times = {k: [] for k in fns}
    for _ in range(reps):
        for k, f in fns.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            f()
            torch.cuda.synchronize()
            times[k].append(1e3 * (time.perf_counter() - t0))
    # back to back, as the bench's timed loop runs steps (host launches overlap device work)
    pipelined, enqueue = [], []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            halo()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        pipelined.append(1e3 * (t2 - t0) / 20)
        enqueue.append(1e3 * (t1 - t0) / 20)
    # CSM_HALO_GRAPH=1: the whole rank pass captured as ONE hipGraph (no host enqueue), replayed
    # back to back; its long-short and listed count checked bit for bit against an eager pass
    graph = None
    if os.environ.get("CSM_HALO_GRAPH") == "1":
        LSe, cnte = [x.clone() for x in halo()[:2]]
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):   # (warm the capture stream's engine binding)
            halo()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            LSg, cntg = halo()[:2]
        g.replay()
        torch.cuda.synchronize()
        same = bool(torch.equal(LSg.view(torch.int64), LSe.view(torch.int64)) and
                    torch.equal(cntg, cnte))
        rep = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                g.replay()
            torch.cuda.synchronize()
            rep.append(1e3 * (time.perf_counter() - t0) / 20)
        graph = {"replay_ms_median": round(float(np.median(rep)), 4),
                 "replay_ms_min": round(float(np.min(rep)), 4), "bits_equal_eager": same}
        del g
    names = ["shard_halo", "signal_shard_halo", "need+union", "summary_cols", "fix_cols",
             "deciles_ids", "gather_emul+long_short"]
    st_ms = {n: [] for n in names}
    for _ in range(reps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(8)]
        _, cnt, _, _, _ = halo(ev)
        torch.cuda.synchronize()
        for i, n in enumerate(names):
            st_ms[n].append(ev[i].elapsed_time(ev[i + 1]))
    S = 6 + J + skip + 1
    diag = None
    if len(sys.argv) > 6 and sys.argv[6] == "diag":   # who is listed, and why
        carry_h, npm_h, flags = eng.shard_halo(P, ms, hp.H, hp.F, J, skip)
        _, _, _, _, st = eng.signal_shard_halo(P, msh, maxd, J, skip, carry_h, npm_h)
        mask = eng.shard_need(flags, st, H)
        idx, cnt = eng.shard_union(torch.stack([other[0], mask, other[2]]), N, cap)
        n = min(int(cnt.item()), cap)
        ii = idx[:n].long()
        f = flags[ii].cpu().numpy()
        t = st.t[:, ii].cpu().numpy()
        bit = lambda m, r: ((m[r][ii // 64] >> (ii % 64)) & 1).cpu().numpy()
        b0 = bit(other[0], 3)
        b2 = bit(other[2], 2)
        from collections import Counter
        diag = Counter(f"flag{int(a)}_n{'>0' if c > 0 else '0'}_pend{int(d >= 0)}_head0{int(h)}"
                       f"_later{int(l)}" for a, c, d, h, l in zip(f, t[0], t[1], b0, b2))
        diag = dict(diag.most_common(12))
    print(json.dumps({
        "diag": diag,
        "N": N, "days_per_rank": dpr, "split_cells": cells or 32768,
        "dec_split": __import__("os").environ.get("CSM_DEC_SPLIT", "default (2: auto)"),
        "fused_halo": fused,
        "tune": __import__("os").environ.get("CSM_TUNE", ""), "T_d_with_halo": int(P.shape[0]), "T_m": T_m, "H": hp.H,
        "F": hp.F, "G_emulated": G, "cap": cap, "listed_this_rank": int(cnt.item()),
        "collective_bytes_per_rank": {"need_bits": 4 * 8 * ((N + 63) // 64),
                                      "records": 8 * S * cap,
                                      "allgather_path_records": 8 * S * N},
        "ms_median": {k: round(float(np.median(v)), 4) for k, v in times.items()},
        "ms_min": {k: round(float(np.min(v)), 4) for k, v in times.items()},
        "halo_back_to_back_ms_median": round(float(np.median(pipelined)), 4),
        "halo_host_enqueue_ms_median": round(float(np.median(enqueue)), 4),
        "halo_graph": graph,
        "halo_stages_ms_median": {n: round(float(np.median(v)), 4) for n, v in st_ms.items()},
    }), flush=True)


if __name__ == "__main__":
    main()
