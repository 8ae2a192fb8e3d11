"""One-GPU rehearsal of a date-shard rank's pass at C4 size (no collective: the all-gather is
replaced by a device stack of the two ranks' summaries).  Times, interleaved:
  single : the 1-GPU fused pass (k_signal + k_deciles + k_long_short)
  unfused: k_month_end -> summary -> fold -> k_momentum(carry) -> deciles -> long-short
  fused  : k_signal<SH>(empty state, PM, end state) -> summary from state -> fold -> k_shard_repair -> deciles -> LS
and checks fused == unfused bit for bit on rank 1's shard.  Prints one JSON line."""
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import csmom  # noqa: E402
from csmom.synth import make_device_panel, shard_calendar  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    days_per_rank = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    indep = len(sys.argv) > 4 and sys.argv[4] == "indep"   # independent per-rank panels
    dev = torch.device("cuda", 0)
    eng = csmom.Engine(0)
    J, skip, nb = 12, 1, 10
    panels, cals = [], []
    for r in range(2):
        days, ms_host, _, months = shard_calendar("1980-01-01", 2 * days_per_rank, 2, r)
        shard = None if indep else (r, 2, 1, days_per_rank)
        panels.append(make_device_panel(N, days, ms_host, seed=1000 + r, device=dev, shard=shard))
        cals.append(ms_host)
    p0, p1 = panels
    maxd = int(max(np.diff(c).max() for c in cals))
    PM0, _ = eng.month_end(p0.P, p0.month_start)
    S0 = eng.shard_summary(PM0, J, skip)
    del PM0
    torch.cuda.synchronize()

    def single():
        _, _, M, NR = eng.signal(p1.P, p1.month_start, maxd, J, skip)
        L, EW, CNT, _ = eng.deciles(M, NR, nb)
        return eng.long_short(EW, CNT), M, NR, L

    def unfused():
        PM, _ = eng.month_end(p1.P, p1.month_start)
        S1 = eng.shard_summary(PM, J, skip)
        carry, npm = eng.fold_carry(torch.stack([S0, S1]), 1, J, skip)
        _, M, NR = eng.momentum(PM, J, skip, carry=carry, next_pm=npm)
        L, EW, CNT, _ = eng.deciles(M, NR, nb)
        return eng.long_short(EW, CNT), M, NR, L

    def fused():
        PM, _, M, NR, st = eng.signal_shard(p1.P, p1.month_start, maxd, J, skip)
        S1 = eng.shard_summary(PM, J, skip, state=st)
        carry, npm = eng.fold_carry(torch.stack([S0, S1]), 1, J, skip)
        eng.shard_repair(PM, carry, npm, st, M, NR, J, skip)
        L, EW, CNT, _ = eng.deciles(M, NR, nb)
        return eng.long_short(EW, CNT), M, NR, L

    IDS = torch.empty((p1.month_start.numel() - 1, N), dtype=torch.int16, device=dev)

    def fused_ids():   # the shard pass writes bucket ids; repair rewrites them; deciles on ids
        PM, _, M, NR, st = eng.signal_shard(p1.P, p1.month_start, maxd, J, skip, ids=IDS)
        S1 = eng.shard_summary(PM, J, skip, state=st)
        carry, npm = eng.fold_carry(torch.stack([S0, S1]), 1, J, skip)
        eng.shard_repair(PM, carry, npm, st, M, NR, J, skip, ids=IDS)
        L, EW, CNT, _ = eng.deciles_ids(M, NR, IDS, nb)
        return eng.long_short(EW, CNT), M, NR, L

    def staged():   # the product path (bucket ids), HIP events between its stages
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(7)]
        ev[0].record()
        PM, _, M, NR, st = eng.signal_shard(p1.P, p1.month_start, maxd, J, skip, ids=IDS)
        ev[1].record()
        S1 = eng.shard_summary(PM, J, skip, state=st)
        ev[2].record()
        SS = torch.stack([S0, S1])
        ev[3].record()
        carry, npm = eng.fold_carry(SS, 1, J, skip)
        ev[4].record()
        eng.shard_repair(PM, carry, npm, st, M, NR, J, skip, ids=IDS)
        ev[5].record()
        L, EW, CNT, _ = eng.deciles_ids(M, NR, IDS, nb)
        ev[6].record()
        torch.cuda.synchronize()
        names = ["signal+PM", "shard_summary", "stack", "fold_carry", "shard_repair",
                 "deciles_ids"]
        return {n: round(ev[i].elapsed_time(ev[i + 1]), 4) for i, n in enumerate(names)}

    def decile_ab():   # the shard's decile pass on ids: split (auto) vs merged, interleaved
        _, _, M, NR, _ = eng.signal_shard(p1.P, p1.month_start, maxd, J, skip, ids=IDS)
        out, res = {}, {}
        for _ in range(reps):
            for v in (2, 0):
                assert eng.lib.csm_tune(b"dec_split", v) == 0
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                r = eng.deciles_ids(M, NR, IDS, nb)
                e1.record()
                torch.cuda.synchronize()
                out.setdefault(v, []).append(e0.elapsed_time(e1))
                res[v] = r
        assert eng.lib.csm_tune(b"dec_split", 2) == 0
        same = bool(torch.equal(res[2][0], res[0][0]) and torch.equal(res[2][2], res[0][2]))
        return {"split_ms": round(float(np.median(out[2])), 4),
                "merged_ms": round(float(np.median(out[0])), 4), "labels_counts_equal": same}

    fns = dict(single=single, unfused=unfused, fused=fused, fused_ids=fused_ids)
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    _, Mu, NRu, Lu = unfused()
    _, Mf, NRf, Lf = fused()
    _, Mi, NRi, Li = fused_ids()
    torch.cuda.synchronize()

    def bits(a, b):
        a, b = a.view(torch.int64), b.view(torch.int64)
        na, nb_ = torch.isnan(a.view(torch.float64)), torch.isnan(b.view(torch.float64))
        return bool(torch.equal(na, nb_) and torch.equal(a[~na], b[~nb_]))

    equal = dict(M=bits(Mf, Mu), NR=bits(NRf, NRu), L=bool(torch.equal(Lf, Lu)),
                 M_ids=bits(Mi, Mu), L_ids=bool(torch.equal(Li, Lu)))
    del Mu, NRu, Lu, Mf, NRf, Lf, Mi, NRi, Li
    times = {k: [] for k in fns}
    for _ in range(reps):
        for k, f in fns.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            f()
            torch.cuda.synchronize()
            times[k].append(1e3 * (time.perf_counter() - t0))
    print(json.dumps({"N": N, "T_d": int(p1.P.shape[0]), "T_m": int(p1.month_start.numel() - 1),
                      "ms_median": {k: round(float(np.median(v)), 4) for k, v in times.items()},
                      "ms_min": {k: round(float(np.min(v)), 4) for k, v in times.items()},
                      "fused_ids_stages_ms": staged(),
                      "deciles_ids_ab": decile_ab(),
                      "fused_equals_unfused": equal}), flush=True)


if __name__ == "__main__":
    main()
