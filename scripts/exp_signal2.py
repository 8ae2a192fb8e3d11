"""Round-2 A/B of the fused signal kernel on C4, interleaved in one process (median of 5
rounds): paired 16-B output stores vs per-asset 8-B stores, with / without the bucket-id
output, store ablation (reads only), 3 vs 4 month buffers; checks the variants' outputs are
bit-identical.  Dev tool: prints one JSON line."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import csmom  # noqa: E402
from csmom.synth import bday_calendar, make_device_panel  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
TD = 10_000
days, ms, _ = bday_calendar("1985-01-01", TD)
pan = make_device_panel(N, days, ms, seed=4000, device="cuda:0", shard=(0, 1, 4, float(TD)))
eng = csmom.Engine(0)
T_m = len(ms) - 1
maxd = int(np.diff(ms).max())
mind = int(np.diff(ms)[1:-1].min())   # interior months
tune = lambda k, v: eng.lib.csm_tune(k.encode(), v)
outs = {}


def timed(fn):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); fn(); b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b)


def run(name):
    M, NR = eng.empty((T_m, N)), eng.empty((T_m, N))
    IDS = eng.empty((T_m, N), torch.int16)
    pair = 0 if name.startswith("nopair") else 1
    tune("signal_pair", pair)
    tune("signal_store", 2 if name == "nostore" else 4 if name.startswith("noscanst") else
         3 if name.startswith("noscan") else 1 if "_nt" in name else 0)
    tune("signal_rr", 1 if "_rr" in name else 0)
    tune("signal_bl", 1 if "_bl" in name else 0)
    tune("signal_nbuf", int(name.split("nbuf")[1][0]) if "nbuf" in name else 4)
    tune("signal_maxd23", 0 if "d24" in name else 1)
    tune("signal_db", int(name.split("db")[1]) if "db" in name else 0)
    tune("signal_bwf", int(name.split("bwf")[1].split("_")[0]) if "bwf" in name else 1)
    if "ids" in name:
        f = lambda: eng.signal_ids(pan.P, pan.month_start, maxd, 12, 1, out=(None, None, M, NR, IDS),
                                   min_month_days=mind)
    else:
        f = lambda: eng.signal(pan.P, pan.month_start, maxd, 12, 1, out=(None, None, M, NR))
    t = timed(f)
    outs[name] = (M, NR, IDS if "ids" in name else None)
    return t


names = (sys.argv[2].split(",") if len(sys.argv) > 2 else
         ["pair_ids", "pair", "nopair_ids", "nopair", "nostore", "pair_ids_nbuf3"])
times = {n: [] for n in names}
for rnd in range(6):
    for n in names:
        t = run(n)
        if rnd:
            times[n].append(t)
for k, v in (("signal_pair", 1), ("signal_store", 0), ("signal_nbuf", 4), ("signal_maxd23", 1), ("signal_db", 0),
             ("signal_bwf", 0), ("signal_rr", 0), ("signal_bl", 0)):
    tune(k, v)
eq = lambda a, b: bool(torch.equal(a.view(torch.int64), b.view(torch.int64)))
base = outs["nopair" if "nopair" in outs else names[0]]
same = {n: eq(outs[n][0], base[0]) and eq(outs[n][1], base[1]) and
        (outs[n][2] is None or base[2] is None or bool(torch.equal(outs[n][2], base[2])))
        for n in names if n != "nostore" and not n.startswith("noscan")}
alg = 8.0 * N * TD + 16.0 * N * T_m
res = {n: round(float(np.median(t)), 4) for n, t in times.items()}
print(json.dumps({"N": N, "T_d": TD, "k_signal_ms": res,
                  "GBps": {n: round(alg / (v * 1e-3) / 1e9, 1) for n, v in res.items()},
                  "bits_equal_to_nopair": same}), flush=True)
