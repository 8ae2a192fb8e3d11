"""C4 A/B: the fused signal kernel vs the split path (row-sweep month-end + per-asset scan),
interleaved in one process (median of 5 rounds).  Dev tool: prints one JSON line."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import csmom  # noqa: E402
from csmom.synth import bday_calendar, make_device_panel  # noqa: E402

N, TD = 100_000, 10_000
days, ms, _ = bday_calendar("1985-01-01", TD)
pan = make_device_panel(N, days, ms, seed=4000, device="cuda:0", shard=(0, 1, 4, float(TD)))
eng = csmom.Engine(0)
T_m = len(ms) - 1
maxd = int(np.diff(ms).max())
tune = lambda k, v: eng.lib.csm_tune(k.encode(), v)
PM = eng.empty((T_m, N))
M, NR = eng.empty((T_m, N)), eng.empty((T_m, N))
IDS = eng.empty((T_m, N), torch.int16)


def timed(fn):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); fn(); b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b)


def v_signal(d23):
    tune("signal_maxd23", d23)
    return timed(lambda: eng.signal_ids(pan.P, pan.month_start, maxd, 12, 1, out=(None, None, M, NR, IDS)))


def v_me(rows):
    tune("month_end_rows", maxd if rows else 0)
    t = timed(lambda: eng.month_end(pan.P, pan.month_start, PM=PM))
    tune("month_end_rows", 0)
    return t


def v_scan():
    return timed(lambda: eng.momentum(PM, 12, 1, out=(None, M, NR), chunked=False))


var = {"signal": lambda: v_signal(0), "signal_d23": lambda: v_signal(1),
       "month_end": lambda: v_me(0), "month_end_rows": lambda: v_me(1), "scan": v_scan}
times = {k: [] for k in var}
for rnd in range(6):
    for k, f in var.items():
        t = f()
        if rnd:
            times[k].append(t)
tune("signal_maxd23", 0)
res = {k: round(float(np.median(v)), 4) for k, v in times.items()}
alg_sig = 8.0 * N * TD + 16.0 * N * T_m
alg_me = 8.0 * N * TD + 8.0 * N * T_m
print(json.dumps({"ms": res, "GBps": {"signal": round(alg_sig / res["signal"] / 1e6, 1),
                                      "signal_d23": round(alg_sig / res["signal_d23"] / 1e6, 1),
                                      "month_end_rows": round(alg_me / res["month_end_rows"] / 1e6, 1),
                                      "scan": round(24.0 * N * T_m / res["scan"] / 1e6, 1)}}), flush=True)
