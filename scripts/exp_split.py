"""A/B: fused k_signal vs split month-end (k_month_end loop / one-shot rows variant) + scan
(single or time-chunked) on C4, interleaved in one process; checks bit-equality.  Dev tool."""
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
pan = make_device_panel(N, days, ms, seed=4, device="cuda:0")
eng = csmom.Engine(0)
T_m = len(ms) - 1
maxd = int(np.diff(ms).max())
tune = lambda k, v: eng.lib.csm_tune(k.encode(), v)
M, NR = eng.empty((T_m, N)), eng.empty((T_m, N))
M2, NR2 = eng.empty((T_m, N)), eng.empty((T_m, N))
PM = eng.empty((T_m, N))
ws = {}
for C in (2, 4, 8):
    nbytes = int(eng.lib.csm_momentum_chunked_workspace(T_m, N, 12, 1, C))
    ws[C] = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")


def ev():
    return torch.cuda.Event(enable_timing=True)


res = {}


def rec(name, t):
    res.setdefault(name, []).append(t)


for rnd in range(6):
    e = [ev() for _ in range(2)]
    e[0].record(); eng.signal(pan.P, pan.month_start, maxd, 12, 1, out=(None, None, M, NR)); e[1].record()
    torch.cuda.synchronize()
    if rnd: rec("fused", e[0].elapsed_time(e[1]))
    for me in ("loop", "rows"):
        tune("month_end_rows", maxd if me == "rows" else 0)
        e = [ev() for _ in range(2)]
        e[0].record(); eng.month_end(pan.P, pan.month_start, PM=PM); e[1].record()
        torch.cuda.synchronize()
        if rnd: rec(f"month_end_{me}", e[0].elapsed_time(e[1]))
    tune("month_end_rows", 0)
    for C in (1, 2, 4, 8):
        e = [ev() for _ in range(2)]
        e[0].record()
        if C == 1:
            eng.momentum(PM, 12, 1, out=(None, M2, NR2))
        else:
            eng.momentum_chunked(PM, 12, 1, chunks=C, out=(None, M2, NR2), workspace=ws[C])
        e[1].record()
        torch.cuda.synchronize()
        if rnd: rec(f"scan_C{C}", e[0].elapsed_time(e[1]))
eq = lambda a, b: bool(torch.equal(a.view(torch.int64), b.view(torch.int64)))
tune("month_end_rows", maxd)
PM2 = eng.empty((T_m, N))
eng.month_end(pan.P, pan.month_start, PM=PM2)
tune("month_end_rows", 0)
eng.month_end(pan.P, pan.month_start, PM=PM)
torch.cuda.synchronize()
out = {k: round(float(np.median(v)), 4) for k, v in res.items()}
alg_me = 8.0 * N * TD + 8.0 * N * T_m
print(json.dumps({"N": N, "T_d": TD, "ms": out,
                  "month_end_GBps": {k: round(alg_me / (out[f"month_end_{k}"] * 1e-3) / 1e9, 1)
                                     for k in ("loop", "rows")},
                  "rows_PM_equal": eq(PM, PM2), "split_equal_fused": eq(M, M2) and eq(NR, NR2)}),
      flush=True)
