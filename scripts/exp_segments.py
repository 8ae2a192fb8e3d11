"""C4: one-shot fused pass vs run_segmented with S segments (signal of segment g overlapped
with the ranking of segment g-1 on a side stream).  Interleaved, median ms, bit check."""
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
pan = make_device_panel(N, days, ms, seed=4, device="cuda:0")
eng = csmom.Engine(0)
T_m = len(ms) - 1
maxd = int(np.diff(ms).max())
M, NR = eng.empty((T_m, N)), eng.empty((T_m, N))
L = eng.empty((T_m, N), torch.int8)
EW, CNT, LS = eng.empty((T_m, 10)), eng.empty((T_m, 10), torch.int32), eng.empty((T_m,))
bufs = {S: (eng.empty((T_m, N)), eng.empty((T_m, N)), eng.empty((T_m, N), torch.int8),
            eng.empty((T_m, 10)), eng.empty((T_m, 10), torch.int32), eng.empty((T_m,)))
        for S in (2, 3, 4, 6, 8)}
plans = {S: eng.segmented_plan(pan.P, ms, 12, 1, S) for S in bufs}


def one():
    eng.signal(pan.P, pan.month_start, maxd, 12, 1, out=(None, None, M, NR))
    eng.deciles(M, NR, 10, out=(L, EW, CNT, None))
    eng.long_short(EW, CNT, LS)


def timed(fn):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(); fn(); b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b)


res = {"one": []}
res.update({f"seg{S}": [] for S in bufs})
for rnd in range(8):
    t = timed(one)
    if rnd: res["one"].append(t)
    for S in bufs:
        t = timed(lambda: eng.run_segmented(pan.P, pan.month_start, plans[S], 12, 1, 10, out=bufs[S]))
        if rnd: res[f"seg{S}"].append(t)
eq = {S: all(torch.equal(x.view(torch.int8) if x.dtype != torch.int8 else x,
                         y.view(torch.int8) if y.dtype != torch.int8 else y)
             for x, y in zip(bufs[S], (M, NR, L, EW, CNT, LS))) for S in bufs}
print(json.dumps({"ms_median": {k: round(float(np.median(v)), 4) for k, v in res.items()},
                  "bits_equal": {f"seg{S}": v for S, v in eq.items()}}), flush=True)
