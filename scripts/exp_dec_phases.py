"""Where k_deciles spends its time on C4: per-date phase durations from the in-kernel
wall-clock marks (csm_tune_ptr("dec_timing")).  Dev tool: prints one JSON line."""
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import csmom  # noqa: E402
from csmom.synth import bday_calendar, make_device_panel  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
IDS = int(sys.argv[2]) if len(sys.argv) > 2 else 0   # 2: fixed-map ids from csm_signal_ids
REG = int(sys.argv[3]) if len(sys.argv) > 3 else 1
ABL = int(sys.argv[4]) if len(sys.argv) > 4 else 0   # dec_ablate bitmask (1: no decile sums)
ROWS = int(sys.argv[5]) if len(sys.argv) > 5 else 0  # >0: time only the first ROWS dates
TD = 10_000
days, ms, _ = bday_calendar("1985-01-01", TD)
pan = make_device_panel(N, days, ms, seed=4, device="cuda:0")
eng = csmom.Engine(0)
T_m = len(ms) - 1
maxd = int(np.diff(ms).max())
M, NR = eng.empty((T_m, N)), eng.empty((T_m, N))
L = eng.empty((T_m, N), torch.int8)
EW, CNT = eng.empty((T_m, 10)), eng.empty((T_m, 10), torch.int32)
IDB = eng.empty((T_m, N), torch.int16)
eng.signal_ids(pan.P, pan.month_start, maxd, 12, 1, out=(None, None, M, NR, IDB))
eng.lib.csm_tune(b"dec_ids", 1 if IDS == 1 else 0)
eng.lib.csm_tune(b"dec_reg", REG)
eng.lib.csm_tune(b"dec_ablate", ABL)
if ROWS:
    M, NR, L, EW, CNT, IDB = M[:ROWS], NR[:ROWS], L[:ROWS], EW[:ROWS], CNT[:ROWS], IDB[:ROWS]
    T_m = ROWS
def dec():
    if IDS == 2:
        eng.deciles_ids(M, NR, IDB, 10, out=(L, EW, CNT, None))
    else:
        eng.deciles(M, NR, 10, out=(L, EW, CNT, None))


for _ in range(3):
    dec()
tim = torch.full((T_m, 9), -1, dtype=torch.int64, device="cuda:0")
eng.lib.csm_tune_ptr(b"dec_timing", ctypes.c_void_p(tim.data_ptr()))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
dec()
e1.record()
torch.cuda.synchronize()
eng.lib.csm_tune_ptr(b"dec_timing", None)
t = tim.cpu().numpy().astype(np.float64) / 100.0   # 100 MHz ticks -> us
ok = (tim.cpu().numpy() >= 0).all(axis=1)
t = t[ok]
names = ["sample", "histogram", "targets", "refine", "gather", "select", "edges+table",
         "labels+sums", ]
if ABL & 16:   # fine marks (csrc/deciles.inc): hist, targets+refine, gather prologue, sweep, ...
    names = ["histogram", "targets+refine", "gather_prologue", "gather_sweep", "gather_flush+minmax",
             "select", "edges", "table"]
d = np.diff(t, axis=1)
out = {"N": N, "ids": IDS, "reg": REG, "ablate": ABL, "rows": T_m, "rows_timed": int(ok.sum()), "kernel_ms": round(e0.elapsed_time(e1), 4),
       "phase_us_mean": {n: round(float(d[:, i].mean()), 2) for i, n in enumerate(names)},
       "phase_us_max": {n: round(float(d[:, i].max()), 2) for i, n in enumerate(names)},
       "row_us_mean": round(float((t[:, -1] - t[:, 0]).mean()), 2),
       "start_spread_us": round(float(t[:, 0].max() - t[:, 0].min()), 2),
       "span_us": round(float(t[:, -1].max() - t[:, 0].min()), 2)}
print(json.dumps(out), flush=True)
