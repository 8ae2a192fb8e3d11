"""Narrow-row deciles (C5 shape: 30k rows of 5k assets): kernel time and per-phase durations
from the in-kernel wall-clock marks.  Dev tool: prints one JSON line."""
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import csmom  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 30_000
N = int(sys.argv[2]) if len(sys.argv) > 2 else 5_000
eng = csmom.Engine(0)
g = torch.Generator(device="cuda:0").manual_seed(3)
M = torch.randn((R, N), dtype=torch.float64, device="cuda:0", generator=g) * 0.2
M[torch.rand((R, N), device="cuda:0", generator=g) < 0.05] = float("nan")
L = eng.empty((R, N), torch.int8)
EW, CNT = eng.empty((R, 10)), eng.empty((R, 10), torch.int32)


def run():
    eng.deciles(M, None, 10, out=(L, EW, CNT, None))


for _ in range(3):
    run()
ts = []
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); run(); e1.record(); torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
tim = torch.full((R, 9), -1, dtype=torch.int64, device="cuda:0")
eng.lib.csm_tune_ptr(b"dec_timing", ctypes.c_void_p(tim.data_ptr()))
run()
torch.cuda.synchronize()
eng.lib.csm_tune_ptr(b"dec_timing", None)
t = tim.cpu().numpy().astype(np.float64) / 100.0   # 100 MHz ticks -> us
ok = (tim.cpu().numpy() >= 0).all(axis=1)
t = t[ok]
names = ["sample", "histogram", "targets", "refine", "gather", "select", "edges+table",
         "labels+sums"]
d = np.diff(t, axis=1)
print(json.dumps({"rows": R, "N": N, "kernel_ms": round(float(np.median(ts)), 4),
                  "rows_timed": int(ok.sum()),
                  "phase_us_mean": {n: round(float(d[:, i].mean()), 2) for i, n in enumerate(names)},
                  "row_us_mean": round(float((t[:, -1] - t[:, 0]).mean()), 2),
                  "span_us": round(float(t[:, -1].max() - t[:, 0].min()), 2)}), flush=True)
