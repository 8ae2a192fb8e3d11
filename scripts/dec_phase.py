"""Dev tool: per-phase wall-clock of the PRE decile pass at a sweep's shape (C5 by default):
boot_scan panels -> csm_deciles_ids with csm_tune_ptr("dec_timing") set.  Prints the mean
microseconds between phase marks (0 start, 1 hist zeroed, 2 histogram, 3 targets, 4 label
table, 5 merged sweep, 6 selection, 7 edges, 8 labels) over the rows the merged pass kept,
and the rows it left to the general kernel.  Usage: python scripts/dec_phase.py [B] [N] [T_d]"""
import ctypes
import sys
import time

import numpy as np
import torch

sys.path.insert(0, str(__import__('pathlib').Path(__file__).resolve().parents[1]))
import csmom  # noqa: E402
from csmom.synth import bday_calendar, make_device_panel  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 100
N = int(sys.argv[2]) if len(sys.argv) > 2 else 5000
T_d = int(sys.argv[3]) if len(sys.argv) > 3 else 6522
eng = csmom.Engine(0)
days, ms_h, _ = bday_calendar("2000-01-03", T_d)
pan = make_device_panel(N, days, ms_h, seed=7, device="cuda:0")
PM, _ = eng.month_end(pan.P, pan.month_start)
R, _, _ = eng.momentum(PM, 12, 1, with_ret=True)
R = R.contiguous()
T_m = R.shape[0]
Js = (3, 6, 9, 12)
_, outs, NR, bad = eng.boot_scan(R, B, Js, 1, b0=0)
rows = T_m * B
for J, (M, IDS) in zip(Js, outs):
    M2, I2 = M.reshape(rows, N), IDS.reshape(rows, N)
    for _ in range(2):
        eng.deciles_ids(M2, None, I2, 10)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        eng.deciles_ids(M2, None, I2, 10)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    tim = torch.zeros(rows * 9, dtype=torch.int64, device="cuda:0")
    eng.lib.csm_tune_ptr(b"dec_timing", ctypes.c_void_p(tim.data_ptr()))
    eng.deciles_ids(M2, None, I2, 10)
    torch.cuda.synchronize()
    eng.lib.csm_tune_ptr(b"dec_timing", ctypes.c_void_p(0))
    t = tim.view(rows, 9).cpu().numpy().astype(np.float64)
    kept = t[:, 8] > 0
    d = np.diff(t[kept], axis=1) / 100.0   # 100 MHz wall clock -> us
    tot = (t[kept, 8] - t[kept, 0]) / 100.0
    # rows in flight: span of the whole launch over the sum of row durations
    span = (t[kept, 8].max() - t[kept, 0].min()) / 100.0
    print(f"J={J}: {ms * 1e3:.1f} us/launch, rows {rows}, merged {kept.sum()} "
          f"(left {rows - kept.sum()}), row {tot.mean():.2f} us (p50 {np.median(tot):.2f}, "
          f"p99 {np.percentile(tot, 99):.2f}), rows in flight {tot.sum() / span:.0f}")
    print("   phase us: " + " ".join(f"{i}-{i + 1}:{v:.2f}" for i, v in enumerate(d.mean(0))))
