"""C4 decile pass on bucket ids: merged sweep (MG kernel) vs the general kernel.  Counts the
rows the merged kernel leaves (csm_tune dec_merge 2 + a sentinel), times MG-only / general /
combined interleaved (median of 5), and the MG kernel's per-row phases (dec_timing marks:
3 -> 4 = pre-table + merged sweep).  Dev tool: prints one JSON line."""
import ctypes
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
M, NR, IDB = eng.empty((T_m, N)), eng.empty((T_m, N)), eng.empty((T_m, N), torch.int16)
L = eng.empty((T_m, N), torch.int8)
EW, CNT = eng.empty((T_m, 10)), eng.empty((T_m, 10), torch.int32)
eng.signal_ids(pan.P, pan.month_start, maxd, 12, 1, out=(None, None, M, NR, IDB))
tune = lambda k, v: eng.lib.csm_tune(k.encode(), v)


def dec():
    eng.deciles_ids(M, NR, IDB, 10, out=(L, EW, CNT, None))


tune("dec_merge", 2)
L.fill_(100)
dec()
torch.cuda.synchronize()
left = np.nonzero((L == 100).any(dim=1).cpu().numpy())[0]
nv = (~torch.isnan(M)).sum(dim=1).cpu().numpy()


def timed(v):
    tune("dec_merge", v)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); dec(); b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b)


times = {v: [] for v in (2, 0, 1, 12, 10)}   # 12 / 10: merged / general without the decile sums
for rnd in range(6):
    for v in times:
        tune("dec_ablate", 1 if v >= 10 else 0)
        t = timed(v % 10)
        if rnd:
            times[v].append(t)
tune("dec_ablate", 0)
tune("dec_merge", 2)
dec()
tim = torch.full((T_m, 9), -1, dtype=torch.int64, device="cuda:0")
eng.lib.csm_tune_ptr(b"dec_timing", ctypes.c_void_p(tim.data_ptr()))
dec()
torch.cuda.synchronize()
eng.lib.csm_tune_ptr(b"dec_timing", None)
tune("dec_merge", 1)
th = tim.cpu().numpy()
ok = (th >= 0).all(axis=1)
t = th[ok].astype(np.float64) / 100.0
d = np.diff(t, axis=1)
names = ["sample", "histogram", "targets", "pretable", "sweep", "offer", "select+edges", "final"]
print(json.dumps({
    "rows_left_by_merged": int(len(left)), "left_rows": left[:40].tolist(),
    "left_rows_ranked_counts": nv[left[:40]].tolist(),
    "ms": {"merged_only": round(float(np.median(times[2])), 4), "general": round(float(np.median(times[0])), 4),
           "merged+general": round(float(np.median(times[1])), 4),
           "merged_only_nosums": round(float(np.median(times[12])), 4),
           "general_nosums": round(float(np.median(times[10])), 4)},
    "mg_rows_timed": int(ok.sum()),
    "phase_us_mean": {n: round(float(d[:, i].mean()), 2) for i, n in enumerate(names)},
    "phase_us_max": {n: round(float(d[:, i].max()), 2) for i, n in enumerate(names)},
    "row_us_mean": round(float((t[:, -1] - t[:, 0]).mean()), 2),
    "span_us": round(float(t[:, -1].max() - t[:, 0].min()), 2)}), flush=True)
