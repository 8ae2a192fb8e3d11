"""Dev tool: per-phase wall-clock of the C2 decile pass (the K = 1 path on a 5k-asset panel:
month-end -> time-chunked scan with ids -> csm_deciles_ids_ls with decile sums and the fused
long-short), csm_tune_ptr("dec_timing") set.  Phase marks as scripts/dec_phase.py.
Usage: python scripts/dec_phase_c2.py [N] [T_d]"""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, str(__import__('pathlib').Path(__file__).resolve().parents[1]))
import csmom  # noqa: E402
from csmom.synth import bday_calendar, make_device_panel  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
T_d = int(sys.argv[2]) if len(sys.argv) > 2 else 6522
eng = csmom.Engine(0)
days, ms_h, _ = bday_calendar("2000-01-03", T_d)
pan = make_device_panel(N, days, ms_h, seed=7, device="cuda:0")
PM, _ = eng.month_end(pan.P, pan.month_start)
T_m = PM.shape[0]
ch = eng.default_chunks(T_m, N, 12, 1)
nbytes = int(eng.lib.csm_momentum_chunked_workspace(T_m, N, 12, 1, ch))
ws = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
M, NR = eng.empty((T_m, N)), eng.empty((T_m, N))
IDS = eng.empty((T_m, N), torch.int16)
eng.momentum_chunked(PM, 12, 1, chunks=ch, out=(None, M, NR), workspace=ws, ids=IDS)
L = eng.empty((T_m, N), torch.int8)
EW, CNT = eng.empty((T_m, 10)), eng.empty((T_m, 10), torch.int32)
LS = eng.empty((T_m,))
run = lambda: eng.deciles_ids(M, NR, IDS, 10, out=(L, EW, CNT, None), LS=LS)
for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    run()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
tim = torch.zeros(T_m * 9, dtype=torch.int64, device="cuda:0")
eng.lib.csm_tune_ptr(b"dec_timing", ctypes.c_void_p(tim.data_ptr()))
run()
torch.cuda.synchronize()
eng.lib.csm_tune_ptr(b"dec_timing", ctypes.c_void_p(0))
t = tim.view(T_m, 9).cpu().numpy().astype(np.float64)
kept = t[:, 8] > 0
d = np.diff(t[kept], axis=1) / 100.0
tot = (t[kept, 8] - t[kept, 0]) / 100.0
span = (t[kept, 8].max() - t[kept, 0].min()) / 100.0
start = (t[kept, 0] - t[kept, 0].min()) / 100.0
print(f"C2 deciles+LS: {ms * 1e3:.1f} us/launch, rows {T_m}, merged {kept.sum()}, row "
      f"{tot.mean():.2f} us (p50 {np.median(tot):.2f}, max {tot.max():.2f}), span {span:.2f} us, "
      f"start spread {start.max():.2f} us, rows in flight {tot.sum() / span:.1f}")
print("   phase us: " + " ".join(f"{i}-{i + 1}:{v:.2f}" for i, v in enumerate(d.mean(0))))
