"""C5-shaped cohort sums (no costs): label sort + segment gathers vs per-wave LDS atomics, interleaved.
100 bootstrap panels of a 5k x 300-month base, J=12, Ks (3,6,9,12).  Dev tool."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import csmom  # noqa: E402
from csmom.synth import bday_calendar, make_device_panel  # noqa: E402

N, TD, B = 5_000, 6_522, 100
days, ms, _ = bday_calendar("2000-01-03", TD)
pan = make_device_panel(N, days, ms, seed=5005, device="cuda:0")
eng = csmom.Engine(0)
PM0, _ = eng.month_end(pan.P, pan.month_start)
R0, _, _ = eng.momentum(PM0, 12, 1, with_ret=True)
_, PMb = eng.bootstrap(R0, B, b0=0)
T_m = PMb.shape[0]
_, M, NR = eng.momentum(PMb, 12, 1)
L, _, _, _ = eng.deciles(M.view(T_m * B, N), None, 10)
L = L.view(T_m, B * N)
ws = torch.empty(int(eng.lib.csm_portfolio_workspace(T_m, B, N, 10, 12)), dtype=torch.uint8,
                 device="cuda:0")


def timed(fn):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); a.record(); fn(); b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b)


MODES = {"seg": (1, 1), "lds": (0, 1)}   # (cohort_seg, cohort_lds)
res = {m: [] for m in MODES}
outs = {}
for rnd in range(6):
    for m, (sg, ld) in MODES.items():
        eng.lib.csm_tune(b"cohort_seg", sg)
        eng.lib.csm_tune(b"cohort_lds", ld)
        t = timed(lambda: outs.__setitem__(m, eng.portfolio_multi(L, NR, 10, Ks=(3, 6, 9, 12), B=B,
                                                                  workspace=ws, with_costs=False)))
        if rnd:
            res[m].append(t)
eng.lib.csm_tune(b"cohort_seg", 1)
eng.lib.csm_tune(b"cohort_lds", 1)
a, b = outs["lds"][12].PR.cpu().numpy(), outs["seg"][12].PR.cpu().numpy()
m = ~np.isnan(a)
rel = float(np.max(np.abs(a[m] - b[m]) / np.maximum(np.abs(a[m]), 1e-300)))
print(json.dumps({"B": B, "N": N, "T_m": T_m,
                  "cohort_plus_overlap_ms": {k: round(float(np.median(v)), 3) for k, v in res.items()},
                  "max_rel_PR": rel}), flush=True)
