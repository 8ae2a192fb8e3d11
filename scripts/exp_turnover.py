"""C5-shaped turnover pass: time k_turnover (costs on - costs off) on real bootstrap labels
(leading months without labels: the non-steady path) and on labels valid from month 0.  Dev tool."""
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
Lf = torch.randint(0, 10, L.shape, dtype=torch.int8, device="cuda:0")
ws = torch.empty(int(eng.lib.csm_portfolio_workspace(T_m, B, N, 10, 12)), dtype=torch.uint8,
                 device="cuda:0")


def timed(fn):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); a.record(); fn(); b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b)


res = {}
for rnd in range(5):
    for name, LL in (("real", L), ("full", Lf)):
        for costs in (True, False):
            t = timed(lambda: eng.portfolio_multi(LL, NR, 10, Ks=(3, 6, 9, 12), B=B, workspace=ws,
                                                  with_costs=costs))
            if rnd:
                res.setdefault(f"{name}_{'costs' if costs else 'nocosts'}", []).append(t)
med = {k: round(float(np.median(v)), 3) for k, v in res.items()}
med["turnover_real"] = round(med["real_costs"] - med["real_nocosts"], 3)
med["turnover_full"] = round(med["full_costs"] - med["full_nocosts"], 3)
print(json.dumps({"B": B, "N": N, "T_m": T_m, "ms": med}), flush=True)
