"""Dev tool: how many (month, panel) rows of a C5 bootstrap batch take the general turnover
launch (some (K, leg) window of month t or t-1 holds an empty cohort), per J, and where they
are in t.  Usage: python scripts/turn_rows.py [B]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import csmom  # noqa: E402
from csmom.synth import bday_calendar, make_device_panel  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 100
N, T_d = 5000, 6522
eng = csmom.Engine(0)
days, ms_h, _ = bday_calendar("2000-01-03", T_d)
pan = make_device_panel(N, days, ms_h, seed=7, device="cuda:0")
PM, _ = eng.month_end(pan.P, pan.month_start)
R, _, _ = eng.momentum(PM, 12, 1, with_ret=True)
R = R.contiguous()
T_m = R.shape[0]
print("R_base NaN months (all assets):", int(torch.isnan(R).all(1).sum()), "of", T_m,
      " rows with any NaN:", int(torch.isnan(R).any(1).sum()))
Js, Ks = (3, 6, 9, 12), (3, 6, 9, 12)
_, outs, NR, bad = eng.boot_scan(R, B, Js, 1, b0=0, with_ids=True)
for J, (M, IDS) in zip(Js, outs):
    L, _, _, _ = eng.deciles_ids(M.reshape(T_m * B, N), None, IDS.reshape(T_m * B, N), 10)
    L = L.reshape(T_m, B, N)
    ne = torch.stack([(L == 9).any(2), (L == 0).any(2)], 0)   # [leg][t][b] cohort non-empty
    gen = torch.zeros(T_m, B, dtype=torch.bool, device=L.device)
    for K in Ks:
        for t in range(T_m):
            w1 = ne[:, max(0, t - K + 1):t + 1].all(1) & (t - K + 1 >= 0)
            w0 = ne[:, max(0, t - K):t].all(1) & (t - K >= 0)
            gen[t] |= ~(w1 & w0).all(0)
    g = gen.sum(1).cpu()
    first = [int(t) for t in torch.nonzero(g < B).flatten()[:1]]
    print(f"J={J}: general rows {int(g.sum())} of {T_m * B} ({100 * g.sum() / (T_m * B):.1f} %), "
          f"all-general months {int((g == B).sum())}, first month with a steady row {first}, "
          f"general rows after month 40: {int(g[40:].sum())}")
