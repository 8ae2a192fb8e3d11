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
    ne = torch.stack([(L == 9).any(2), (L == 0).any(2)], 0).int()   # [leg][t][b] non-empty cohort
    cs = torch.cat([torch.zeros_like(ne[:, :1]), ne.cumsum(1)], 1)   # cs[:, t] = months < t
    gen = torch.zeros(T_m, B, dtype=torch.bool, device=L.device)
    empty = torch.ones(T_m, B, dtype=torch.bool, device=L.device)
    Kmax = max(Ks)
    for t in range(T_m):
        lo = max(0, t - Kmax)
        empty[t] = (cs[:, t + 1] - cs[:, lo]).sum(0) == 0
        for K in Ks:   # steady (telescoping): t >= K and as many non-empty cohorts in both windows
            k1 = cs[:, t + 1] - cs[:, max(0, t - K + 1)]
            k0 = cs[:, t] - cs[:, max(0, t - K)]
            gen[t] |= ~((k1 == k0) & (t >= K)).all(0)
    gen &= ~empty
    g = gen.sum(1).cpu()
    print(f"J={J}: general rows {int(g.sum())} of {T_m * B} ({100 * g.sum() / (T_m * B):.1f} %), "
          f"empty rows {int(empty.sum())}, general rows after month 40: {int(g[40:].sum())}")
