"""How many turnover rows of one C5 batch (100 bootstrap panels, J = 12, K set {3,6,9,12},
legs-only) go to the general launch: the work-list count the steady launch leaves in the
portfolio workspace, against a host count of rows with a non-full leg window."""
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import csmom  # noqa: E402
from csmom.synth import bday_calendar, make_device_panel  # noqa: E402

dev = torch.device("cuda:0")
N, T_d, B, Ks = 5000, 6522, 100, (3, 6, 9, 12)
days, ms_host, _ = bday_calendar("2000-01-03", T_d)
eng = csmom.Engine(0)
panel = make_device_panel(N, days, ms_host, seed=5, device=dev)
PM0, _ = eng.month_end(panel.P, panel.month_start)
R0, _, _ = eng.momentum(PM0, 12, 1, with_ret=True)
_, PMb = eng.bootstrap(R0, B, b0=0, seed=5000, mean_block=6.0)
T_m = PMb.shape[0]
_, M, NR = eng.momentum(PMb, 12, 1)
L, _, _, _ = eng.deciles(M.reshape(T_m * B, N), None, 10)
L = L.reshape(T_m, B * N)
rows, Kmax, nb = T_m * B, max(Ks), 10
# pf_layout (csrc/portfolio.hip) for C = Ct = 1 (rows >= 4096)
cs = rows * Kmax * 1 * nb
fwt = 2 * cs + rows * 2
turn = fwt + rows * 2
cost = turn + 4 * rows
nbytes = (cost + 4 * rows) * 8 + 256
gen_b = (nbytes + 255) // 256 * 256
ws_bytes = int(eng.lib.csm_portfolio_workspace(T_m, B, N, nb, Kmax))
ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=dev)
out = eng.portfolio_multi(L, NR, nb, Ks=Ks, B=B, legs_only=True, workspace=ws)
torch.cuda.synchronize()
n_gen = int(ws[gen_b:gen_b + 4].view(torch.int32).item())
# host: leg counts per formation row, then the full rule per (t, b)
Lh = L.cpu().numpy().reshape(T_m, B, N)
ne = np.stack([(Lh == 9).any(axis=2), (Lh == 0).any(axis=2)], axis=-1)   # [T_m][B][2]
gen = np.zeros((T_m, B), dtype=bool)
for K in Ks:
    for t in range(T_m):
        j1 = [t - j for j in range(K)]
        j0 = [t - j for j in range(1, K + 1)]
        ok1 = all(s >= 0 for s in j1) and ne[[s for s in j1]].all(axis=0)
        ok0 = t >= 1 and all(s >= 0 for s in j0) and ne[[s for s in j0]].all(axis=0)
        full = np.logical_and(ok1, ok0) if not isinstance(ok1, bool) else np.zeros((B, 2), bool)
        if isinstance(ok0, bool):
            full = np.zeros((B, 2), bool)
        gen[t] |= ~full.all(axis=1)
print(f"rows {rows}  general-list count {n_gen}  host count {int(gen.sum())}  "
      f"first steady month per panel (min/max) {int((~gen).argmax(axis=0).min())}/{int((~gen).argmax(axis=0).max())}")
# time the call
for _ in range(2):
    eng.portfolio_multi(L, NR, nb, Ks=Ks, B=B, legs_only=True, workspace=ws)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    eng.portfolio_multi(L, NR, nb, Ks=Ks, B=B, legs_only=True, workspace=ws)
torch.cuda.synchronize()
print(f"portfolio_multi {1e3 * (time.perf_counter() - t0) / 5:.3f} ms per call")
