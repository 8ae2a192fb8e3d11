"""Diagnose one-process vs virtual-shard EW differences on the 20,000-asset rows (bucket ids)."""
import sys
from pathlib import Path
import numpy as np
import torch
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
import csmom
from csmom.distributed import virtual_shards
from oracle.synth_np import make_panel

eng = csmom.Engine(0)
pan = make_panel(20000, 1400, seed=29, start="1990-01-01", with_volume=False,
                 nan_day=0.02, absent_month=0.01, nan_month=0.005, cents=True)
ms = pan["month_start"].astype(np.int64)
Pd = torch.from_numpy(pan["P"]).to(eng.device)
msd = torch.from_numpy(ms).to(eng.device)
one = eng.pipeline(Pd, msd, 12, 1, 10)
one2 = eng.pipeline(Pd, msd, 12, 1, 10)
def bits(a):
    return a.cpu().numpy().view(np.uint64)
print("pipeline deterministic EW:", np.array_equal(bits(one.EW), bits(one2.EW)))
for G in (2, 5):
    M, NR, L, EW, CNT, LS = virtual_shards(eng, Pd, ms, G, 12, 1, 10, fused=True)
    e1, e2 = one.EW.cpu().numpy(), EW.cpu().numpy()
    same = (np.isnan(e1) == np.isnan(e2)) & ((e1 == e2) | np.isnan(e1))
    bad = np.where(~same.all(1))[0]
    print(f"G={G}: M eq {torch.equal(M.view(torch.int64), one.M.view(torch.int64))} L eq {torch.equal(L, one.L)} "
          f"EW rows differing {bad.tolist()[:20]} (of {len(bad)})")
    for t in bad[:3]:
        print("  row", t, e1[t], e2[t], "rel", np.nanmax(np.abs(e1[t] - e2[t]) / np.abs(e1[t])))
    # ids of one vs the re-derived ids through deciles_ids on the same M rows
    L2, EW2, CNT2, _ = eng.deciles(one.M, one.NR, 10)
    print("  streaming deciles vs pipeline rows differing:",
          int((~((EW2.cpu().numpy() == e1) | np.isnan(e1)).all(1)).sum()))
