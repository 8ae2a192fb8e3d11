"""C5-shaped momentum scan (a batch of 100 bootstrap panels: 300 months x 500k assets): plain vs
nontemporal output stores, interleaved.  Dev tool: one JSON line."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import csmom  # noqa: E402

T_m, N = 300, 500_000
eng = csmom.Engine(0)
g = torch.Generator(device="cuda:0").manual_seed(5)
R = torch.randn((T_m, N), dtype=torch.float64, device="cuda:0", generator=g) * 0.08
PM = 100.0 * torch.cumprod(1.0 + R, dim=0)
del R


def timed(fn):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); a.record(); fn(); b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b)


res, outs = {}, {}
for rnd in range(6):
    for st in (0, 1):
        eng.lib.csm_tune(b"momentum_store", st)
        t = timed(lambda: outs.__setitem__(st, eng.momentum(PM, 12, 1, chunked=False)))
        if rnd:
            res.setdefault(st, []).append(t)
eng.lib.csm_tune(b"momentum_store", 0)
same = all(torch.equal(torch.nan_to_num(a, 7.0), torch.nan_to_num(b, 7.0))
           for a, b in zip(outs[0], outs[1]) if a is not None)
print(json.dumps({"T_m": T_m, "N": N, "ms": {"plain": round(float(np.median(res[0])), 3),
                                               "nontemporal": round(float(np.median(res[1])), 3)},
                  "identical": same}), flush=True)
