"""A/B the k_signal layouts on C4 (row-major [T_d][N] vs asset-tiled [N/128][T_d][128]) and
month-buffer depths, interleaved in one process; checks the tiled outputs are bit-identical
to the row-major ones.  Dev tool: prints one JSON line."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import csmom  # noqa: E402
from csmom.synth import bday_calendar, make_device_panel  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
TD = 10_000
days, ms, _ = bday_calendar("1985-01-01", TD)
pan = make_device_panel(N, days, ms, seed=4, device="cuda:0")
eng = csmom.Engine(0)
T_m = len(ms) - 1
maxd = int(np.diff(ms).max())
M, NR = eng.empty((T_m, N)), eng.empty((T_m, N))
M2, NR2 = eng.empty((T_m, N)), eng.empty((T_m, N))
tune = lambda k, v: eng.lib.csm_tune(k.encode(), v)

e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
Pt = eng.tile_panel(pan.P)
e1.record()
torch.cuda.synchronize()
tile_ms = e0.elapsed_time(e1)


def timed(fn):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); fn(); b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b)


var = {("row", 3): [], ("row", 4): [], ("bw", 2): [], ("bw", 4): [], ("mw", 22): [],
       ("nostore", 4): []}
outs = {k: (eng.empty((T_m, N)), eng.empty((T_m, N))) for k in var if k[0] in ("mw", "bw")}
for rnd in range(6):
    for (lay, nb) in var:
        tune("signal_vec", 2); tune("signal_nbuf", nb if lay != "mw" else 4)
        tune("signal_mw", nb if lay == "mw" else 0)
        tune("signal_store", {"nt": 1, "nostore": 2}.get(lay, 0))
        tune("signal_bw", nb if lay == "bw" else 1)
        if lay == "mw":
            t = timed(lambda: eng.signal(pan.P, pan.month_start, maxd, 12, 1,
                                         out=(None, None) + outs[(lay, nb)]))
        elif lay == "bw":
            t = timed(lambda: eng.signal(pan.P, pan.month_start, maxd, 12, 1, out=(None, None) + outs[(lay, nb)]))
        elif lay in ("nt", "nostore"):
            t = timed(lambda: eng.signal(pan.P, pan.month_start, maxd, 12, 1, out=(None, None, M2, NR2)))
        elif lay == "row":
            t = timed(lambda: eng.signal(pan.P, pan.month_start, maxd, 12, 1, out=(None, None, M, NR)))
        else:
            t = timed(lambda: eng.signal_tiled(Pt, TD, N, pan.month_start, maxd, 12, 1,
                                               out=(None, None, M2, NR2)))
        if rnd:
            var[(lay, nb)].append(t)
tune("signal_nbuf", 4)
tune("signal_mw", 0)
tune("signal_bw", 1)
tune("signal_store", 1)
eng.signal(pan.P, pan.month_start, maxd, 12, 1, out=(None, None, M2, NR2))
tune("signal_store", 0)
torch.cuda.synchronize()
nt_same = bool(torch.equal(M.view(torch.int64), M2.view(torch.int64)) and
               torch.equal(NR.view(torch.int64), NR2.view(torch.int64)))
eq = lambda a, b: bool(torch.equal(a.view(torch.int64), b.view(torch.int64)))
mw_same = {f"{k[0]}{k[1]}": eq(M, v[0]) and eq(NR, v[1]) for k, v in outs.items()}
Pt2 = eng.signal_tiled(Pt, TD, N, pan.month_start, maxd, 12, 1, out=(None, None, M2, NR2))
torch.cuda.synchronize()
same = bool(torch.equal(M.view(torch.int64), M2.view(torch.int64)) and
            torch.equal(NR.view(torch.int64), NR2.view(torch.int64)))
alg = 8.0 * N * TD + 16.0 * N * T_m
res = {f"{l}_nbuf{b}": round(float(np.median(t)), 4) for (l, b), t in var.items()}
print(json.dumps({"N": N, "T_d": TD, "k_signal_ms": res,
                  "k_signal_GBps": {k: round(alg / (v * 1e-3) / 1e9, 1) for k, v in res.items()},
                  "tile_panel_ms": round(tile_ms, 3), "tiled_bits_equal_row": same,
                  "mw_bits_equal_row": mw_same, "nt_bits_equal_row": nt_same}), flush=True)
