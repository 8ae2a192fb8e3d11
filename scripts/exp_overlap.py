"""C4 A/B: is the decile pass hidden if it runs CONCURRENTLY with the fused signal kernel?
The decile kernel ranks a previous pass's mom_J / next_ret / ids (independent data) on a side
stream while k_signal runs on the main stream; compared with back-to-back launches.
Interleaved, median of 5 rounds.  Dev tool: prints one JSON line."""
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
mind = int(np.diff(ms)[1:-1].min())
tune = lambda k, v: eng.lib.csm_tune(k.encode(), v)
bwf = [int(a) for a in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["1", "4"])]
M, NR, IDS = eng.empty((T_m, N)), eng.empty((T_m, N)), eng.empty((T_m, N), torch.int16)
M2, NR2, IDS2 = eng.empty((T_m, N)), eng.empty((T_m, N)), eng.empty((T_m, N), torch.int16)
L = eng.empty((T_m, N), torch.int8)
EW, CNT = eng.empty((T_m, 10)), eng.empty((T_m, 10), torch.int32)
main = torch.cuda.current_stream()
side = torch.cuda.Stream()


def sig(Mx, NRx, IDx):
    eng.signal_ids(pan.P, pan.month_start, maxd, 12, 1, out=(None, None, Mx, NRx, IDx), min_month_days=mind)


def dec():
    eng.deciles_ids(M2, NR2, IDS2, 10, out=(L, EW, CNT, None))


tune("signal_nbuf", 2)
tune("signal_bwf", 4)
sig(M2, NR2, IDS2)
torch.cuda.synchronize()


def seq():
    sig(M, NR, IDS)
    dec()


def conc():
    side.wait_stream(main)
    sig(M, NR, IDS)
    with torch.cuda.stream(side):
        dec()
    main.wait_stream(side)


def timed(fn):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(); fn(); b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b)


var = {}
for w in bwf:
    nb = 2 if w > 1 else 4
    def mk(f, w=w, nb=nb):
        def g():
            tune("signal_nbuf", nb); tune("signal_bwf", w)
            return timed(f)
        return g
    var[f"sig_bwf{w}"] = mk(lambda: sig(M, NR, IDS))
    var[f"seq_bwf{w}"] = mk(seq)
    var[f"conc_bwf{w}"] = mk(conc)
var["dec"] = lambda: timed(dec)
times = {k: [] for k in var}
for rnd in range(6):
    for k, f in var.items():
        t = f()
        if rnd:
            times[k].append(t)
tune("signal_nbuf", 4); tune("signal_bwf", 1)
print(json.dumps({"ms": {k: round(float(np.median(v)), 4) for k, v in times.items()},
                  "spread": {k: round(float(np.max(v) - np.min(v)), 4) for k, v in times.items()}}), flush=True)
