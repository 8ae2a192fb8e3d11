"""A/B the k_signal variants and k_deciles pass ablations on C4, interleaved in one process
(MI355X methodology rule 24).  Ablation timings come from builds of the same kernel that skip
work: their outputs are wrong by design and are never checked here."""
import json, sys, ctypes
from pathlib import Path
import numpy as np
import torch
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import csmom
from csmom.synth import bday_calendar, make_device_panel

N, TD = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000, 10_000
days, ms, _ = bday_calendar("1985-01-01", TD)
pan = make_device_panel(N, days, ms, seed=4, device="cuda:0")
eng = csmom.Engine(0)
T_m = len(ms) - 1
maxd = int(np.diff(ms).max())
M, NR = eng.empty((T_m, N)), eng.empty((T_m, N))
L = eng.empty((T_m, N), torch.int8)
EW, CNT = eng.empty((T_m, 10)), eng.empty((T_m, 10), torch.int32)
tune = lambda k, v: eng.lib.csm_tune(k.encode(), v)

def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); fn(); e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1)

sig = {(v, b): [] for v in (1, 2) for b in (3, 4)}
for rnd in range(5):
    for (v, b) in sig:
        tune("signal_vec", v); tune("signal_nbuf", b)
        t = timed(lambda: eng.signal(pan.P, pan.month_start, maxd, 12, 1, out=(None, None, M, NR)))
        if rnd:
            sig[(v, b)].append(t)
tune("signal_vec", 2); tune("signal_nbuf", 3)
eng.signal(pan.P, pan.month_start, maxd, 12, 1, out=(None, None, M, NR))
print(json.dumps({'k_signal_ms': {f'vec{v}_nbuf{b}': round(float(np.median(t)), 4) for (v, b), t in sig.items()}}), flush=True)
abl = {a: [] for a in (0, 1, 2, 4, 1 | 2 | 4, 8, 1 | 2 | 4 | 8)}
for rnd in range(5):
    for a in abl:
        tune("dec_ablate", a)
        t = timed(lambda: eng.deciles(M, NR, 10, out=(L, EW, CNT, None)))
        if rnd:
            abl[a].append(t)
tune("dec_ablate", 0)
out = {"N": N, "T_d": TD,
       "k_signal_ms": {f"vec{v}_nbuf{b}": round(float(np.median(t)), 4) for (v, b), t in sig.items()},
       "k_deciles_ms": {f"ablate{a}": round(float(np.median(t)), 4) for a, t in abl.items()},
       "ablate_bits": "1 no accumulate, 2 no gather pass, 4 no label pass, 8 no histogram atomics"}
print(json.dumps(out))
