"""C4 A/B: can the decile pass hide under the fused signal kernel when the two run on
DISJOINT compute units (CU-masked streams, hipExtStreamCreateWithCUMask)?  The decile kernel
ranks a previous pass's mom_J / next_ret / ids (independent data) on the masked side stream
while k_signal runs on the complementary CUs; compared with back-to-back launches and with
unmasked concurrency.  Interleaved, median of 5 rounds.  Dev tool: prints one JSON line."""
import ctypes
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
n_cu = torch.cuda.get_device_properties(0).multi_processor_count
hip = ctypes.CDLL("libamdhip64.so.7")   # the runtime torch already loaded (same soname)
hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                             ctypes.POINTER(ctypes.c_uint32)]


def masked_stream(cus):
    words = (n_cu + 31) // 32
    m = [0] * words
    for c in cus:
        m[c // 32] |= 1 << (c % 32)
    arr = (ctypes.c_uint32 * words)(*m)
    h = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), words, arr)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(h.value, device="cuda:0")


M, NR, IDS = eng.empty((T_m, N)), eng.empty((T_m, N)), eng.empty((T_m, N), torch.int16)
M2, NR2, IDS2 = eng.empty((T_m, N)), eng.empty((T_m, N)), eng.empty((T_m, N), torch.int16)
L = eng.empty((T_m, N), torch.int8)


def sig(Mx, NRx, IDx):
    eng.signal_ids(pan.P, pan.month_start, maxd, 12, 1, out=(None, None, Mx, NRx, IDx), min_month_days=mind)


def dec():
    eng.deciles_ids(M2, NR2, IDS2, 10, out=(L, torch.empty((T_m, 10), dtype=torch.float64, device="cuda:0")
                                            if False else eng.empty((T_m, 10)),
                                            eng.empty((T_m, 10), torch.int32), None))


sig(M2, NR2, IDS2)
torch.cuda.synchronize()
splits = {}
for k in (32, 60, 64):
    dec_cus = list(range(n_cu - k, n_cu))           # the last k logical CUs
    sig_cus = list(range(0, n_cu - k))
    splits[f"mask{k}"] = (masked_stream(sig_cus), masked_stream(dec_cus))
    # interleaved numbering: every (n_cu // k)-th CU to the deciles
    step = n_cu // k
    dec_i = list(range(0, n_cu, step))[:k]
    sig_i = [c for c in range(n_cu) if c not in set(dec_i)]
    splits[f"maskI{k}"] = (masked_stream(sig_i), masked_stream(dec_i))
plain_side = torch.cuda.Stream()
main = torch.cuda.current_stream()


def timed(fn):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(main); fn(); b.record(main); torch.cuda.synchronize()
    return a.elapsed_time(b)


def conc_on(s_sig, s_dec):
    def f():
        s_sig.wait_stream(main); s_dec.wait_stream(main)
        with torch.cuda.stream(s_sig):
            sig(M, NR, IDS)
        with torch.cuda.stream(s_dec):
            dec()
        main.wait_stream(s_sig); main.wait_stream(s_dec)
    return f


def sig_on(s_sig):
    def f():
        s_sig.wait_stream(main)
        with torch.cuda.stream(s_sig):
            sig(M, NR, IDS)
        main.wait_stream(s_sig)
    return f


def dec_on(s_dec):
    def f():
        s_dec.wait_stream(main)
        with torch.cuda.stream(s_dec):
            dec()
        main.wait_stream(s_dec)
    return f


var = {"sig": lambda: sig(M, NR, IDS), "dec": dec, "seq": lambda: (sig(M, NR, IDS), dec()),
       "conc_plain": conc_on(main, plain_side)}
for k, (a, b) in splits.items():
    var[f"sig_{k}"] = sig_on(a)
    var[f"dec_{k}"] = dec_on(b)
    var[f"conc_{k}"] = conc_on(a, b)
times = {k: [] for k in var}
for rnd in range(6):
    for k, f in var.items():
        t = timed(f)
        if rnd:
            times[k].append(t)
print(json.dumps({"n_cu": n_cu, "ms": {k: round(float(np.median(v)), 4) for k, v in times.items()}}), flush=True)
