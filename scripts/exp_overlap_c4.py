"""C4 step pipelining experiment: step s's decile pass (+ long-short) on a second stream while
step s+1's signal runs, M / NR / ids double-buffered, against the serial steps the bench times.
Two engines (one csm context per stream).  Prints one JSON line with ms per step both ways
and whether the pipelined outputs equal the serial ones bit for bit.
Usage: exp_overlap_c4.py [N] [days] [steps]"""
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import csmom  # noqa: E402
from csmom.synth import make_device_panel, bday_calendar  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    T_d = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    dev = torch.device("cuda", 0)
    days, ms, _ = bday_calendar("1985-01-01", T_d)
    pan = make_device_panel(N, days, ms, seed=1000, device=dev)
    T_m = len(ms) - 1
    maxd = int(np.diff(ms).max())
    mind = int(np.diff(ms)[1:-1].min())
    J, skip, nb = 12, 1, 10
    ea, eb = csmom.Engine(0), csmom.Engine(0)
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    bufs = [dict(M=ea.empty((T_m, N)), NR=ea.empty((T_m, N)),
                 IDS=ea.empty((T_m, N), torch.int16)) for _ in range(2)]
    L = ea.empty((T_m, N), torch.int8)
    EW, CNT = ea.empty((T_m, nb)), ea.empty((T_m, nb), torch.int32)
    LS = ea.empty((T_m,))

    def signal(e, b):
        e.signal_ids(pan.P, pan.month_start, maxd, J, skip, out=(None, None, b["M"], b["NR"], b["IDS"]),
                     min_month_days=mind)

    def deciles(e, b):
        e.deciles_ids(b["M"], b["NR"], b["IDS"], nb, out=(L, EW, CNT, None), LS=LS)

    def serial(k):
        with torch.cuda.stream(sa):
            for _ in range(k):
                signal(ea, bufs[0])
                deciles(ea, bufs[0])

    done_sig = [torch.cuda.Event() for _ in range(2)]
    done_dec = [torch.cuda.Event() for _ in range(2)]

    def pipelined(k):
        for s in range(k):
            b = s % 2
            with torch.cuda.stream(sa):
                if s >= 2:
                    sa.wait_event(done_dec[b])   # buffer b's deciles (step s - 2) have read it
                signal(ea, bufs[b])
                done_sig[b].record(sa)
            with torch.cuda.stream(sb):
                sb.wait_event(done_sig[b])
                deciles(eb, bufs[b])
                done_dec[b].record(sb)
        torch.cuda.current_stream(dev).wait_stream(sa)
        torch.cuda.current_stream(dev).wait_stream(sb)

    res = {}
    for name, f in (("serial", serial), ("pipelined", pipelined), ("serial2", serial),
                    ("pipelined2", pipelined)):
        f(2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f(K)
        torch.cuda.synchronize()
        res[name] = 1e3 * (time.perf_counter() - t0) / K
        if name.startswith("serial"):
            ref = (LS.clone(), EW.clone(), L.clone())
        else:
            same = (torch.equal(LS.view(torch.int64), ref[0].view(torch.int64)) and
                    torch.equal(EW.view(torch.int64), ref[1].view(torch.int64)) and
                    torch.equal(L, ref[2]))
            res[name + "_bits_equal"] = bool(same)
    # stage times alone
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    with torch.cuda.stream(sa):
        ev[0].record(sa)
        signal(ea, bufs[0])
        ev[1].record(sa)
        deciles(ea, bufs[0])
        ev[2].record(sa)
    torch.cuda.synchronize()
    res["signal_ms"] = ev[0].elapsed_time(ev[1])
    res["deciles_ms"] = ev[1].elapsed_time(ev[2])
    res.update(N=N, T_d=T_d, T_m=T_m, steps=K)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
