"""Phase stamps of k_signal_tc (build with EXTRA_FLAGS=-DTC_TIMING into ab/libcsmom_tct.so and
run with CSMOM_LIB=ab/libcsmom_tct.so): per workgroup the wall-clock (100 MHz) times of month-end
done, record published, earlier chunks' records acquired, fold done, scan done, relative to the
earliest workgroup start.  Prints per-chunk medians (us) as JSON.  Usage: exp_tc_phases.py [C]"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import csmom  # noqa: E402
from csmom.synth import make_device_panel  # noqa: E402


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    dev = torch.device("cuda", 0)
    eng = csmom.Engine(0)
    N, days = 5_000, 6_522
    from csmom.synth import shard_calendar
    d, ms_host, _, _ = shard_calendar("2000-01-03", days, 1, 0)
    pan = make_device_panel(N, d, ms_host, seed=4000, device=dev)
    T_m = len(ms_host) - 1
    C = C or eng.default_chunks(T_m, N, 12, 1)
    maxd = int(np.diff(ms_host).max())
    ws = None
    for _ in range(5):
        _, _, _, _, ws = eng.signal_chunked(pan.P, pan.month_start, maxd, 12, 1, chunks=C,
                                            workspace=ws)
    torch.cuda.synchronize()
    nbx = (N + 255) // 256
    W = 13
    SR = 6 + W + 1 + 1
    sync_b = ((4 + C * nbx) * 4 + 255) // 256 * 256
    off = sync_b + C * nbx * SR * 256 * 8
    st = ws[off:off + C * nbx * 64].view(torch.int64).view(C * nbx, 8).cpu().numpy()
    t0 = st[:, 0].min()
    rel = (st[:, :6] - t0) / 100.0   # us
    g = st[:, 6]
    out = {"C": C, "workgroups": int(C * nbx),
           "kernel_span_us": float(rel[:, 5].max()),
           "start_spread_us": float(rel[:, 0].max())}
    names = ["start", "monthend", "published", "acquired", "folded", "scanned"]
    per = {}
    for c in range(C):
        r = rel[g == c]
        per[c] = {n: round(float(np.median(r[:, k])), 2) for k, n in enumerate(names)}
    out["per_chunk_median_us"] = per
    print(json.dumps(out))


if __name__ == "__main__":
    main()
