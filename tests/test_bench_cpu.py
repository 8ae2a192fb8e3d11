"""CPU: the bench's host plumbing -- the business-day calendar (pd.bdate_range on numpy days, so
weak-scaling calendars past pandas' Timestamp range work), the whole-month date shards of 2 / 4 /
8 ranks in both scaling modes, and `bench.py --gpus N`'s self-launch decision (the parent starts
the workers and never touches the GPU)."""
import sys
from pathlib import Path

import numpy as np
import pandas as pd
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


@pytest.mark.parametrize("start,n", [("1985-01-01", 10_000), ("2000-01-03", 6_522),
                                     ("1985-01-05", 1_100), ("2000-01-01", 1)])
def test_bday_calendar_is_pandas(start, n):
    from csmom.panel import month_offsets
    from csmom.synth import bday_calendar
    days, ms, mend = bday_calendar(start, n)
    ref = pd.bdate_range(start, periods=n)
    ms_r, mend_r = month_offsets(ref)
    assert days.equals(ref) and np.array_equal(ms, ms_r) and mend.equals(mend_r)


@pytest.mark.parametrize("G", [1, 2, 4, 8])
@pytest.mark.parametrize("scaling", ["strong", "weak"])
def test_shard_calendar_c4(G, scaling):
    """C4's calendar split over G ranks: strong = the fixed 10,000 bdays, weak = 10,000 per rank
    (8 ranks: 80,000 bdays from 1985, past 2262).  The shards are contiguous whole months that
    cover the calendar, and every rank agrees on the month counts."""
    from csmom.synth import bday_calendar, shard_calendar
    total = 10_000 * (G if scaling == "weak" else 1)
    days, ms, mend = bday_calendar("1985-01-01", total)
    T_m = len(ms) - 1
    got_days, parts = [], None
    for r in range(G):
        d, msl, me, months = shard_calendar("1985-01-01", total, G, r)
        parts = parts or months
        assert months == parts and sum(months) == T_m and len(msl) == months[r] + 1
        assert msl[0] == 0 and msl[-1] == len(d) and (np.diff(msl) > 0).all()
        got_days.append(np.asarray(d).astype("datetime64[D]"))
    assert np.array_equal(np.concatenate(got_days), np.asarray(days).astype("datetime64[D]"))
    assert max(parts) - min(parts) <= 1


def test_make_device_panel_past_pandas_range():
    """The weak-scaling 8-rank calendar's last shard (dates in the 2280s) builds a panel."""
    import torch
    from csmom.synth import make_device_panel, shard_calendar
    d, ms, _, _ = shard_calendar("1985-01-01", 80_000, 8, 7)
    assert np.asarray(d).astype("datetime64[D]")[-1] > np.datetime64("2262-04-11")
    k = 14                                      # its first 14 months
    pan = make_device_panel(8, d[:ms[k]], ms[:k + 1], seed=1, device="cpu",
                            shard=(7, 8, 4, 10_000.0))
    assert pan.P.shape[0] == ms[k] and pan.P.dtype == torch.float64
    assert len(pan.month_end) == len(pan.month_start_host) - 1


def test_gpus_n_self_launches(monkeypatch):
    """Without a torchrun environment `--gpus N > 1` hands the argv to spawn_workers (the parent
    imports no torch); with WORLD_SIZE set (a worker) it runs the bench itself."""
    import bench
    seen = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "spawn_workers", lambda argv: seen.append(argv) or 0)
    argv = ["--gpus", "8", "--steps", "5"]
    assert bench.main(argv) is None and seen == [argv]
    monkeypatch.setattr(bench, "spawn_workers", lambda argv: 3)
    with pytest.raises(SystemExit) as e:
        bench.main(argv)
    assert e.value.code == 3
    assert bench.parse([]).scaling == "strong" and bench.parse([]).gpus == 1
