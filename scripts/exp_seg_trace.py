"""rocprofv3 target: a few run_segmented passes (S from argv) on C4, nothing else timed."""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import csmom  # noqa: E402
from csmom.synth import bday_calendar, make_device_panel  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 4
N, TD = 100_000, 10_000
days, ms, _ = bday_calendar("1985-01-01", TD)
pan = make_device_panel(N, days, ms, seed=4, device="cuda:0")
eng = csmom.Engine(0)
plan = eng.segmented_plan(pan.P, ms, 12, 1, S)
for _ in range(4):
    out = eng.run_segmented(pan.P, pan.month_start, plan, 12, 1, 10)
torch.cuda.synchronize()
print("ok")
