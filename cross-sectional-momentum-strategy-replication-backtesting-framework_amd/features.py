"""Drop-in counterparts of src/features.py's monthly functions, backed by the HIP engine.

`compute_monthly_momentum_from_daily` keeps the reference signature and output frame
(src/features.py:5-57) but runs month-end aggregation and the ret/mom scan on the GPU.
`compute_monthly_turnover` (src/features.py:60-107) is host-side pandas: its result is never
used by the momentum path, so it is kept for API completeness only.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch

from .engine import Engine
from .panel import MONTHLY_COLUMNS, DensePanel, from_long, monthly_frame

_ENGINES: dict[int, Engine] = {}


def get_engine(device=None) -> Engine:
    idx = torch.cuda.current_device() if device is None else torch.device(
        "cuda", device).index if isinstance(device, int) else torch.device(device).index
    eng = _ENGINES.get(idx)
    if eng is None:
        eng = Engine(idx)
        _ENGINES[idx] = eng
    return eng


def upload_panel(panel: DensePanel, eng: Engine, with_volume: bool = True):
    dev = eng.device
    P = torch.from_numpy(np.ascontiguousarray(panel.P)).to(dev)
    V = torch.from_numpy(np.ascontiguousarray(panel.V)).to(dev) if with_volume else None
    ms = torch.from_numpy(panel.month_start.astype(np.int64)).to(dev)
    return P, V, ms


def monthly_signal(daily_df, lookback_months=12, skip_months=1, device=None):
    """Run month-end + scan on the GPU; returns (panel, host dict of dense arrays, device
    tensors) for callers that continue on the device."""
    panel = from_long(daily_df)
    if panel.P.size == 0 or panel.T_m == 0:
        return panel, None, None
    eng = get_engine(device)
    P, V, ms = upload_panel(panel, eng)
    PM, VOL = eng.month_end(P, ms, V)
    R, M, NR = eng.momentum(PM, lookback_months, skip_months, with_ret=True)
    dev = dict(PM=PM, VOL=VOL, R=R, M=M, NR=NR)
    host = {k: v.cpu().numpy() for k, v in dev.items()}
    return panel, host, dev


def compute_monthly_momentum_from_daily(daily_df, lookback_months=12, skip_months=1,
                                        device=None):
    """src/features.py:5-57 on the GPU.

    Returns DataFrame ['ticker','date','adj_close','monthly_volume','ret_1m','mom_J'], one
    row per (ticker, calendar month) with at least one daily row, sorted by (ticker, date).
    """
    panel, host, _ = monthly_signal(daily_df, lookback_months, skip_months, device)
    if host is None:
        return monthly_frame(panel, np.empty((0, 0)), None, None, None)
    return monthly_frame(panel, host["PM"], host["VOL"], host["R"], host["M"])


def compute_monthly_turnover(monthly_df, shares_info_map=None, lookback_months=3):
    """src/features.py:60-107 (host pandas; the momentum path never consumes it)."""
    df = monthly_df.copy()
    df["monthly_volume"] = pd.to_numeric(
        df.get("monthly_volume", df.get("volume", np.nan)), errors="coerce").fillna(0)
    df["adv_est"] = df["monthly_volume"] / 21.0
    n = len(df)
    so = np.full(n, np.nan, dtype=object)
    if isinstance(shares_info_map, dict) and n:
        tick = df["ticker"].to_numpy()
        price = df["adj_close"].to_numpy() if "adj_close" in df.columns else np.full(n, np.nan)
        for t in pd.unique(tick):
            info = shares_info_map.get(t, {})
            rows = np.nonzero(tick == t)[0]
            s = info.get("shares_outstanding")
            if s is not None and not pd.isna(s):
                so[rows] = s
                continue
            mcap = info.get("market_cap")
            for r in rows:  # features.py:90-96: int(mcap / price) when mcap and price > 0
                p = price[r]
                if mcap and p and p > 0:
                    try:
                        so[r] = int(mcap / p)
                    except Exception:
                        so[r] = np.nan
    df["shares_outstanding"] = pd.Series(list(so), index=df.index).infer_objects()
    sov = pd.to_numeric(df["shares_outstanding"], errors="coerce")
    with np.errstate(invalid="ignore", divide="ignore"):
        df["turnover_monthly"] = np.where(sov > 0, df["adv_est"] / sov, np.nan)
    df["turn_avg"] = (df.groupby("ticker")["turnover_monthly"]
                      .rolling(lookback_months, min_periods=1).mean()
                      .reset_index(level=0, drop=True))
    return df


__all__ = ["compute_monthly_momentum_from_daily", "compute_monthly_turnover", "get_engine",
           "MONTHLY_COLUMNS"]
