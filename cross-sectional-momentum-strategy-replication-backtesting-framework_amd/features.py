"""Drop-in counterparts of src/features.py's monthly functions, backed by the HIP engine.

`compute_monthly_momentum_from_daily` keeps the reference signature and output frame
(src/features.py:5-57) but runs month-end aggregation and the ret/mom scan on the GPU.
`compute_monthly_turnover` (src/features.py:60-107) keeps the reference frame contract and
computes adv / turnover / the rolling mean with csm_turnover_features on the GPU (its result is
not consumed by the decile path, SURVEY.md 8(a) a5, but monthly_replication computes it as
run_demo.py:33 does).
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


def _shares_column(df, shares_info_map):
    """The `shares_outstanding` column of features.py:78-97 (a per-ticker lookup, with the
    int(market_cap / price) fallback per row), built as the reference's row-wise apply would
    build it so the column's dtype matches (int64 when every value is an int, else float)."""
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
    return pd.Series(list(so), index=df.index).infer_objects()


def _shares_arrays(tickers, shares_info_map):
    """Per-asset so / mcap for csm_turnover_features (NaN = not given; the kernel applies the
    same so-else-int(mcap / price) rule per row)."""
    N = len(tickers)
    so, mcap = np.full(N, np.nan), np.full(N, np.nan)
    if isinstance(shares_info_map, dict):
        for a, t in enumerate(tickers):
            info = shares_info_map.get(t, {})
            s = info.get("shares_outstanding")
            if s is not None and not pd.isna(s):
                so[a] = float(s)
            m = info.get("market_cap")
            if m is not None and m is not False:
                try:
                    mcap[a] = float(m)
                except (TypeError, ValueError):
                    mcap[a] = np.nan
    return so, mcap


def compute_monthly_turnover(monthly_df, shares_info_map=None, lookback_months=3, device=None):
    """src/features.py:60-107 with the arithmetic on the GPU (csm_turnover_features, rule T1).

    Same input and output frame as the reference: adv_est, shares_outstanding,
    turnover_monthly and turn_avg columns added to a copy.  The rolling mean runs over each
    ticker's rows in frame order (the reference's groupby-rolling), so the dense layout is
    [row rank within ticker][ticker]; lookback_months in [1, 48].
    """
    df = monthly_df.copy()
    df["monthly_volume"] = pd.to_numeric(
        df.get("monthly_volume", df.get("volume", np.nan)), errors="coerce").fillna(0)
    n = len(df)
    df["adv_est"] = df["monthly_volume"] / 21.0
    df["shares_outstanding"] = _shares_column(df, shares_info_map)
    if n == 0:
        df["turnover_monthly"] = np.array([], dtype=np.float64)
        df["turn_avg"] = np.array([], dtype=np.float64)
        return df
    codes, tickers = pd.factorize(df["ticker"], sort=False)
    rank = pd.Series(codes).groupby(codes).cumcount().to_numpy()
    T, N = int(rank.max()) + 1, len(tickers)
    eng = get_engine(device)
    PM = np.full((T, N), np.nan)
    PM.view(np.uint64)[...] = np.uint64(0x7FF4000000000001)    # ABSENT: ticker has no k-th row
    price = (pd.to_numeric(df["adj_close"], errors="coerce").to_numpy(dtype=np.float64)
             if "adj_close" in df.columns else np.full(n, np.nan))
    PM[rank, codes] = price
    VOL = np.zeros((T, N))
    VOL[rank, codes] = df["monthly_volume"].to_numpy(dtype=np.float64)
    so, mcap = _shares_arrays(list(tickers), shares_info_map)
    up = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(eng.device)
    ADV, SH, TURN, TAVG = eng.turnover_features(up(PM), up(VOL), up(so), up(mcap),
                                                int(lookback_months))
    df["adv_est"] = ADV.cpu().numpy()[rank, codes]
    df["turnover_monthly"] = TURN.cpu().numpy()[rank, codes]
    df["turn_avg"] = TAVG.cpu().numpy()[rank, codes]
    return df


__all__ = ["compute_monthly_momentum_from_daily", "compute_monthly_turnover", "get_engine",
           "MONTHLY_COLUMNS"]
