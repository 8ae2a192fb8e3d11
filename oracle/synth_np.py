"""Seeded synthetic daily panels on the host -- TEST INFRASTRUCTURE ONLY.

Conventions follow SURVEY.md section 8(d) / appendix B: GBM log-returns N(mu_a, sigma_a) with
mu_a ~ N(3e-4, 2e-4), sigma_a ~ U(0.01, 0.04), P0 = 100, integer lognormal(13, 1) volume,
business-day calendar, and a masking mix of late listings, early delistings, NaN days,
absent (asset, month) rows and all-NaN months.  Tickers are `S%06d` so lexicographic
order equals numeric order.  Used by the golden-fixture script, the GPU parity tests
(inputs are uploaded, the oracle checks the outputs) and bench.py's CPU baseline.
"""
from __future__ import annotations

import numpy as np
import pandas as pd

from .csmom_oracle import ABSENT_BITS


def calendar(T: int, start: str = "2000-01-03", monthly: bool = False):
    """Business days (or business month-ends) and month offsets.

    Returns (dates DatetimeIndex, month_start int64[T_m+1], month_end DatetimeIndex of
    calendar month-ends -- the labels pandas' `Grouper(freq='ME')` gives).
    """
    if monthly:
        days = pd.date_range(start, periods=T, freq="BME")
    else:
        days = pd.bdate_range(start, periods=T)
    key = np.asarray(days.year) * 12 + np.asarray(days.month)
    change = np.nonzero(np.diff(key))[0] + 1
    month_start = np.concatenate([[0], change, [T]]).astype(np.int64)
    # consecutive calendar months are assumed (true for business-day calendars)
    mends = days[month_start[:-1]] + pd.offsets.MonthEnd(0)
    return days, month_start, mends


def make_panel(N: int, T: int, seed: int, start: str = "2000-01-03", monthly: bool = False,
               late: float = 0.05, delist: float = 0.05, nan_day: float = 0.01,
               absent_month: float = 0.002, nan_month: float = 0.001,
               cents: bool = False, with_volume: bool = True) -> dict:
    rng = np.random.default_rng(seed)
    days, month_start, mends = calendar(T, start, monthly)
    T_m = len(month_start) - 1
    scale = 21.0 if monthly else 1.0
    mu = rng.normal(3e-4, 2e-4, N) * scale
    sig = rng.uniform(0.01, 0.04, N) * np.sqrt(scale)
    lr = rng.standard_normal((T, N)) * sig + mu
    P = 100.0 * np.exp(np.cumsum(lr, axis=0))
    if cents:
        P = np.round(P, 2)
    V = np.round(rng.lognormal(13.0, 1.0, (T, N))) if with_volume else None
    bits = P.view(np.uint64)
    absent = np.uint64(ABSENT_BITS)
    if late > 0:
        a = np.nonzero(rng.random(N) < late)[0]
        d = rng.integers(1, max(2, T // 2), len(a))
        for ai, di in zip(a, d):
            bits[:di, ai] = absent
    if delist > 0:
        a = np.nonzero(rng.random(N) < delist)[0]
        d = rng.integers(T // 2, T, len(a))
        for ai, di in zip(a, d):
            bits[di:, ai] = absent
    if nan_month > 0:
        mm, aa = np.nonzero(rng.random((T_m, N)) < nan_month)
        for m, a in zip(mm, aa):
            seg = bits[month_start[m]:month_start[m + 1], a]
            seg[seg != absent] = np.float64(np.nan).view(np.uint64)
    if absent_month > 0:
        mm, aa = np.nonzero(rng.random((T_m, N)) < absent_month)
        for m, a in zip(mm, aa):
            bits[month_start[m]:month_start[m + 1], a] = absent
    if nan_day > 0:
        nd = (rng.random((T, N)) < nan_day) & (bits != absent)
        P[nd] = np.nan
    tickers = np.array([f"S{i:06d}" for i in range(N)])
    return dict(P=P, V=V, days=days, month_start=month_start, month_end=mends,
                tickers=tickers)


def to_long(panel: dict) -> pd.DataFrame:
    """The reference's daily input: one row per present (date, ticker) cell, sorted by
    ticker then date (the per-ticker CSV concatenation order of `data_io.fetch_daily`)."""
    P = panel["P"]
    T, N = P.shape
    pres = (P.view(np.uint64) & np.uint64(0x7FF7FFFFFFFFFFFF)) != np.uint64(ABSENT_BITS)
    aa, dd = np.nonzero(pres.T)
    df = pd.DataFrame({
        "date": panel["days"][dd],
        "ticker": panel["tickers"][aa],
        "adj_close": P[dd, aa],
        "volume": panel["V"][dd, aa] if panel.get("V") is not None else np.zeros(len(dd)),
    })
    return df
