"""Long <-> dense panel conversion (host side of the drop-in boundary).

The reference's functions take a long DataFrame of daily rows (date, ticker, adj_close,
volume, ...).  The engine works on a dense `[T_d][N]` float64 panel in HBM with assets in
lexicographic ticker order (the order pandas' groupby sorts to) and a business-day axis
that is the union of all dates.  Cells without a daily row carry the ABSENT NaN payload.

Column coercion follows src/features.py:15-31 exactly (date from 'date' or 'Date';
price from 'adj_close' > 'Adj Close' > 'close'; volume numeric with NaN -> 0).
"""
from __future__ import annotations

import warnings
from dataclasses import dataclass

import numpy as np
import pandas as pd

from ._lib import ABSENT_BITS

MONTHLY_COLUMNS = ["ticker", "date", "adj_close", "monthly_volume", "ret_1m", "mom_J"]


@dataclass
class DensePanel:
    P: np.ndarray            # [T_d][N] float64 prices, ABSENT / NaN encoded
    V: np.ndarray            # [T_d][N] float64 volume (0 where absent)
    days: pd.DatetimeIndex   # [T_d]
    tickers: np.ndarray      # [N] object, sorted
    month_start: np.ndarray  # [T_m+1] int64
    month_end: pd.DatetimeIndex  # [T_m] calendar month-end labels ('ME')

    @property
    def shape(self):
        return self.P.shape

    @property
    def T_m(self):
        return len(self.month_start) - 1


def month_offsets(days: pd.DatetimeIndex):
    """Offsets of each calendar month in a sorted day axis + its 'ME' label."""
    if len(days) == 0:
        return np.zeros(1, dtype=np.int64), pd.DatetimeIndex([])
    key = np.asarray(days.year, dtype=np.int64) * 12 + np.asarray(days.month, dtype=np.int64)
    change = np.nonzero(np.diff(key))[0] + 1
    ms = np.concatenate([[0], change, [len(days)]]).astype(np.int64)
    labels = (days[ms[:-1]] + pd.offsets.MonthEnd(0)).normalize()
    return ms, pd.DatetimeIndex(labels)


def _coerce(daily_df: pd.DataFrame):
    """features.py:15-31: returns (date, ticker, price, volume) arrays, NaT dates dropped."""
    date = pd.to_datetime(daily_df.get("date", daily_df.get("Date", None)), errors="coerce")
    if date is None:
        date = pd.Series(pd.NaT, index=daily_df.index)
    date = pd.Series(date, index=daily_df.index)
    if "adj_close" in daily_df.columns:
        price = pd.to_numeric(daily_df["adj_close"], errors="coerce")
    elif "Adj Close" in daily_df.columns:
        price = pd.to_numeric(daily_df["Adj Close"], errors="coerce")
    elif "close" in daily_df.columns:
        price = pd.to_numeric(daily_df["close"], errors="coerce")
    else:
        price = pd.Series(np.nan, index=daily_df.index)
    vol_src = daily_df.get("volume", daily_df.get("Volume", None))
    if vol_src is None:
        volume = pd.Series(0.0, index=daily_df.index)
    else:
        volume = pd.to_numeric(vol_src, errors="coerce").fillna(0)
    keep = date.notna().to_numpy()
    ticker = daily_df["ticker"].to_numpy()[keep]
    return (date.to_numpy()[keep], ticker, price.to_numpy(dtype=np.float64)[keep],
            volume.to_numpy(dtype=np.float64)[keep])


def from_long(daily_df: pd.DataFrame) -> DensePanel:
    """Pivot the reference's daily frame to the dense engine layout."""
    date, ticker, price, volume = _coerce(daily_df)
    if len(date) == 0:
        return DensePanel(np.empty((0, 0)), np.empty((0, 0)), pd.DatetimeIndex([]),
                          np.array([], dtype=object), np.zeros(1, dtype=np.int64),
                          pd.DatetimeIndex([]))
    dcode, days = pd.factorize(pd.DatetimeIndex(date).normalize(), sort=True)
    tcode, tickers = pd.factorize(pd.Series(ticker, dtype=object), sort=True)
    days = pd.DatetimeIndex(days)
    T_d, N = len(days), len(tickers)
    cell = tcode.astype(np.int64) * T_d + dcode
    # The reference takes the last non-NaN price per (ticker, month) in ROW order; the dense
    # layout walks days in date order.  They agree when each ticker's rows are date-sorted
    # and unique, which holds for every cached/downloaded frame; otherwise say so.
    order = np.argsort(cell, kind="stable")
    sorted_cell = cell[order]
    dup = sorted_cell[1:] == sorted_cell[:-1]
    if (np.diff(cell[np.argsort(tcode, kind="stable")]) < 0).any() or dup.any():
        warnings.warn("csmom: daily rows are not unique and date-ordered per ticker; the dense "
                      "pivot keeps the last non-NaN price per (ticker, date) and month-end "
                      "'last' is taken in date order", RuntimeWarning, stacklevel=3)
    P = np.full(T_d * N, ABSENT_BITS, dtype=np.uint64).view(np.float64)
    V = np.zeros(T_d * N)
    flat = dcode.astype(np.int64) * N + tcode
    if dup.any():
        # last non-NaN per cell in row order; volume summed in row order
        s = pd.DataFrame({"c": flat, "p": price, "v": volume})
        g = s.groupby("c", sort=False)
        lastp = g["p"].last()
        sumv = g["v"].sum()
        P[lastp.index.to_numpy()] = lastp.to_numpy()
        V[sumv.index.to_numpy()] = sumv.to_numpy()
    else:
        P[flat] = price
        V[flat] = volume
    ms, mend = month_offsets(days)
    return DensePanel(P.reshape(T_d, N), V.reshape(T_d, N), days,
                      np.asarray(tickers, dtype=object), ms, mend)


def monthly_frame(panel: DensePanel, PM: np.ndarray, VOL: np.ndarray, R: np.ndarray,
                  M: np.ndarray) -> pd.DataFrame:
    """The reference's monthly output (features.py:55): one row per present (ticker, month),
    sorted by (ticker, date), columns MONTHLY_COLUMNS."""
    if PM.size == 0:
        return pd.DataFrame({c: pd.Series(dtype=t) for c, t in zip(
            MONTHLY_COLUMNS, [object, "datetime64[ns]", float, float, float, float])})
    pres = (PM.view(np.uint64) & np.uint64(0x7FF7FFFFFFFFFFFF)) != np.uint64(ABSENT_BITS)
    aa, mm = np.nonzero(pres.T)
    return pd.DataFrame({
        "ticker": panel.tickers[aa],
        "date": panel.month_end[mm],
        "adj_close": PM[mm, aa],
        "monthly_volume": VOL[mm, aa],
        "ret_1m": R[mm, aa],
        "mom_J": M[mm, aa],
    })
