"""Cached daily CSVs -> the long frame -> the dense HBM panel.

`fetch_daily` keeps the reference's cache contract (src/data_io.py:131-180): one
`<ticker>_daily.csv` per ticker under `data_dir`, read with `pd.read_csv(low_memory=False)`,
normalised to the canonical lower-case schema, rows with unparseable dates dropped, tickers
with no valid row skipped with a warning.  There is no network: a ticker without a cached file
is skipped as if yfinance had returned nothing (data_io.py:153-157).

Normalisation quirks kept on purpose (data_io.py:23-73), because they decide which rows reach
the momentum path:
  * duplicate column names keep the first occurrence;
  * 'Adj Close' is copied from 'Close' when missing;
  * a missing 'Date' column makes every date NaT, so the whole file is dropped -- this is why
    the 3-row-header `AAPL_daily.csv` (first column 'Price') never reaches the replication;
  * the yfinance ticker row (',MSFT,MSFT,...') parses to a NaT date and is dropped; numeric
    columns are coerced with errors='coerce'.
"""
from __future__ import annotations

import os

import numpy as np
import pandas as pd

from .panel import DensePanel, from_long

DAILY_COLUMNS = ["date", "ticker", "open", "high", "low", "close", "adj_close", "volume"]
_RENAME = {"Date": "date", "Ticker": "ticker", "Open": "open", "High": "high", "Low": "low",
           "Close": "close", "Adj Close": "adj_close", "Volume": "volume"}


def cache_path(data_dir: str, ticker: str, freq: str = "daily") -> str:
    return os.path.join(data_dir, f"{ticker}_{freq}.csv")


def normalize_daily_columns(df: pd.DataFrame, ticker: str) -> pd.DataFrame:
    """Canonical daily schema, the rules of src/data_io.py:23-73."""
    df = pd.DataFrame(df)
    if df.columns.duplicated().any():
        df = df.loc[:, ~df.columns.duplicated()]
    if "Adj Close" not in df.columns and "Close" in df.columns:
        df["Adj Close"] = df["Close"]
    if "Ticker" not in df.columns and "ticker" not in df.columns:
        df["Ticker"] = ticker
    df = df.rename(columns={k: v for k, v in _RENAME.items() if k in df.columns})
    df["date"] = pd.to_datetime(df["date"], errors="coerce") if "date" in df.columns else pd.NaT
    for col in ("open", "high", "low", "close", "adj_close", "volume"):
        df[col] = pd.to_numeric(df[col], errors="coerce") if col in df.columns else np.nan
    for col in DAILY_COLUMNS:
        if col not in df.columns:
            df[col] = np.nan
    return df[DAILY_COLUMNS].copy()


def fetch_daily(tickers, data_dir: str = "data", verbose: bool = True) -> pd.DataFrame:
    """Offline `fetch_daily` (src/data_io.py:131-180): cached CSVs only."""
    parts = []
    for t in tickers:
        p = cache_path(data_dir, t, "daily")
        if not os.path.exists(p):
            if verbose:
                print(f"[fetch_daily] warning: no cached data for {t} (offline)")
            continue
        try:
            df = normalize_daily_columns(pd.read_csv(p, low_memory=False), t)
            df = df.dropna(subset=["date"])
            if df.shape[0] == 0:
                if verbose:
                    print(f"[fetch_daily] warning: after normalization no valid rows for {t}")
                continue
            parts.append(df)
            if verbose:
                print(f"[fetch_daily] loaded {t} rows={len(df)}")
        except Exception as e:  # data_io.py:176-178: a bad file skips the ticker
            print(f"[fetch_daily] error loading {t}: {e!r} -- skipping ticker.")
    if not parts:
        return pd.DataFrame(columns=DAILY_COLUMNS)
    return pd.concat(parts, ignore_index=True)


def load_daily_panel(tickers, data_dir: str = "data", verbose: bool = False) -> DensePanel:
    """Cached CSVs straight to the dense [T_d][N] panel the engine uploads (ABSENT-encoded,
    tickers in lexicographic order, union business-day axis)."""
    return from_long(fetch_daily(tickers, data_dir, verbose))


__all__ = ["DAILY_COLUMNS", "cache_path", "normalize_daily_columns", "fetch_daily",
           "load_daily_panel"]
