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


# Module-level cache directory, as the reference's DATA_DIR (data_io.py:8); relative to the
# working directory like the reference's.  Unlike the reference, importing this module does
# not create it (a read-only cache is never written here: there is no network to fill it).
DATA_DIR = "data"


def cache_path(ticker: str, freq: str = "daily", data_dir: str | None = None) -> str:
    """data_io.py:11-12: `<DATA_DIR>/<ticker>_<freq>.csv` (data_dir overrides DATA_DIR)."""
    return os.path.join(DATA_DIR if data_dir is None else data_dir, f"{ticker}_{freq}.csv")


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


def fetch_daily(tickers, start=None, end=None, interval="1d", force_refresh=False, verbose=True,
                data_dir: str | None = None) -> pd.DataFrame:
    """Drop-in `fetch_daily` (src/data_io.py:131-180), cached CSVs only.

    Same signature and return value as the reference (data_dir is an extra keyword that
    overrides DATA_DIR).  Like the reference, a cached read ignores start / end / interval
    (data_io.py:149-151 reads the whole file).  A ticker without a cached file -- or every
    ticker when force_refresh=True -- would need yfinance (data_io.py:153); offline that is
    the reference's "yfinance returned no data" branch: a warning and the ticker is skipped.
    """
    parts = []
    for t in tickers:
        p = cache_path(t, "daily", data_dir)
        if force_refresh or not os.path.exists(p):
            if verbose:
                print(f"[fetch_daily] warning: yfinance returned no data for {t} "
                      f"(offline: no download of {start}..{end} at {interval})")
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


def load_daily_panel(tickers, data_dir: str | None = None, verbose: bool = False) -> DensePanel:
    """Cached CSVs straight to the dense [T_d][N] panel the engine uploads (ABSENT-encoded,
    tickers in lexicographic order, union business-day axis)."""
    return from_long(fetch_daily(tickers, verbose=verbose, data_dir=data_dir))


__all__ = ["DAILY_COLUMNS", "DATA_DIR", "cache_path", "normalize_daily_columns", "fetch_daily",
           "load_daily_panel"]
