"""CPU: the offline daily-CSV loader (src/data_io.py:23-73,131-180 rules) and the long -> dense
ingestion.  Pinned by the real-data fixture (made by the reference's own fetch_daily over its
cached CSVs): the loader must reproduce that dense panel bit for bit and drop AAPL (the
3-row-header file) exactly as the reference does.  The reference's data/ directory is read
only when it is present (this container); the GPU box never runs these tests."""
from pathlib import Path

import numpy as np
import pandas as pd
import pytest

from conftest import bits_equal, load_golden

REF_DATA = Path("/root/reference/data")
TICKERS = ["AAPL", "MSFT", "AMZN", "GOOGL", "NVDA", "TSLA", "META", "JPM", "BAC", "WMT", "PG",
           "KO", "DIS", "CSCO", "ORCL", "INTC", "AMD", "NFLX", "C", "GS"]  # run_demo.py:15-16


def test_normalize_quirks():
    import csmom.data as D
    # yfinance multi-row header: the ticker row becomes a NaT date (dropped later)
    raw = pd.DataFrame({"Date": ["", "2020-01-02"], "Adj Close": ["MSFT", "1.5"],
                        "Close": ["MSFT", "2.0"], "Volume": ["MSFT", "10"]})
    out = D.normalize_daily_columns(raw, "MSFT")
    assert list(out.columns) == D.DAILY_COLUMNS
    assert pd.isna(out["date"].iloc[0]) and out["adj_close"].iloc[1] == 1.5
    assert np.isnan(out["adj_close"].iloc[0]) and (out["ticker"] == "MSFT").all()
    # no 'Date' column -> every date NaT (the AAPL file)
    raw2 = pd.DataFrame({"Price": ["Ticker", "2020-01-02"], "Close": ["AAPL", "3.0"]})
    out2 = D.normalize_daily_columns(raw2, "AAPL")
    assert out2["date"].isna().all() and out2["adj_close"].iloc[1] == 3.0
    # duplicate columns keep the first; Close fills a missing Adj Close
    raw3 = pd.DataFrame([[1.0, 2.0, "2020-01-03"]], columns=["Close", "Close", "Date"])
    out3 = D.normalize_daily_columns(raw3, "X")
    assert out3["adj_close"].iloc[0] == 1.0 and out3["close"].iloc[0] == 1.0


def test_missing_file_is_skipped(tmp_path, capsys):
    import csmom.data as D
    (tmp_path / "OK_daily.csv").write_text("Date,Adj Close,Volume\n2020-01-02,5.0,7\n")
    df = D.fetch_daily(["NOPE", "OK"], data_dir=str(tmp_path))
    assert list(df["ticker"]) == ["OK"] and df["adj_close"].iloc[0] == 5.0
    assert "yfinance returned no data for NOPE" in capsys.readouterr().out


def test_reference_call_signature(tmp_path, monkeypatch, capsys):
    """run_demo.py:196 calls fetch_daily(tickers, start=..., end=..., verbose=True) with the
    cache in DATA_DIR (data_io.py:8); cached reads ignore start / end (data_io.py:149-151)."""
    import inspect
    import csmom.data as D
    params = list(inspect.signature(D.fetch_daily).parameters)
    assert params[:6] == ["tickers", "start", "end", "interval", "force_refresh", "verbose"]
    (tmp_path / "OK_daily.csv").write_text("Date,Adj Close,Volume\n2017-06-02,5.0,7\n"
                                           "2020-01-02,6.0,8\n")
    monkeypatch.setattr(D, "DATA_DIR", str(tmp_path))
    df = D.fetch_daily(["OK"], start="2018-01-01", end="2024-12-31", verbose=True)
    assert list(df["adj_close"]) == [5.0, 6.0]          # the 2017 row is kept, as in the reference
    assert "loaded OK rows=2" in capsys.readouterr().out
    assert D.fetch_daily(["OK"], force_refresh=True, verbose=False).empty   # would download
    assert list(D.fetch_daily([], verbose=False).columns) == D.DAILY_COLUMNS


@pytest.mark.skipif(not REF_DATA.exists(), reason="reference data/ not present")
def test_loader_reproduces_reference_panel():
    import csmom.data as D
    z = load_golden("real_data")
    panel = D.load_daily_panel(TICKERS, str(REF_DATA))
    assert list(panel.tickers) == list(z["tickers"])           # AAPL dropped, sorted
    assert np.array_equal(panel.days.asi8, z["day_ns"])
    assert np.array_equal(panel.month_start, z["month_start"])
    assert bits_equal(panel.P, z["P"]) and bits_equal(panel.V, z["V"])
    from oracle import csmom_oracle as O
    assert (O.is_absent(panel.P) == O.is_absent(z["P"])).all()
