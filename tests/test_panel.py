"""Host-side boundary: long DataFrame -> dense panel (features.py:15-31 coercion) and the
monthly output frame layout (features.py:55)."""
import numpy as np
import pandas as pd
import pytest

from conftest import bits_equal, load_golden
from oracle import csmom_oracle as O


def _long_from_fixture():
    z = load_golden("real_data")
    P, V = z["P"], z["V"]
    days = pd.DatetimeIndex(z["day_ns"])
    tick = z["tickers"]
    pres = ~O.is_absent(P)
    aa, dd = np.nonzero(pres.T)
    return pd.DataFrame({"date": days[dd], "ticker": tick[aa], "adj_close": P[dd, aa],
                         "volume": V[dd, aa]}), z


def test_from_long_roundtrip_real_data():
    import csmom
    df, z = _long_from_fixture()
    pan = csmom.from_long(df)
    assert list(pan.tickers) == list(z["tickers"])
    assert bits_equal(pan.P, z["P"])
    assert np.array_equal(pan.month_start, z["month_start"])
    assert pan.month_end.equals(pd.DatetimeIndex(z["month_end_ns"]))


def test_column_variants_and_nat_rows():
    import csmom
    df = pd.DataFrame({"Date": ["2020-01-02", "2020-01-03", "bad", "2020-02-03"],
                       "ticker": ["B", "A", "A", "A"], "close": ["10", "x", "3", "4.5"],
                       "Volume": [1, None, 3, 4]})
    pan = csmom.from_long(df)
    assert list(pan.tickers) == ["A", "B"]
    assert len(pan.days) == 3             # NaT row dropped
    assert np.isnan(pan.P[1, 0]) and not O.is_absent(pan.P[1:2, 0]).any()  # present, "x" -> NaN
    assert O.is_absent(pan.P[1:2, 1]).all()  # B has no row on 2020-01-03
    assert pan.P[0, 1] == 10.0 and pan.V[1, 0] == 0.0     # NaN volume -> 0
    assert list(pan.month_start) == [0, 2, 3]
    df2 = df.rename(columns={"close": "Adj Close"})
    assert bits_equal(csmom.from_long(df2).P, pan.P)


def test_duplicate_rows_warn():
    import csmom
    df = pd.DataFrame({"date": ["2020-01-02", "2020-01-02"], "ticker": ["A", "A"],
                       "adj_close": [1.0, np.nan], "volume": [1.0, 2.0]})
    with pytest.warns(RuntimeWarning):
        pan = csmom.from_long(df)
    assert pan.P[0, 0] == 1.0 and pan.V[0, 0] == 3.0


def test_monthly_frame_layout():
    import csmom
    df, z = _long_from_fixture()
    pan = csmom.from_long(df)
    PM, VOL = O.month_end(pan.P, pan.month_start, pan.V)
    R, M, _, _ = O.momentum_scan(PM, 12, 1)
    out = csmom.monthly_frame(pan, PM, VOL, R, M)
    assert list(out.columns) == ["ticker", "date", "adj_close", "monthly_volume", "ret_1m", "mom_J"]
    assert len(out) == int(z["J12s1_present"].sum())
    assert out["date"].dtype == "datetime64[ns]"
    assert (out.groupby("ticker")["date"].apply(lambda s: s.is_monotonic_increasing)).all()


def _turnover_case():
    m = pd.DataFrame({"ticker": ["A"] * 4 + ["B"] * 2,
                      "date": pd.to_datetime(["2020-01-31", "2020-02-29", "2020-03-31",
                                              "2020-04-30", "2020-01-31", "2020-02-29"]),
                      "adj_close": [10.0, np.nan, 20.0, 0.0, 5.0, 5.0],
                      "monthly_volume": [2100.0, 4200.0, 0.0, 21.0, 2100.0, np.nan]})
    info = {"A": {"market_cap": 1000}, "B": {"shares_outstanding": 50}}
    return m, info


def test_turnover_shares_column_host_rules():
    """The shares_outstanding lookup of features.py:78-97 (host: a per-ticker dict lookup with
    the int(market_cap / price) fallback); the arithmetic columns are the GPU kernel's."""
    from csmom.features import _shares_arrays, _shares_column
    m, info = _turnover_case()
    so = _shares_column(m, info).to_numpy(dtype=float)
    assert so[0] == 100 and np.isnan(so[1]) and so[2] == 50 and np.isnan(so[3])
    assert so[4] == 50 and so[5] == 50
    a, b = _shares_arrays(["A", "B", "C"], info)
    assert np.isnan(a[0]) and a[1] == 50 and np.isnan(a[2])
    assert b[0] == 1000 and np.isnan(b[1]) and np.isnan(b[2])


@pytest.mark.gpu
def test_turnover_matches_reference_rules_gpu():
    import csmom
    m, info = _turnover_case()
    out = csmom.compute_monthly_turnover(m, info, 3)
    assert list(out["adv_est"]) == [100.0, 200.0, 0.0, 1.0, 100.0, 0.0]
    so = out["shares_outstanding"].to_numpy(dtype=float)
    assert so[0] == 100 and np.isnan(so[1]) and so[2] == 50 and np.isnan(so[3])
    assert so[4] == 50 and so[5] == 50
    assert out["turnover_monthly"].iloc[0] == 1.0
    assert abs(out["turn_avg"].iloc[2] - 0.5) < 1e-15
