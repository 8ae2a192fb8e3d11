"""Generate the golden fixtures by running the REFERENCE itself (run once, in the build
container; the reference never travels to the GPU box).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--only-turnover]

* The reference is imported from /root/reference with a `yfinance` stub (the network is
  never touched) and executed from a scratch working directory with plotting disabled, so
  nothing is written under /root/reference.
* Each case stores its dense inputs and the reference's outputs as `.npz` data.  The step
  sequence of `monthly_replication` (run_demo.py:32-67) is driven through the reference's
  own functions so that the intermediates (labels, next_ret, decile means) can be kept;
  for J=12/skip=1 cases `monthly_replication` itself is also run and its printed mean and
  Sharpe are recorded as a cross-check.
* Versions pinned: pandas 2.3.3, NumPy 2.2.6 (recorded in every fixture).
"""
from __future__ import annotations

import contextlib
import hashlib
import io
import os
import sys
import tempfile
import types
from pathlib import Path

import numpy as np
import pandas as pd

REPO = Path(__file__).resolve().parents[2]
REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

from oracle.csmom_oracle import ABSENT_BITS, absent_like  # noqa: E402
from oracle.synth_np import calendar, make_panel, to_long  # noqa: E402


def load_reference():
    yf = types.ModuleType("yfinance")

    def _offline(*a, **k):
        raise RuntimeError("yfinance disabled: no network")

    yf.download = _offline
    yf.Ticker = _offline
    sys.modules["yfinance"] = yf
    scratch = tempfile.mkdtemp(prefix="csmom_ref_")
    os.chdir(scratch)  # run_demo/data_io create results/ and data/ relative to cwd
    import matplotlib
    matplotlib.use("Agg")
    sys.path.insert(0, str(REF))
    import run_demo  # noqa: E402
    from src import data_io, features, utils  # noqa: E402
    run_demo.RESULTS = scratch
    run_demo.save_plot = lambda fig, path: __import__("matplotlib.pyplot").pyplot.close(fig)
    return run_demo, data_io, features, utils


def replication_steps(rd, feats, utils, daily_df, shares_info, J, skip, n_bins=10):
    """run_demo.py:32-67 through the reference's own functions, keeping intermediates."""
    monthly = feats.compute_monthly_momentum_from_daily(daily_df, lookback_months=J, skip_months=skip)
    monthly = feats.compute_monthly_turnover(monthly, shares_info_map=shares_info, lookback_months=3)
    df = monthly.dropna(subset=["mom_J"]).copy()
    df["decile"] = df.groupby("date")["mom_J"].transform(
        lambda s: rd.assign_deciles_per_date(s, n=n_bins))
    df["next_ret"] = df.groupby("ticker")["adj_close"].pct_change().shift(-1)
    kept = df.dropna(subset=["next_ret", "decile"])
    ew = kept.groupby(["date", "decile"])["next_ret"].mean().unstack(level="decile")
    if (n_bins - 1) in ew.columns and 0 in ew.columns:
        mom_ret = ew[n_bins - 1] - ew[0]
    else:
        mom_ret = ew.max(axis=1) - ew.min(axis=1)
    mom_ret = mom_ret.dropna()
    return monthly, df, ew, mom_ret


def to_dense(frame, col, tix, mix, T_m, N, fill=np.nan, dtype=np.float64):
    out = np.full((T_m, N), fill, dtype=dtype)
    a = frame["ticker"].map(tix).to_numpy()
    m = frame["date"].map(mix).to_numpy()
    out[m, a] = frame[col].to_numpy()
    return out


def _digest(a):
    return np.array(hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest())


def run_case(name, rd, feats, utils, P, V, days, month_start, month_end, tickers,
             configs, full=True):
    """full=False keeps the large per-cell outputs as sha256 digests plus a seeded sample
    of cells (the C1 fixture would otherwise be ~20 MB)."""
    T_m = len(month_start) - 1
    N = P.shape[1]
    tix = {t: i for i, t in enumerate(tickers)}
    mix = {d: i for i, d in enumerate(month_end)}
    daily = to_long(dict(P=P, V=V, days=days, tickers=tickers))
    shares = {t: {} for t in tickers}
    arrays = dict(P=P, day_ns=days.asi8, month_start=month_start,
                  month_end_ns=month_end.asi8, tickers=tickers.astype("U"),
                  pandas_version=np.array(pd.__version__), numpy_version=np.array(np.__version__))
    if V is not None:
        arrays["V"] = V
    for (J, skip) in configs:
        tag = f"J{J}s{skip}"
        monthly, df, ew, mom_ret = replication_steps(rd, feats, utils, daily, shares, J, skip)
        assert monthly["date"].isin(mix).all(), "month-end label outside calendar"
        pm = to_dense(monthly, "adj_close", tix, mix, T_m, N, fill=np.nan)
        present = to_dense(monthly.assign(one=1), "one", tix, mix, T_m, N, fill=0, dtype=np.int8)
        pm[present == 0] = absent_like(1)[0]
        big = {"M": to_dense(monthly, "mom_J", tix, mix, T_m, N)}
        if "PM" not in arrays and "PM_sha256" not in arrays:  # J-independent outputs once
            big["PM"] = pm
            big["R"] = to_dense(monthly, "ret_1m", tix, mix, T_m, N)
            if V is not None:
                big["VOL"] = to_dense(monthly, "monthly_volume", tix, mix, T_m, N, fill=0.0)
            arrays["present"] = present
        lab = to_dense(df, "decile", tix, mix, T_m, N)
        arrays[f"{tag}_L"] = np.where(np.isnan(lab), -1, lab).astype(np.int8)
        big["NR"] = to_dense(df, "next_ret", tix, mix, T_m, N)
        rs = np.random.default_rng(99)
        sample = rs.choice(T_m * N, size=min(T_m * N, 4000), replace=False)
        for k, v in big.items():
            key = k if k in ("PM", "R", "VOL") else f"{tag}_{k}"
            if full:
                arrays[key] = v
            else:
                arrays[key + "_sha256"] = _digest(v)
                arrays[key + "_sample"] = v.reshape(-1)[sample]
                arrays["sample_idx"] = sample
        ew_d = np.full((T_m, 10), np.nan)
        for d in ew.columns:
            ew_d[[mix[x] for x in ew.index], int(d)] = ew[d].to_numpy()
        arrays[f"{tag}_EW"] = ew_d
        ls = np.full(T_m, np.nan)
        ls[[mix[x] for x in mom_ret.index]] = mom_ret.to_numpy()
        arrays[f"{tag}_LS"] = ls
        arrays[f"{tag}_mean"] = np.float64(mom_ret.mean()) if len(mom_ret) else np.nan
        arrays[f"{tag}_sharpe"] = np.float64(utils.sharpe(mom_ret.values, freq_per_year=12))
        arrays[f"{tag}_cum"] = (1 + mom_ret).cumprod().to_numpy()
        if (J, skip) == (12, 1):
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                rd.monthly_replication(daily, shares)
            arrays["printed"] = np.array(buf.getvalue())
        print(f"  {name} {tag}: rows={len(monthly)} ranked={len(df)} months={len(mom_ret)} "
              f"mean={arrays[f'{tag}_mean']!r}")
    np.savez_compressed(OUT / f"{name}.npz", **arrays)


def real_data_case(rd, data_io, feats, utils):
    data_io.DATA_DIR = str(REF / "data")  # read-only use of the cached CSVs
    daily = data_io.fetch_daily(rd.DEFAULT_TICKERS, start="2018-01-01", end="2024-12-31",
                                verbose=False)
    tickers = np.array(sorted(daily["ticker"].unique()))
    days = pd.DatetimeIndex(sorted(daily["date"].unique()))
    key = np.asarray(days.year) * 12 + np.asarray(days.month)
    change = np.nonzero(np.diff(key))[0] + 1
    month_start = np.concatenate([[0], change, [len(days)]]).astype(np.int64)
    month_end = days[month_start[:-1]] + pd.offsets.MonthEnd(0)
    T, N = len(days), len(tickers)
    P = absent_like((T, N))
    V = np.zeros((T, N))
    di = {d: i for i, d in enumerate(days)}
    ti = {t: i for i, t in enumerate(tickers)}
    r = daily["date"].map(di).to_numpy()
    c = daily["ticker"].map(ti).to_numpy()
    assert not pd.DataFrame({"r": r, "c": c}).duplicated().any()
    P[r, c] = daily["adj_close"].to_numpy()
    V[r, c] = pd.to_numeric(daily["volume"], errors="coerce").fillna(0).to_numpy()
    # feed the frame exactly as fetch_daily returned it (row order matters for `last`)
    T_m = len(month_start) - 1
    tix = {t: i for i, t in enumerate(tickers)}
    mix = {d: i for i, d in enumerate(month_end)}
    shares = {t: {} for t in rd.DEFAULT_TICKERS}
    monthly, df, ew, mom_ret = replication_steps(rd, feats, utils, daily, shares, 12, 1)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        rd.monthly_replication(daily, shares)
    pm = to_dense(monthly, "adj_close", tix, mix, T_m, N)
    present = to_dense(monthly.assign(one=1), "one", tix, mix, T_m, N, fill=0, dtype=np.int8)
    pm[present == 0] = absent_like(1)[0]
    lab = to_dense(df, "decile", tix, mix, T_m, N)
    ls = np.full(T_m, np.nan)
    ls[[mix[x] for x in mom_ret.index]] = mom_ret.to_numpy()
    ew_d = np.full((T_m, 10), np.nan)
    for d in ew.columns:
        ew_d[[mix[x] for x in ew.index], int(d)] = ew[d].to_numpy()
    cum = (1 + mom_ret).cumprod()
    np.savez_compressed(
        OUT / "real_data.npz", P=P, V=V, day_ns=days.asi8, month_start=month_start,
        month_end_ns=month_end.asi8, tickers=tickers.astype("U"),
        J12s1_PM=pm, J12s1_present=present,
        J12s1_VOL=to_dense(monthly, "monthly_volume", tix, mix, T_m, N, fill=0.0),
        J12s1_R=to_dense(monthly, "ret_1m", tix, mix, T_m, N),
        J12s1_M=to_dense(monthly, "mom_J", tix, mix, T_m, N),
        J12s1_L=np.where(np.isnan(lab), -1, lab).astype(np.int8),
        J12s1_NR=to_dense(df, "next_ret", tix, mix, T_m, N),
        J12s1_EW=ew_d, J12s1_LS=ls,
        J12s1_mean=np.float64(mom_ret.mean()),
        J12s1_sharpe=np.float64(utils.sharpe(mom_ret.values, freq_per_year=12)),
        J12s1_cum=cum.to_numpy(), cum_dates_ns=cum.index.asi8,
        printed=np.array(buf.getvalue()),
        pandas_version=np.array(pd.__version__), numpy_version=np.array(np.__version__))
    print(f"  real_data: tickers={N} months={len(mom_ret)} mean={mom_ret.mean()!r} "
          f"sharpe={utils.sharpe(mom_ret.values, freq_per_year=12)!r}")
    print("  printed:", buf.getvalue().strip().replace("\n", " | "))


def decile_cases(rd, n_cases=3000, seed=7):
    rng = np.random.default_rng(seed)
    vals, offs, labs = [], [0], []
    for i in range(n_cases):
        n = int(rng.integers(0, 61))
        kind = i % 5
        if kind == 0:
            x = rng.normal(0, 1, n)
        elif kind == 1:
            x = np.round(rng.normal(0, 1, n), 1)  # heavy ties
        elif kind == 2:
            x = rng.integers(0, 4, n).astype(float)  # very heavy ties
        elif kind == 3:
            x = np.round(rng.lognormal(0, 1, n) - 1, 3)
        else:
            x = np.full(n, 0.25)
            if n:
                x[rng.integers(0, n)] = 1.5
        nanm = rng.random(n) < 0.15
        x[nanm] = np.nan
        lab = rd.assign_deciles_per_date(pd.Series(x), n=10).to_numpy(dtype=np.float64)
        vals.append(x)
        labs.append(lab)
        offs.append(offs[-1] + n)
    # a few large cross-sections
    for n, tie in [(1000, None), (2500, 2), (4096, 3), (777, 0)]:
        x = rng.standard_normal(n)
        if tie is not None:
            x = np.round(x, tie)
        lab = rd.assign_deciles_per_date(pd.Series(x), n=10).to_numpy(dtype=np.float64)
        vals.append(x)
        labs.append(lab)
        offs.append(offs[-1] + n)
    np.savez_compressed(OUT / "deciles.npz", values=np.concatenate(vals),
                        offsets=np.array(offs, dtype=np.int64), labels=np.concatenate(labs))
    print(f"  deciles: {len(offs) - 1} cross-sections")


def turnover_case(rd, feats):
    """compute_monthly_turnover (src/features.py:60-107) on the edge panel's monthly frame with
    a shares map mixing every branch of its _get_shares: shares_outstanding given, market_cap
    only (positive, zero, negative, NaN), and missing tickers.  Looks back 3 (run_demo's value)
    and 2 / 5 months."""
    ed = make_panel(160, 640, seed=11, start="2015-01-01", late=0.15, delist=0.15,
                    nan_day=0.03, absent_month=0.03, nan_month=0.03, cents=True)
    P, V, days, ms, mend, tickers = (ed["P"], ed["V"], ed["days"], ed["month_start"],
                                     ed["month_end"], ed["tickers"])
    T_m, N = len(ms) - 1, P.shape[1]
    tix = {t: i for i, t in enumerate(tickers)}
    mix = {d: i for i, d in enumerate(mend)}
    rng = np.random.default_rng(23)
    so = np.full(N, np.nan)
    mcap = np.full(N, np.nan)
    shares = {}
    for i, t in enumerate(tickers):
        kind = i % 6
        if kind in (0, 1):
            so[i] = float(int(rng.integers(10**6, 10**9)))
            shares[t] = {"shares_outstanding": int(so[i]), "market_cap": None}
        elif kind == 2:
            mcap[i] = float(rng.uniform(1e8, 1e11))
            shares[t] = {"shares_outstanding": None, "market_cap": mcap[i]}
        elif kind == 3:
            mcap[i] = [0.0, -5.0e9, np.nan][i % 3]
            shares[t] = {"shares_outstanding": np.nan, "market_cap": mcap[i]}
        elif kind == 4:
            shares[t] = {}
    daily = to_long(dict(P=P, V=V, days=days, tickers=tickers))
    monthly = feats.compute_monthly_momentum_from_daily(daily, lookback_months=12, skip_months=1)
    arrays = dict(P=P, V=V, day_ns=days.asi8, month_start=ms, month_end_ns=mend.asi8,
                  tickers=tickers.astype("U"), so=so, mcap=mcap,
                  pandas_version=np.array(pd.__version__), numpy_version=np.array(np.__version__))
    for lb in (3, 2, 5):
        out = feats.compute_monthly_turnover(monthly, shares_info_map=shares, lookback_months=lb)
        for col in ("adv_est", "shares_outstanding", "turnover_monthly", "turn_avg"):
            key = col if lb == 3 or col == "turn_avg" else None
            if key is None:
                continue
            arrays[f"lb{lb}_{col}"] = to_dense(out, col, tix, mix, T_m, N)
        print(f"  turnover lb={lb}: rows={len(out)} "
              f"valid turn_avg={int(out['turn_avg'].notna().sum())}")
    np.savez_compressed(OUT / "turnover.npz", **arrays)


def main():
    rd, data_io, feats, utils = load_reference()
    if "--only-turnover" in sys.argv:
        turnover_case(rd, feats)
        return
    print("real data ...")
    real_data_case(rd, data_io, feats, utils)
    print("deciles ...")
    decile_cases(rd)
    print("C1 (500 x 360 monthly) ...")
    c1 = make_panel(500, 360, seed=1, start="1990-01-31", monthly=True, absent_month=0.002,
                    nan_month=0.0, nan_day=0.003)
    run_case("c1", rd, feats, utils, c1["P"], None, c1["days"], c1["month_start"],
             c1["month_end"], c1["tickers"], [(12, 1), (3, 0)], full=False)
    print("edge daily panel ...")
    ed = make_panel(160, 640, seed=11, start="2015-01-01", late=0.15, delist=0.15,
                    nan_day=0.03, absent_month=0.03, nan_month=0.03, cents=True)
    run_case("edge", rd, feats, utils, ed["P"], ed["V"], ed["days"], ed["month_start"],
             ed["month_end"], ed["tickers"], [(12, 1), (3, 0), (6, 1), (9, 2), (1, 0)])
    print("small-universe panel (n<10 cross-sections) ...")
    sm = make_panel(7, 400, seed=13, start="2010-01-01", late=0.3, delist=0.3,
                    nan_day=0.05, absent_month=0.05, nan_month=0.05, cents=True)
    run_case("small", rd, feats, utils, sm["P"], sm["V"], sm["days"], sm["month_start"],
             sm["month_end"], sm["tickers"], [(12, 1), (3, 1)])
    print("long-window panel ...")
    lw = make_panel(40, 1700, seed=17, start="2001-01-01", nan_day=0.01, absent_month=0.01,
                    nan_month=0.01)
    run_case("longwin", rd, feats, utils, lw["P"], lw["V"], lw["days"], lw["month_start"],
             lw["month_end"], lw["tickers"], [(24, 1), (48, 3)])
    print("turnover features ...")
    turnover_case(rd, feats)


if __name__ == "__main__":
    main()
