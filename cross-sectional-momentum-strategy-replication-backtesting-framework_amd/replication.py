"""Drop-in counterparts of run_demo.py's momentum replication, backed by the HIP engine.

`assign_deciles_per_date` keeps run_demo.py:18-29's contract (Series in, labels aligned to
the input index out).  `monthly_replication` runs run_demo.py:31-79 -- signal, per-date
qcut deciles, next-row return, equal-weight decile means, top-minus-bottom, mean/Sharpe,
cumulative curve -- with every per-cell stage on the GPU, prints what the reference prints
and additionally RETURNS the results (the reference returns None).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np
import pandas as pd
import torch

from .features import compute_monthly_turnover, get_engine, monthly_signal
from .panel import monthly_frame
from .utils import save_plot, sharpe

RESULTS = "results"


def assign_deciles_per_date(series, n=10, device=None):
    """run_demo.py:18-29: `pd.qcut(s.dropna(), q=n, labels=False, duplicates='drop')`
    reindexed to `series.index`, computed by the GPU label kernel."""
    s = pd.Series(series)
    vals = pd.to_numeric(s, errors="coerce").to_numpy(dtype=np.float64)
    ok = ~np.isnan(vals)
    if not ok.any():
        return pd.Series(index=series.index, data=np.nan)
    eng = get_engine(device)
    M = torch.from_numpy(np.ascontiguousarray(vals[None, :])).to(eng.device)
    L, _, _, _ = eng.deciles(M, None, n)
    lab = L.cpu().numpy()[0].astype(np.float64)
    lab[lab < 0] = np.nan
    if np.isnan(lab).any():
        return pd.Series(lab, index=series.index)
    return pd.Series(lab.astype(np.int64), index=series.index)


@dataclass
class ReplicationResult:
    mom_ret: pd.Series        # top-minus-bottom monthly returns (NaN months dropped)
    ew: pd.DataFrame          # equal-weight mean next_ret per (date, label)
    mean: float
    sharpe: float
    cum: pd.Series            # (1 + mom_ret).cumprod()
    monthly: pd.DataFrame | None = None   # signal frame (features.py:55 columns)
    turnover: pd.DataFrame | None = None  # compute_monthly_turnover output, when requested


def monthly_replication(daily_df, shares_info=None, lookback_months=12, skip_months=1,
                        n_bins=10, plot_path=os.path.join(RESULTS, "monthly_mom_cum.png"),
                        compute_turnover=True, keep_monthly=False, device=None,
                        verbose=True):
    """run_demo.py:31-79 with the GPU engine.  Returns a ReplicationResult, or None where the
    reference prints a message and returns early.  Like run_demo.py:33 it computes the share
    turnover features (on the GPU, csm_turnover_features) even though the decile path does not
    use them; compute_turnover=False skips them."""
    panel, host, dev = monthly_signal(daily_df, lookback_months, skip_months, device)
    monthly = None
    if host is not None and (keep_monthly or compute_turnover):
        monthly = monthly_frame(panel, host["PM"], host["VOL"], host["R"], host["M"])
    turnover = None
    if compute_turnover and monthly is not None:
        turnover = compute_monthly_turnover(monthly, shares_info_map=shares_info,
                                            lookback_months=3, device=device)
    if host is None or np.isnan(host["M"]).all():
        if verbose:
            print("No monthly momentum data available after cleaning.")
        return None
    eng = get_engine(device)
    L, EW, CNT, _ = eng.deciles(dev["M"], dev["NR"], n_bins)
    LS = eng.long_short(EW, CNT)
    ew_h, cnt_h, ls_h = EW.cpu().numpy(), CNT.cpu().numpy(), LS.cpu().numpy()
    if not (cnt_h > 0).any():
        if verbose:
            print("No rows after next_ret/decile filtering.")
        return None
    rows = (cnt_h > 0).any(axis=1)
    cols = (cnt_h > 0).any(axis=0)
    ew = pd.DataFrame(np.where(cnt_h > 0, ew_h, np.nan)[rows][:, cols],
                      index=pd.DatetimeIndex(panel.month_end[rows], name="date"),
                      columns=pd.Index(np.nonzero(cols)[0].astype(np.float64), name="decile"))
    if ew.empty:   # run_demo.py:55-58 (unreachable once a count is positive; mirrored)
        if verbose:
            print("No decile returns calculated.")
        return None
    keep = ~np.isnan(ls_h)
    mom_ret = pd.Series(ls_h[keep], index=pd.DatetimeIndex(panel.month_end[keep], name="date"))
    if mom_ret.empty:
        if verbose:
            print("No momentum returns computed.")
        return None
    mean = mom_ret.mean()
    sh = sharpe(mom_ret.values, freq_per_year=12)
    if verbose:
        print("Monthly replication: mean monthly mom_ret:", mean)
        print("Sharpe (annualized, 12 periods):", sh)
    cum = (1 + mom_ret).cumprod()
    if plot_path:
        import matplotlib.pyplot as plt

        d = os.path.dirname(plot_path)
        if d:
            os.makedirs(d, exist_ok=True)
        fig = plt.figure(figsize=(8, 3))
        plt.plot(cum.index, cum.values)
        plt.title("Cumulative Top-minus-Bottom Momentum (yfinance)")
        save_plot(fig, plot_path)
    return ReplicationResult(mom_ret=mom_ret, ew=ew, mean=float(mean), sharpe=float(sh),
                             cum=cum, monthly=monthly if keep_monthly else None,
                             turnover=turnover)
