"""Momentum x trading-volume double sort (Lee & Swaminathan 2000, section II; SURVEY 8(f)
rank 3).  The reference computes share turnover (src/features.py:60-107) but never uses it;
this finishes the thought its LeSw00.pdf describes: stocks are sorted independently each
month into momentum deciles (the reference's qcut rule, run_demo.py:18-29) and turnover
terciles (the same rule with 3 bins on the rolling turnover, over the rows with a valid
signal), and the 30 cell portfolios are held K months (rules E1..E5 with 30 groups).

Everything runs on the device: csm_turnover_features, csm_deciles (twice),
csm_double_sort_labels, csm_portfolio (n_bins = 30).  Parity: the turnover features are
bit-exact with the reference (tests/golden/turnover.npz); the sort and cell returns are
pinned only by the oracle restatement (rule T2, oracle/features_oracle.py).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch


@dataclass
class DoubleSortResult:
    Lm: torch.Tensor          # [T_m][N] momentum decile
    Lv: torch.Tensor          # [T_m][N] turnover tercile
    Lc: torch.Tensor          # [T_m][N] cell = n_vol * Lm + Lv
    PR: torch.Tensor          # [T_m][n_mom][n_vol] cell returns (K-overlapped)
    LS: torch.Tensor          # [T_m][n_vol] top minus bottom momentum decile per tercile
    TAVG: torch.Tensor        # [T_m][N] rolling turnover used for the terciles


def momentum_volume_double_sort(eng, PM, VOL, M, NR, so, mcap, n_mom=10, n_vol=3, K=1,
                                lookback=3, W=None) -> DoubleSortResult:
    T_m, N = M.shape
    _, _, _, TAVG = eng.turnover_features(PM, VOL, so, mcap, lookback)
    Lm, _, _, _ = eng.deciles(M, None, n_mom)
    Lv, _, _, _ = eng.deciles(eng.mask_by(M, TAVG), None, n_vol)
    Lc = eng.combine_labels(Lm, Lv, n_vol)
    out = eng.portfolio(Lc, NR, n_mom * n_vol, K=K, W=W, with_costs=False)
    PR = out.PR[:, 0, :].reshape(T_m, n_mom, n_vol)
    LS = PR[:, n_mom - 1, :] - PR[:, 0, :]
    return DoubleSortResult(Lm=Lm, Lv=Lv, Lc=Lc, PR=PR, LS=LS, TAVG=TAVG)


__all__ = ["DoubleSortResult", "momentum_volume_double_sort"]
