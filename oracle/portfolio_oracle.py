"""CPU oracle for the portfolio-accounting extensions -- TEST INFRASTRUCTURE ONLY.

SURVEY.md 8(f) rank 2: Jegadeesh-Titman overlapping K-month holding portfolios, equal or
value weights, long-short portfolio turnover and transaction costs, plus the bootstrap
panels and (J, K) sweeps of BASELINE configs C3 / C5.  The reference implements only the
K = 1 equal-weight, cost-free case (`run_demo.py:49-67`); everything beyond it is
**parity unpinned** against the reference.  This restatement is the executable spec
(rules E1..E6), and it collapses to the reference path at K = 1 /
equal weight (`tests/test_portfolio_oracle.py` checks that against the golden fixtures).
Like csmom_oracle, only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s CPU-baseline
leg may import it; the product never does.

Indexing: everything is at formation-date granularity, `t` = month row.  `NR[t][a]` is the
asset's return over (t, t+1] (the reference's `next_ret`), so a cohort formed at `s` earns
`NR[t]` in holding months t = s .. s+K-1.  Batched panels are [T_m][B][N] (B cross-sections
per month row), the engine's sweep layout.

  E1 cohort return  CR[s][t][d] = sum_{a in V} W[s][a] NR[t][a] / sum_{a in V} W[s][a],
                    members C_s^d = {a: L[s][a] = d, W[s][a] finite and > 0} (EW: W = 1),
                    V = members with NR[t][a] not NaN; NaN if V is empty.
  E2 overlap        PR[t][d] = mean of CR[t-k][t][d] over k in [0, K) with t-k >= 0 and
                    CR not NaN; NaN if none.  (K = 1: the reference's decile mean.)
  E3 long-short     the reference's rule (`run_demo.py:60-67`) on PR: top minus bottom if
                    both columns are non-NaN somewhere, else row max - min; NaN dropped.
  E4 turnover       cohort leg weights omega_s^d[a] = W[s][a] / sum_{C_s^d} W (all members,
                    fixed at formation); w_t^d = mean of omega_{t-k}^d over the K_t
                    non-empty cohorts; TURN[t] = 1/2 sum_a (|dw^top| + |dw^0|), w_{-1} = 0.
  E5 costs          `src/execution_models.py:4-12`: per unit of traded notional
                    spread/2 + k * vol * sqrt(|size| / adv); with the trade |dw| * AUM and
                    adv = ADV[t][a] (dollars): COST[t] = sum_a sum_legs |dw| *
                    (spread/2 + k * SIG[t][a] * sqrt(|dw| * AUM / ADV[t][a])) (no impact
                    term when ADV is not given or ADV <= 0; SIG defaults to 0.02, the
                    reference's `vol_map` fallback).  NET[t] = LS[t] - COST[t].
  E6 bootstrap      stationary bootstrap of months (mean block length Lb) with a
                    counter-based splitmix64 stream keyed by (seed, panel, month); panel b's
                    month price is a sequential product of the source months' returns.
"""
from __future__ import annotations

import numpy as np

from .csmom_oracle import absent_like, is_absent, long_short as _long_short_ref

HALF_SPREAD = 0.0005   # execution_models.py:9 spread=0.001
K_IMPACT = 0.1         # execution_models.py:4 k=0.1
DEFAULT_VOL = 0.02     # backtester.py vol_map fallback


def _as_batched(X: np.ndarray, B: int | None) -> np.ndarray:
    if X.ndim == 3:
        return X
    return X[:, None, :] if B in (None, 1) else X.reshape(X.shape[0], B, -1)


def member_weights(L: np.ndarray, d: int, W: np.ndarray | None) -> np.ndarray:
    """Formation weights of the members of label d (0 outside), float64, same shape as L."""
    m = L == d
    if W is None:
        return m.astype(np.float64)
    ok = m & np.isfinite(W) & (W > 0)
    return np.where(ok, W, 0.0)


def cohort_returns(L, NR, n_bins: int, K: int, W=None):
    """E1: CR[t][k][b][d] = return in holding month t of the cohort formed at t-k.
    L, NR, W: [T_m][B][N] (or [T_m][N]).  Returns (CR, SWR, SW, CNT) with sums over V."""
    L, NR = _as_batched(L, None), _as_batched(NR, None)
    W = None if W is None else _as_batched(W, None)
    T_m, B, N = L.shape
    SWR = np.zeros((T_m, K, B, n_bins))
    SW = np.zeros((T_m, K, B, n_bins))
    CNT = np.zeros((T_m, K, B, n_bins), dtype=np.int64)
    for t in range(T_m):
        r = NR[t]
        rv = ~np.isnan(r)
        for k in range(K):
            s = t - k
            if s < 0:
                continue
            for d in range(n_bins):
                w = member_weights(L[s], d, None if W is None else W[s])
                use = (w > 0) & rv
                SWR[t, k, :, d] = np.where(use, w * np.where(rv, r, 0.0), 0.0).sum(axis=1)
                SW[t, k, :, d] = np.where(use, w, 0.0).sum(axis=1)
                CNT[t, k, :, d] = use.sum(axis=1)
    with np.errstate(invalid="ignore", divide="ignore"):
        CR = np.where(CNT > 0, SWR / np.where(SW > 0, SW, 1.0), np.nan)
    return CR, SWR, SW, CNT


def overlap_returns(CR: np.ndarray) -> np.ndarray:
    """E2: PR[t][b][d] = mean over the available cohorts (NaN if none)."""
    ok = ~np.isnan(CR)
    n = ok.sum(axis=1)
    s = np.where(ok, CR, 0.0).sum(axis=1)
    with np.errstate(invalid="ignore", divide="ignore"):
        return np.where(n > 0, s / np.maximum(n, 1), np.nan)


def long_short_k(PR: np.ndarray) -> np.ndarray:
    """E3 per panel: PR [T_m][B][n_bins] -> LS [T_m][B]."""
    T_m, B, nb = PR.shape
    LS = np.full((T_m, B), np.nan)
    for b in range(B):
        cnt = (~np.isnan(PR[:, b, :])).astype(np.int64)
        LS[:, b] = _long_short_ref(PR[:, b, :], cnt)
    return LS


def leg_weights(L, n_bins: int, K: int, W=None):
    """E4: aggregate leg weights w[t][leg][b][a] for legs (top, bottom)."""
    L = _as_batched(L, None)
    W = None if W is None else _as_batched(W, None)
    T_m, B, N = L.shape
    out = np.zeros((T_m, 2, B, N))
    for li, d in enumerate((n_bins - 1, 0)):
        om = np.zeros((T_m, B, N))
        ne = np.zeros((T_m, B), dtype=bool)
        for s in range(T_m):
            w = member_weights(L[s], d, None if W is None else W[s])
            tot = w.sum(axis=1)
            ne[s] = tot > 0
            with np.errstate(invalid="ignore", divide="ignore"):
                om[s] = np.where(tot[:, None] > 0, w / np.where(tot > 0, tot, 1.0)[:, None], 0.0)
        for t in range(T_m):
            acc = np.zeros((B, N))
            kt = np.zeros(B)
            for k in range(K):
                s = t - k
                if s < 0:
                    continue
                acc += om[s]
                kt += ne[s]
            with np.errstate(invalid="ignore", divide="ignore"):
                out[t, li] = np.where(kt[:, None] > 0, acc / np.maximum(kt, 1)[:, None], 0.0)
    return out


def turnover_costs(L, n_bins: int, K: int, W=None, half_spread: float = HALF_SPREAD,
                   k_impact: float = K_IMPACT, aum: float = 0.0, ADV=None, SIG=None):
    """E4 + E5: TURN[t][b], COST[t][b]."""
    L = _as_batched(L, None)
    T_m, B, N = L.shape
    w = leg_weights(L, n_bins, K, W)
    prev = np.zeros((2, B, N))
    TURN = np.zeros((T_m, B))
    COST = np.zeros((T_m, B))
    ADVb = None if ADV is None else _as_batched(ADV, None)
    SIGb = None if SIG is None else _as_batched(SIG, None)
    for t in range(T_m):
        dw = np.abs(w[t] - prev)          # [2][B][N]
        TURN[t] = 0.5 * dw.sum(axis=(0, 2))
        unit = np.full((2, B, N), half_spread)
        if ADVb is not None and aum > 0:
            sig = DEFAULT_VOL if SIGb is None else np.where(np.isnan(SIGb[t]), DEFAULT_VOL, SIGb[t])
            adv = ADVb[t]
            with np.errstate(invalid="ignore", divide="ignore"):
                imp = np.where(adv > 0, k_impact * sig * np.sqrt(dw * aum / np.where(adv > 0, adv, 1.0)), 0.0)
            unit = unit + np.nan_to_num(imp)
        COST[t] = (dw * unit).sum(axis=(0, 2))
        prev = w[t]
    return TURN, COST


def portfolio(L, NR, n_bins: int = 10, K: int = 1, W=None, half_spread: float = HALF_SPREAD,
              k_impact: float = K_IMPACT, aum: float = 0.0, ADV=None, SIG=None) -> dict:
    """E1..E5 end to end on [T_m][B][N] (or [T_m][N]) labels / next returns."""
    CR, SWR, SW, CNT = cohort_returns(L, NR, n_bins, K, W)
    PR = overlap_returns(CR)
    LS = long_short_k(PR)
    TURN, COST = turnover_costs(L, n_bins, K, W, half_spread, k_impact, aum, ADV, SIG)
    return dict(CR=CR, CNT=CNT, PR=PR, LS=LS, TURN=TURN, COST=COST, NET=LS - COST)


# ------------------------------------------------------------------------------ E6
_M64 = (1 << 64) - 1


def splitmix64(x: np.ndarray) -> np.ndarray:
    """The splitmix64 finaliser on uint64 arrays (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = (x + np.uint64(0x9E3779B97F4A7C15)).astype(np.uint64)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _uniform(seed: int, b: np.ndarray, t: int, stream: int) -> np.ndarray:
    """U[0,1) from the counter (seed, panel b, month t, stream) -- same as the device."""
    with np.errstate(over="ignore"):
        key = (np.uint64(seed) * np.uint64(0xD1B54A32D192ED03)
               + b.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
               + np.uint64(t * 4 + stream))
    return (splitmix64(key) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def bootstrap_indices(T_m: int, B: int, seed: int, mean_block: float, b0: int = 0) -> np.ndarray:
    """Stationary-bootstrap source months src[B][T_m] for panels b0 .. b0+B-1."""
    b = np.arange(b0, b0 + B, dtype=np.int64)
    src = np.zeros((B, T_m), dtype=np.int64)
    p_new = 1.0 / mean_block
    for t in range(T_m):
        u_pos = _uniform(seed, b, t, 0)
        jump = np.minimum((u_pos * T_m).astype(np.int64), T_m - 1)
        if t == 0:
            src[:, 0] = jump
        else:
            new = _uniform(seed, b, t, 1) < p_new
            src[:, t] = np.where(new, jump, (src[:, t - 1] + 1) % T_m)
    return src


def bootstrap_panel(R: np.ndarray, src: np.ndarray, p0: float = 100.0) -> np.ndarray:
    """E6 panel prices PMb[T_m][B][N] from base month returns R[T_m][N] (absent payload or
    NaN = no row): cell absent if the source return is absent / NaN, else
    price = prev * (1 + r) with prev starting at p0 (sequential fp64 product)."""
    B, T_m = src.shape
    N = R.shape[1]
    out = absent_like((T_m, B, N))
    prev = np.full((B, N), p0)
    for t in range(T_m):
        r = R[src[:, t]]                  # [B][N]
        ok = ~np.isnan(r)
        nxt = prev * (1.0 + np.where(ok, r, 0.0))
        out[t] = np.where(ok, nxt, out[t])
        prev = np.where(ok, nxt, prev)
    return out


__all__ = ["cohort_returns", "overlap_returns", "long_short_k", "leg_weights",
           "turnover_costs", "portfolio", "splitmix64", "bootstrap_indices",
           "bootstrap_panel", "is_absent"]
