"""CPU: the portfolio-extension oracle (rules E1..E6, oracle/portfolio_oracle.py).

Beyond K = 1 / equal weight the reference has no counterpart (parity unpinned); these tests
pin the restatement to the reference where they overlap (K = 1 EW against the golden
fixtures made by running the reference) and check the extension's defining properties.
"""
import numpy as np
import pytest

from conftest import golden_tags, load_golden, max_rel
from oracle import csmom_oracle as O
from oracle import portfolio_oracle as PO

REL = 1e-10


def _fixture_L_NR(name, tag):
    z = load_golden(name)
    J, s = int(tag[1:tag.index("s")]), int(tag[tag.index("s") + 1:])
    PM, _ = O.month_end(z["P"], z["month_start"].astype(np.int64))
    _, M, NR, _ = O.momentum_scan(PM, J, s)
    L = O.assign_deciles(M, 10)
    assert np.array_equal(L, z[f"{tag}_L"])
    return z, L, NR, PM


@pytest.mark.parametrize("name", ["edge", "c1", "real_data"])
def test_k1_equal_weight_collapses_to_reference(name):
    z = load_golden(name)
    for tag in golden_tags(z):
        _, L, NR, _ = _fixture_L_NR(name, tag)
        out = PO.portfolio(L, NR, 10, K=1)
        ew = out["PR"][:, 0, :]
        ref = z[f"{tag}_EW"]
        assert np.array_equal(np.isnan(ew), np.isnan(ref)), tag
        assert max_rel(ew, ref) <= REL, tag
        ls = out["LS"][:, 0]
        assert np.array_equal(np.isnan(ls), np.isnan(z[f"{tag}_LS"])), tag
        assert max_rel(ls, z[f"{tag}_LS"]) <= REL, tag


def test_overlap_is_mean_of_cohorts():
    z, L, NR, _ = _fixture_L_NR("c1", "J12s1")
    K = 6
    out = PO.portfolio(L, NR, 10, K=K)
    one = [PO.cohort_returns(L, NR, 10, K)[0][:, k, 0, :] for k in range(K)]
    st = np.stack(one, axis=1)                       # [T][K][d]
    ok = ~np.isnan(st)
    with np.errstate(invalid="ignore"):
        ref = np.where(ok, st, 0.0).sum(axis=1) / ok.sum(axis=1)
    assert max_rel(out["PR"][:, 0, :], ref) <= 1e-13
    # cohort k of month t is cohort 0 (K=1) of the same formation month with NR of month t
    for t in range(20, 40):
        for k in range(K):
            s = t - k
            sel = L[s] == 9
            ok = sel & ~np.isnan(NR[t])
            if ok.any():
                assert abs(st[t, k, 9] - NR[t][ok].mean()) <= 1e-13 * max(1, abs(NR[t][ok].mean()))


def test_value_weight_constant_equals_equal_weight():
    _, L, NR, _ = _fixture_L_NR("c1", "J12s1")
    W = np.full(L.shape, 3.5)
    W[0, 0] = np.nan  # an invalid weight removes that member
    a = PO.portfolio(L, NR, 10, K=3)
    b = PO.portfolio(L, NR, 10, K=3, W=W)
    assert max_rel(b["PR"][1:], a["PR"][1:]) <= 1e-12
    assert max_rel(b["TURN"][2:], a["TURN"][2:]) <= 1e-12


def test_turnover_properties():
    _, L, NR, _ = _fixture_L_NR("c1", "J12s1")
    T_m, N = L.shape
    # constant labels: only the initial build trades (both legs bought once at K=1)
    Lc = np.tile(L[200], (T_m, 1))
    tr, _ = PO.turnover_costs(Lc, 10, 1)
    assert abs(tr[0, 0] - 1.0) <= 1e-12 and np.abs(tr[1:, 0]).max() <= 1e-12
    # K-overlap builds the position over K months then stops trading
    tr3, _ = PO.turnover_costs(Lc, 10, 3)
    assert abs(tr3[0, 0] - 1.0) <= 1e-12 and np.abs(tr3[1:, 0]).max() <= 1e-12
    # real labels: turnover in [0, 2], and a longer holding period trades less on average
    t1, c1 = PO.turnover_costs(L, 10, 1)
    t6, c6 = PO.turnover_costs(L, 10, 6)
    assert (t1 >= 0).all() and (t1 <= 2 + 1e-12).all()
    assert t6[30:].mean() < t1[30:].mean()
    # linear cost = half spread x traded notional (2 x turnover)
    assert max_rel(c1, 2 * t1 * PO.HALF_SPREAD) <= 1e-12


def test_impact_cost_matches_execution_model():
    """E5 against the reference's own formula (src/execution_models.py:4-12) on one cell."""
    L = np.array([[9, 0, 5]], dtype=np.int8)
    ADV = np.array([[2.0e6, 5.0e5, 1.0e6]])
    SIG = np.array([[0.03, np.nan, 0.01]])
    aum = 1.0e6
    tr, cost = PO.turnover_costs(L, 10, 1, aum=aum, ADV=ADV, SIG=SIG)
    # trades: asset 0 buys weight 1 of the long leg, asset 1 weight 1 of the short leg
    def ref_unit(size, adv, vol):  # spread/2 + square_root_impact(size, adv, vol)
        return 0.001 / 2.0 + 0.1 * vol * (abs(size) / adv) ** 0.5
    expect = 1.0 * ref_unit(aum, 2.0e6, 0.03) + 1.0 * ref_unit(aum, 5.0e5, 0.02)
    assert abs(cost[0, 0] - expect) <= 1e-15 * expect * 10
    assert tr[0, 0] == 1.0


def test_bootstrap_indices_and_identity_panel():
    src = PO.bootstrap_indices(50, 7, seed=5000, mean_block=4.0)
    assert src.shape == (7, 50) and src.min() >= 0 and src.max() < 50
    assert np.array_equal(src, PO.bootstrap_indices(50, 7, seed=5000, mean_block=4.0))
    # panel b is independent of which batch it was generated in (shard-invariant)
    assert np.array_equal(src[3:], PO.bootstrap_indices(50, 4, seed=5000, mean_block=4.0, b0=3))
    # mean block length ~ Lb: fraction of continuations ~ 1 - 1/Lb
    big = PO.bootstrap_indices(400, 64, seed=7, mean_block=4.0)
    cont = ((big[:, 1:] - big[:, :-1]) % 400 == 1).mean()
    assert 0.70 < cont < 0.80
    # identity resampling reproduces a cumulative-return price path
    R = np.array([[0.1, np.nan], [-0.2, 0.05], [np.nan, 0.5]])
    pm = PO.bootstrap_panel(R, np.array([[0, 1, 2]]), p0=100.0)
    assert pm.shape == (3, 1, 2)
    assert pm[0, 0, 0] == 100.0 * (1.0 + 0.1) and O.is_absent(pm[0, 0, 1])
    assert pm[1, 0, 0] == (100.0 * 1.1) * (1.0 - 0.2) and pm[1, 0, 1] == 100.0 * 1.05
    assert O.is_absent(pm[2, 0, 0]) and pm[2, 0, 1] == (100.0 * 1.05) * 1.5


def test_batched_layout_equals_per_panel():
    _, L, NR, _ = _fixture_L_NR("c1", "J12s1")
    L2 = np.stack([L, L[:, ::-1]], axis=1)          # [T][2][N]
    NR2 = np.stack([NR, NR[:, ::-1]], axis=1)
    both = PO.portfolio(L2, NR2, 10, K=3)
    for b, (l, r) in enumerate(((L, NR), (L[:, ::-1], NR[:, ::-1]))):
        one = PO.portfolio(l, r, 10, K=3)
        assert max_rel(both["PR"][:, b], one["PR"][:, 0]) <= 1e-13
        assert max_rel(both["TURN"][:, b], one["TURN"][:, 0]) <= 1e-12
