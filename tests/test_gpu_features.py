"""GPU: csm_turnover_features against the reference's compute_monthly_turnover
(tests/golden/turnover.npz, bit for bit) and the momentum x volume double sort against the
oracle (labels exact, cell returns within 1e-10)."""
import numpy as np
import pytest
import torch

from conftest import bits_equal, load_golden
from oracle import csmom_oracle as O
from oracle import features_oracle as F
from oracle import portfolio_oracle as PO

pytestmark = pytest.mark.gpu


def _up(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to("cuda:0")


@pytest.fixture(scope="module")
def case(engine):
    z = load_golden("turnover")
    PM, VOL = engine.month_end(_up(z["P"]), _up(z["month_start"].astype(np.int64)), _up(z["V"]))
    return z, PM, VOL


@pytest.mark.parametrize("lb", [3, 2, 5])
def test_turnover_features_bit_exact(engine, case, lb):
    z, PM, VOL = case
    ADV, SH, TURN, TAVG = engine.turnover_features(PM, VOL, _up(z["so"]), _up(z["mcap"]), lb)
    if lb == 3:
        assert bits_equal(ADV.cpu().numpy(), z["lb3_adv_est"])
        assert bits_equal(SH.cpu().numpy(), z["lb3_shares_outstanding"])
        assert bits_equal(TURN.cpu().numpy(), z["lb3_turnover_monthly"])
    assert bits_equal(TAVG.cpu().numpy(), z[f"lb{lb}_turn_avg"])


def test_turnover_features_rejects_long_window(engine, case):
    import csmom
    z, PM, VOL = case
    with pytest.raises(csmom.CsmError):
        engine.turnover_features(PM, VOL, _up(z["so"]), _up(z["mcap"]), 49)


@pytest.mark.parametrize("K", [1, 3])
def test_double_sort_vs_oracle(engine, case, K):
    import csmom
    z, PM, VOL = case
    _, M, NR = engine.momentum(PM, 12, 1)
    res = csmom.momentum_volume_double_sort(engine, PM, VOL, M, NR, _up(z["so"]),
                                            _up(z["mcap"]), K=K)
    Mh, NRh = M.cpu().numpy(), NR.cpu().numpy()
    tv = F.turnover_features(VOL.cpu().numpy(), PM.cpu().numpy(), z["so"], z["mcap"])["turn_avg"]
    Lm, Lv, Lc = F.double_sort_labels(Mh, tv)
    assert np.array_equal(res.Lm.cpu().numpy(), Lm)
    assert np.array_equal(res.Lv.cpu().numpy(), Lv)
    assert np.array_equal(res.Lc.cpu().numpy(), Lc)
    ref = PO.portfolio(Lc, NRh, 30, K=K)
    pr = res.PR.cpu().numpy().reshape(-1, 30)
    rp = ref["PR"][:, 0, :]
    assert np.array_equal(np.isnan(pr), np.isnan(rp))
    m = ~np.isnan(rp)
    assert (np.abs(pr[m] - rp[m]) <= 1e-10 * np.maximum(np.abs(rp[m]), 1e-12)).all()
    ls = res.LS.cpu().numpy()
    rls = rp.reshape(-1, 10, 3)[:, 9, :] - rp.reshape(-1, 10, 3)[:, 0, :]
    assert np.array_equal(np.isnan(ls), np.isnan(rls))


def _fixture_shares_map(z):
    """The shares map tests/golden/make_golden.py:264-277 built (every branch of the
    reference's _get_shares), recovered from the fixture's so / mcap arrays."""
    shares = {}
    for i, t in enumerate(z["tickers"]):
        kind = i % 6
        if kind in (0, 1):
            shares[str(t)] = {"shares_outstanding": int(z["so"][i]), "market_cap": None}
        elif kind == 2:
            shares[str(t)] = {"shares_outstanding": None, "market_cap": float(z["mcap"][i])}
        elif kind == 3:
            shares[str(t)] = {"shares_outstanding": np.nan, "market_cap": float(z["mcap"][i])}
        elif kind == 4:
            shares[str(t)] = {}
    return shares


@pytest.mark.parametrize("lb", [3, 2, 5])
def test_drop_in_compute_monthly_turnover_bit_exact(engine, lb):
    """csmom.compute_monthly_turnover (the drop-in of src/features.py:60-107, GPU arithmetic)
    on the frame csmom.compute_monthly_momentum_from_daily returns, against the reference's
    own outputs (turnover.npz)."""
    import pandas as pd

    import csmom
    from oracle.synth_np import to_long
    z = load_golden("turnover")
    days = pd.DatetimeIndex(z["day_ns"])
    daily = to_long(dict(P=z["P"], V=z["V"], days=days, tickers=z["tickers"].astype(object)))
    monthly = csmom.compute_monthly_momentum_from_daily(daily, lookback_months=12, skip_months=1)
    out = csmom.compute_monthly_turnover(monthly, shares_info_map=_fixture_shares_map(z),
                                         lookback_months=lb)
    tix = {str(t): i for i, t in enumerate(z["tickers"])}
    mix = {d: i for i, d in enumerate(pd.DatetimeIndex(z["month_end_ns"]))}
    T_m, N = z[f"lb{lb}_turn_avg"].shape

    def dense(col):
        a = np.full((T_m, N), np.nan)
        a[out["date"].map(mix).to_numpy(), out["ticker"].map(tix).to_numpy()] = \
            pd.to_numeric(out[col], errors="coerce").to_numpy(dtype=np.float64)
        return a
    assert bits_equal(dense("turn_avg"), z[f"lb{lb}_turn_avg"])
    if lb == 3:
        for col in ("adv_est", "shares_outstanding", "turnover_monthly"):
            assert bits_equal(dense(col), z[f"lb3_{col}"]), col
