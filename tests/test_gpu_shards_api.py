"""GPU: date-shard decomposition == unsharded (bit for bit) and the drop-in API on real data."""
import io
import contextlib

import numpy as np
import pandas as pd
import pytest
import torch

from conftest import bits_equal, load_golden, max_rel
from oracle import csmom_oracle as O

pytestmark = pytest.mark.gpu


def _up(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to("cuda:0")


@pytest.mark.parametrize("J,skip", [(12, 1), (3, 0), (9, 2)])
@pytest.mark.parametrize("G", [2, 3, 5, 8])
def test_virtual_shards_equal_unsharded(engine, J, skip, G):
    import csmom
    from csmom.distributed import virtual_shards
    z = load_golden("edge")
    P, ms = _up(z["P"]), z["month_start"].astype(np.int64)
    out = engine.run(P, _up(ms), J, skip, 10)
    M, NR, L, EW, CNT, LS = virtual_shards(engine, P, ms, G, J, skip, 10)
    assert bits_equal(M.cpu().numpy(), out.M.cpu().numpy())
    assert bits_equal(NR.cpu().numpy(), out.NR.cpu().numpy())
    assert torch.equal(L, out.L)
    assert torch.equal(CNT, out.CNT)
    assert bits_equal(EW.cpu().numpy(), out.EW.cpu().numpy())
    assert bits_equal(LS.cpu().numpy(), out.LS.cpu().numpy())


@pytest.mark.parametrize("J,skip", [(12, 1), (3, 0), (9, 2)])
@pytest.mark.parametrize("G", [2, 3, 5, 8])
def test_fused_virtual_shards_equal_unsharded(engine, J, skip, G):
    """Speculative fused shards (signal from an empty state + shard_repair) == one pass."""
    from csmom.distributed import virtual_shards
    z = load_golden("edge")
    P, ms = _up(z["P"]), z["month_start"].astype(np.int64)
    out = engine.run(P, _up(ms), J, skip, 10)
    M, NR, L, EW, CNT, LS = virtual_shards(engine, P, ms, G, J, skip, 10, fused=True)
    assert bits_equal(M.cpu().numpy(), out.M.cpu().numpy())
    assert bits_equal(NR.cpu().numpy(), out.NR.cpu().numpy())
    assert torch.equal(L, out.L)
    assert torch.equal(CNT, out.CNT)
    assert bits_equal(EW.cpu().numpy(), out.EW.cpu().numpy())
    assert bits_equal(LS.cpu().numpy(), out.LS.cpu().numpy())


@pytest.mark.parametrize("J,skip,G", [(24, 1, 3), (48, 1, 2), (48, 0, 4)])
def test_fused_shards_long_windows(engine, J, skip, G):
    from csmom.distributed import virtual_shards
    z = load_golden("longwin")
    P, ms = _up(z["P"]), z["month_start"].astype(np.int64)
    out = engine.run(P, _up(ms), J, skip, 10)
    M, NR, L, EW, CNT, LS = virtual_shards(engine, P, ms, G, J, skip, 10, fused=True)
    assert bits_equal(M.cpu().numpy(), out.M.cpu().numpy())
    assert bits_equal(NR.cpu().numpy(), out.NR.cpu().numpy())
    assert torch.equal(L, out.L)
    assert bits_equal(LS.cpu().numpy(), out.LS.cpu().numpy())


@pytest.mark.parametrize("G", [2, 7])
def test_fused_shards_sparse_panel(engine, G):
    """Gappy synthetic panel: many absent months and NaN month prices, so repairs run long
    (past several shard boundaries) and pending rows cross shards."""
    from oracle.synth_np import make_panel
    from csmom.distributed import virtual_shards
    pan = make_panel(512, 2600, seed=11, nan_day=0.05, absent_month=0.25, nan_month=0.15,
                     cents=True)
    P, ms = _up(pan["P"]), pan["month_start"].astype(np.int64)
    out = engine.run(P, _up(ms), 12, 1, 10, with_ret=True)
    M, NR, L, EW, CNT, LS = virtual_shards(engine, P, ms, G, 12, 1, 10, fused=True)
    assert bits_equal(M.cpu().numpy(), out.M.cpu().numpy())
    assert bits_equal(NR.cpu().numpy(), out.NR.cpu().numpy())
    assert torch.equal(L, out.L)
    assert bits_equal(LS.cpu().numpy(), out.LS.cpu().numpy())


@pytest.mark.parametrize("G", [2, 7])
@pytest.mark.parametrize("J,skip", [(12, 1), (3, 0)])
def test_fused_shards_four_wave_blocks(engine, G, J, skip):
    """The shard signal kernel on the C4 configuration (4 barrier-free waves per workgroup,
    2 month buffers, raw buffer loads; chosen by default at >= 92,160 assets, forced here) on a
    gappy panel: equal to the one-GPU pass bit for bit."""
    from oracle.synth_np import make_panel
    from csmom.distributed import virtual_shards
    pan = make_panel(1_000, 2600, seed=13, nan_day=0.05, absent_month=0.2, nan_month=0.1,
                     cents=True)
    P, ms = _up(pan["P"]), pan["month_start"].astype(np.int64)
    out = engine.run(P, _up(ms), J, skip, 10, with_ret=True)
    lib = engine.lib
    try:
        assert lib.csm_tune(b"signal_bwf", 4) == 0
        M, NR, L, EW, CNT, LS = virtual_shards(engine, P, ms, G, J, skip, 10, fused=True)
    finally:
        lib.csm_tune(b"signal_bwf", 0)
    assert bits_equal(M.cpu().numpy(), out.M.cpu().numpy())
    assert bits_equal(NR.cpu().numpy(), out.NR.cpu().numpy())
    assert torch.equal(L, out.L)
    assert bits_equal(LS.cpu().numpy(), out.LS.cpu().numpy())


@pytest.mark.parametrize("G", [2, 5])
def test_fused_shards_bucket_ids(engine, G):
    """Rows wider than the narrow-row kernels: the shard pass writes bucket ids, the repair
    rewrites those of the cells it replays, each shard ranks from its ids -- equal to the
    one-GPU csm_pipeline (which ranks from ids too) bit for bit, decile means included."""
    from oracle.synth_np import make_panel
    from csmom.distributed import virtual_shards
    pan = make_panel(20_000, 1_400, seed=17, with_volume=False, nan_day=0.03, absent_month=0.05,
                     nan_month=0.05, cents=True)
    P, ms = _up(pan["P"]), pan["month_start"].astype(np.int64)
    out = engine.pipeline(P, _up(ms), 12, 1, 10)
    M, NR, L, EW, CNT, LS = virtual_shards(engine, P, ms, G, 12, 1, 10, fused=True)
    assert bits_equal(M.cpu().numpy(), out.M.cpu().numpy())
    assert bits_equal(NR.cpu().numpy(), out.NR.cpu().numpy())
    assert torch.equal(L, out.L)
    assert torch.equal(CNT, out.CNT)
    assert bits_equal(EW.cpu().numpy(), out.EW.cpu().numpy())
    assert bits_equal(LS.cpu().numpy(), out.LS.cpu().numpy())
    ref = O.pipeline(pan["P"], ms, 12, 1, 10)
    assert np.array_equal(L.cpu().numpy(), ref["L"])


def test_shard_repair_rewrites_ret(engine):
    """With R requested, the repaired R of a shard equals the carried scan's R."""
    z = load_golden("edge")
    J, skip = 12, 1
    P, ms = z["P"], z["month_start"].astype(np.int64)
    PMd, _ = engine.month_end(_up(P), _up(ms))
    T_m = PMd.shape[0]
    m0 = T_m // 2
    d0 = int(ms[m0])
    sums = torch.stack([engine.shard_summary(PMd[:m0].contiguous(), J, skip),
                        engine.shard_summary(PMd[m0:].contiguous(), J, skip)])
    carry, npm = engine.fold_carry(sums, 1, J, skip)
    R0, M0, NR0 = engine.momentum(PMd[m0:].contiguous(), J, skip, with_ret=True, carry=carry,
                                  next_pm=npm)
    maxd = int(np.diff(ms).max())
    PM, R, M, NR, st = engine.signal_shard(_up(P[d0:]), _up(ms[m0:] - d0), maxd, J, skip,
                                           with_ret=True)
    engine.shard_repair(PM, carry, npm, st, M, NR, J, skip, R=R)
    assert bits_equal(R.cpu().numpy(), R0.cpu().numpy())
    assert bits_equal(M.cpu().numpy(), M0.cpu().numpy())
    assert bits_equal(NR.cpu().numpy(), NR0.cpu().numpy())


@pytest.mark.parametrize("panel", ["edge", "longwin", "sparse"])
@pytest.mark.parametrize("J,skip", [(12, 1), (24, 0)])
def test_summary_from_state_equals_full_pass(engine, panel, J, skip):
    """csm_shard_summary_state (walks from the shard's ends; months PM does not keep are
    re-derived from P) == csm_shard_summary (full pass over the full PM), on every shard of a
    2- and 3-way split, and signal_shard's kept PM rows / end state are right."""
    from oracle.synth_np import make_panel
    if panel == "sparse":   # ~240 months: shards longer than the kept edges, long walks
        z = make_panel(300, 5000, seed=3, nan_day=0.05, absent_month=0.3, nan_month=0.3)
    else:
        z = load_golden(panel)
    P, ms = z["P"], z["month_start"].astype(np.int64)
    T_m = len(ms) - 1
    H = J + skip + 8
    for G in (2, 3):
        for a, b in O.month_ranges(T_m, G):
            d0, d1 = int(ms[a]), int(ms[b])
            msl = ms[a:b + 1] - d0
            maxd = int(np.diff(msl).max())
            PM, _, M, NR, st = engine.signal_shard(_up(P[d0:d1]), _up(msl), maxd, J, skip)
            PMref, _ = engine.month_end(_up(P[d0:d1]), _up(msl))
            tm = b - a
            kept = [m for m in range(tm) if m < H or m >= tm - H]
            assert bits_equal(PM.cpu().numpy()[kept], PMref.cpu().numpy()[kept])
            full = engine.shard_summary(PMref, J, skip)
            fast = engine.shard_summary(PM, J, skip, state=st)
            assert bits_equal(fast.cpu().numpy(), full.cpu().numpy()), (panel, G, a, b)
            pres = ~O.is_absent(PMref.cpu().numpy())
            s = st.t.cpu().numpy()
            assert np.array_equal(s[0], pres.sum(0))
            idx = np.arange(tm)[:, None]
            assert np.array_equal(s[3], np.where(pres.any(0), np.where(pres, idx, 10**9).min(0),
                                                 -1))
            assert np.array_equal(s[4], np.where(pres.any(0), np.where(pres, idx, -1).max(0),
                                                 -1))


def test_summary_and_fold_match_oracle(engine):
    z = load_golden("edge")
    J, skip = 12, 1
    PM = O.month_end(z["P"], z["month_start"])[0]
    parts = O.month_ranges(PM.shape[0], 4)
    sums = np.stack([O.shard_summary(PM[a:b], J, skip) for a, b in parts])
    gs = torch.stack([engine.shard_summary(_up(PM[a:b]), J, skip) for a, b in parts])
    assert bits_equal(gs.cpu().numpy(), sums)
    for g in range(4):
        st, npm = O.fold_carry(sums, g, J, skip)
        carry, next_pm = engine.fold_carry(gs, g, J, skip)
        c = carry.cpu().numpy()
        assert bits_equal(c[:J + skip], 1.0 + st.ring), g
        assert bits_equal(c[J + skip], st.pff), g
        assert bits_equal(c[J + skip + 1], st.psff), g
        assert bits_equal(next_pm.cpu().numpy(), npm), g


def test_carry_out_chains(engine):
    """Running the scan in two chunks with carry_out -> carry equals one scan."""
    z = load_golden("longwin")
    PM, _ = engine.month_end(_up(z["P"]), _up(z["month_start"].astype(np.int64)))
    J, skip = 24, 1
    _, M, NR = engine.momentum(PM, J, skip)
    cut = PM.shape[0] // 2
    co = torch.empty((J + skip + 2, PM.shape[1]), dtype=torch.float64, device="cuda:0")
    _, M1, _ = engine.momentum(PM[:cut].contiguous(), J, skip, carry_out=co)
    _, M2, _ = engine.momentum(PM[cut:].contiguous(), J, skip, carry=co)
    assert bits_equal(torch.cat([M1, M2]).cpu().numpy(), M.cpu().numpy())


def _real_long():
    z = load_golden("real_data")
    P, V = z["P"], z["V"]
    days = pd.DatetimeIndex(z["day_ns"])
    tick = z["tickers"]
    pres = ~O.is_absent(P)
    dd, aa = np.nonzero(pres.T)[1], np.nonzero(pres.T)[0]
    return pd.DataFrame({"date": days[dd], "ticker": tick[aa], "adj_close": P[dd, aa],
                         "volume": V[dd, aa]}), z


def test_compute_monthly_momentum_frame(engine):
    import csmom
    df, z = _real_long()
    out = csmom.compute_monthly_momentum_from_daily(df, 12, 1)
    assert list(out.columns) == ["ticker", "date", "adj_close", "monthly_volume", "ret_1m", "mom_J"]
    tix = {t: i for i, t in enumerate(z["tickers"])}
    mix = {d: i for i, d in enumerate(pd.DatetimeIndex(z["month_end_ns"]))}
    a = out["ticker"].map(tix).to_numpy()
    m = out["date"].map(mix).to_numpy()
    assert len(out) == int(z["J12s1_present"].sum())
    assert bits_equal(out["adj_close"].to_numpy(), z["J12s1_PM"][m, a])
    assert bits_equal(out["ret_1m"].to_numpy(), z["J12s1_R"][m, a])
    assert bits_equal(out["mom_J"].to_numpy(), z["J12s1_M"][m, a])
    assert bits_equal(out["monthly_volume"].to_numpy(), z["J12s1_VOL"][m, a])


def test_monthly_replication_prints_reference_numbers(engine, tmp_path):
    import csmom
    df, z = _real_long()
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        res = csmom.monthly_replication(df, {}, plot_path=str(tmp_path / "cum.png"))
    assert len(res.mom_ret) == 70
    assert abs(res.mean - float(z["J12s1_mean"])) <= 1e-10 * abs(float(z["J12s1_mean"]))
    assert abs(res.sharpe - float(z["J12s1_sharpe"])) <= 1e-10 * abs(float(z["J12s1_sharpe"]))
    assert max_rel(res.cum.to_numpy(), z["J12s1_cum"]) <= 1e-10
    assert (tmp_path / "cum.png").exists()
    # the two printed lines, number formatting included (run_demo.py:72-73)
    printed = str(z["printed"]).splitlines()
    got = [ln for ln in buf.getvalue().splitlines() if ln.startswith(("Monthly", "Sharpe"))]
    assert got == [ln for ln in printed if ln.startswith(("Monthly", "Sharpe"))]


def test_ingestion_csv_to_engine(engine, tmp_path):
    """Cached CSVs -> csmom.fetch_daily (the reference's call, run_demo.py:196) ->
    monthly_replication on the GPU: the real-data numbers.  The CSVs are written here from the
    real-data fixture's present rows in the cache's column layout (data_io.py:23-73)."""
    import csmom
    df, z = _real_long()
    for t, g in df.groupby("ticker", sort=False):
        out = pd.DataFrame({"Date": g["date"].dt.strftime("%Y-%m-%d"), "Adj Close": g["adj_close"],
                            "Close": g["adj_close"], "Volume": g["volume"]})
        out.to_csv(tmp_path / f"{t}_daily.csv", index=False)
    daily = csmom.fetch_daily(list(z["tickers"]), start="2018-01-01", end="2024-12-31",
                              verbose=False, data_dir=str(tmp_path))
    assert len(daily) == len(df)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        res = csmom.monthly_replication(daily, {}, plot_path=None)
    assert len(res.mom_ret) == 70
    assert abs(res.mean - float(z["J12s1_mean"])) <= 1e-10 * abs(float(z["J12s1_mean"]))
    assert abs(res.sharpe - float(z["J12s1_sharpe"])) <= 1e-10 * abs(float(z["J12s1_sharpe"]))
    assert res.turnover is not None and "turn_avg" in res.turnover.columns


def test_assign_deciles_per_date_api(engine):
    import csmom
    d = load_golden("deciles")
    v, o, lab = d["values"], d["offsets"], d["labels"]
    for i in range(0, len(o) - 1, 97):
        x = pd.Series(v[o[i]:o[i + 1]], index=np.arange(o[i + 1] - o[i]) * 3)
        got = csmom.assign_deciles_per_date(x, n=10)
        ref = lab[o[i]:o[i + 1]]
        assert np.array_equal(got.to_numpy(dtype=np.float64), ref, equal_nan=True)
        assert got.index.equals(x.index)


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    import csmom
    from csmom import _lib
    monkeypatch.setattr(_lib, "_LIB", None)
    monkeypatch.setenv("CSMOM_LIB", str(tmp_path / "nope.so"))
    with pytest.raises(csmom.CsmUnavailable):
        csmom.Engine(0)


@pytest.mark.parametrize("name,J,skip", [("edge", 12, 1), ("edge", 3, 0), ("longwin", 24, 1),
                                         ("c1", 12, 1)])
@pytest.mark.parametrize("C", [2, 3, 7, 16])
def test_chunked_scan_equals_single_scan(engine, name, J, skip, C):
    z = load_golden(name)
    PM, _ = engine.month_end(_up(z["P"]), _up(z["month_start"].astype(np.int64)))
    R, M, NR = engine.momentum(PM, J, skip, with_ret=True, chunked=False)
    Rc, Mc, NRc = engine.momentum_chunked(PM, J, skip, chunks=C, with_ret=True)
    assert bits_equal(Rc.cpu().numpy(), R.cpu().numpy())
    assert bits_equal(Mc.cpu().numpy(), M.cpu().numpy())
    assert bits_equal(NRc.cpu().numpy(), NR.cpu().numpy())


def test_chunked_scan_with_tail_next_pm(engine):
    """next_pm (the price after the panel) reaches the pending row of the last chunk and of
    assets absent from all later chunks."""
    z = load_golden("edge")
    PM, _ = engine.month_end(_up(z["P"]), _up(z["month_start"].astype(np.int64)))
    npm = PM[-1].clone()
    _, M, NR = engine.momentum(PM[:-1].contiguous(), 12, 1, next_pm=npm)
    _, Mc, NRc = engine.momentum_chunked(PM[:-1].contiguous(), 12, 1, chunks=5, next_pm=npm)
    assert bits_equal(NRc.cpu().numpy(), NR.cpu().numpy())
    assert bits_equal(Mc.cpu().numpy(), M.cpu().numpy())


# ------------------------------------------------------------------ halo date shards
def _halo_equal(out, res, ew=True):
    M, NR, L, EW, CNT, LS, cnt = res
    assert bits_equal(M.cpu().numpy(), out.M.cpu().numpy())
    assert bits_equal(NR.cpu().numpy(), out.NR.cpu().numpy())
    assert torch.equal(L, out.L)
    assert torch.equal(CNT, out.CNT)
    if ew:
        assert bits_equal(EW.cpu().numpy(), out.EW.cpu().numpy())
        assert bits_equal(LS.cpu().numpy(), out.LS.cpu().numpy())
    return cnt


@pytest.mark.parametrize("J,skip", [(12, 1), (3, 0), (9, 2)])
@pytest.mark.parametrize("G", [2, 3, 5, 8])
def test_halo_virtual_shards_equal_unsharded(engine, J, skip, G):
    """Halo shards (k_shard_halo state + k_signal<SH> from it; the exchange and repair only for
    the assets the halo leaves uncertain) == one pass, bit for bit, on the reference-generated
    edge panel (late listings, delistings, absent and all-NaN months)."""
    from csmom.distributed import virtual_shards_halo
    z = load_golden("edge")
    P, ms = _up(z["P"]), z["month_start"].astype(np.int64)
    out = engine.run(P, _up(ms), J, skip, 10)
    _halo_equal(out, virtual_shards_halo(engine, P, ms, G, J, skip, 10))


@pytest.mark.parametrize("J,skip,G", [(24, 1, 3), (48, 1, 2), (48, 0, 4)])
def test_halo_shards_long_windows(engine, J, skip, G):
    from csmom.distributed import virtual_shards_halo
    z = load_golden("longwin")
    P, ms = _up(z["P"]), z["month_start"].astype(np.int64)
    out = engine.run(P, _up(ms), J, skip, 10)
    _halo_equal(out, virtual_shards_halo(engine, P, ms, G, J, skip, 10))


@pytest.mark.parametrize("G", [2, 7])
@pytest.mark.parametrize("H", [None, 0, 2])
@pytest.mark.parametrize("cols_wg,fold_repair", [(1, False), (1, True), (0, True)])
def test_halo_shards_sparse_panel(engine, G, H, cols_wg, fold_repair):
    """Gappy panel (25 % absent months, 15 % NaN months): most assets are flagged and go
    through the exchange; H = 0 (no halo at all) and H = 2 (shorter than the window) flag
    every asset with history -- still bit for bit.  The listed columns' fold and replay in one
    launch (shard_fix_cols, the default), and the fold + convergence-tested repair with the
    summary and repair one workgroup per column (month prices derived together into LDS) or one
    thread per column (tune cols_wg 0)."""
    from oracle.synth_np import make_panel
    from csmom.distributed import virtual_shards_halo
    pan = make_panel(512, 2600, seed=11, nan_day=0.05, absent_month=0.25, nan_month=0.15,
                     cents=True)
    P, ms = _up(pan["P"]), pan["month_start"].astype(np.int64)
    out = engine.run(P, _up(ms), 12, 1, 10, with_ret=True)
    lib = engine.lib
    try:
        assert lib.csm_tune(b"cols_wg", cols_wg) == 0
        res = virtual_shards_halo(engine, P, ms, G, 12, 1, 10, H=H, fold_repair=fold_repair)
    finally:
        lib.csm_tune(b"cols_wg", 1)
    cnt = _halo_equal(out, res, ew=False)
    assert cnt > 0


@pytest.mark.parametrize("G", [2, 7])
@pytest.mark.parametrize("j12", [1, 0])
def test_halo_shards_four_wave_blocks(engine, G, j12):
    """The halo rank's shard kernel in the C4 block shape, J = 12 with its product length fixed
    at compile time (the default) and with the runtime J: the one-GPU pass's bits."""
    from oracle.synth_np import make_panel
    from csmom.distributed import virtual_shards_halo
    pan = make_panel(1_000, 2600, seed=13, nan_day=0.05, absent_month=0.2, nan_month=0.1,
                     cents=True)
    P, ms = _up(pan["P"]), pan["month_start"].astype(np.int64)
    out = engine.run(P, _up(ms), 12, 1, 10, with_ret=True)
    lib = engine.lib
    try:
        assert lib.csm_tune(b"signal_bwf", 4) == 0
        assert lib.csm_tune(b"signal_j12", j12) == 0
        res = virtual_shards_halo(engine, P, ms, G, 12, 1, 10)
    finally:
        lib.csm_tune(b"signal_bwf", 0)
        lib.csm_tune(b"signal_j12", 1)
    _halo_equal(out, res, ew=False)


@pytest.mark.parametrize("G", [2, 5, 8])
def test_halo_shards_bucket_ids(engine, G):
    """Wide rows: halo shards write bucket ids (the repair rewrites the ids of replayed cells)
    and rank from them -- csm_pipeline's labels, counts and means bit for bit (the split pass
    on the shards, and on the whole panel too at these row counts), the oracle's labels; few
    assets need the exchange on this panel."""
    from oracle.synth_np import make_panel
    from csmom.distributed import virtual_shards_halo
    pan = make_panel(20_000, 1_400, seed=17, with_volume=False, nan_day=0.03, absent_month=0.05,
                     nan_month=0.05, cents=True)
    P, ms = _up(pan["P"]), pan["month_start"].astype(np.int64)
    out = engine.pipeline(P, _up(ms), 12, 1, 10)
    res = virtual_shards_halo(engine, P, ms, G, 12, 1, 10)
    _halo_equal(out, res)
    ref = O.pipeline(pan["P"], ms, 12, 1, 10)
    assert np.array_equal(res[2].cpu().numpy(), ref["L"])


def test_halo_flags_and_union(engine):
    """k_shard_halo's flags on hand-made assets; k_shard_need / k_shard_union bit layout."""
    from csmom.synth import bday_calendar
    days, ms_h, _ = bday_calendar("2001-01-01", 22 * 40)
    T_d, N = len(days), 256
    rng = np.random.default_rng(3)
    P = np.exp(np.cumsum(rng.normal(0, 0.01, (T_d, N)), 0)) * 50.0
    ABS = np.array([0x7FF4000000000001], dtype=np.uint64).view(np.float64)[0]
    H, T_m = 16, 20
    d_h, d_f = ms_h[H], ms_h[H + T_m]
    P[:, 1][:d_h] = ABS                       # listed at the shard start: no halo history
    P[:, 2][:ms_h[H - 5]] = ABS               # 5 halo months: fewer than J + skip + 1
    P[ms_h[H + T_m]:ms_h[H + T_m + 1], 3] = ABS   # no row in the forward month
    P[:, 4][d_h:] = ABS                       # delisted at the shard start (no forward row,
                                              # but no pending row either: not needed)
    msd = _up(ms_h[:H + T_m + 2].astype(np.int64))
    Pd = _up(P[:ms_h[H + T_m + 1]])
    carry, npm, flags = engine.shard_halo(Pd, msd, H, 1, 12, 1, before=True, after=True)
    f = flags.cpu().numpy()
    assert f[0] == 0 and f[1] == 1 and f[2] == 1 and f[3] == 2 and f[4] == 2
    assert O.is_absent(npm.cpu().numpy()[3:4]).all()
    PM, _, M, NR, st = engine.signal_shard_halo(Pd, msd[H:H + T_m + 1], 23, 12, 1, carry, npm)
    mask = engine.shard_need(flags, st, H).cpu().numpy().view(np.uint64)
    cand = mask[0] | mask[1]
    bits = [(int(cand[a >> 6]) >> (a & 63)) & 1 for a in range(N)]
    assert bits[:5] == [0, 1, 1, 1, 0] and sum(bits) == 3
    pres = [(int(mask[2][a >> 6]) >> (a & 63)) & 1 for a in range(N)]
    assert pres[:5] == [1, 1, 1, 1, 0] and sum(pres) == N - 1
    # three ranks with these bits: rank 1 has history before its halo (rank 0's head rows) for
    # assets 1 and 2, and later rows for asset 3's pending row; a cap of 2 overflows
    idx, cnt = engine.shard_union(torch.stack([engine.shard_need(flags, st, H)] * 3), N, 2)
    assert int(cnt.item()) == 3 and idx.cpu().numpy().tolist() == [1, 2]
    # one rank alone: no rank before or after it, so nothing needs the exchange
    idx, cnt = engine.shard_union(engine.shard_need(flags, st, H)[None], N, 2)
    assert int(cnt.item()) == 0


@pytest.fixture(scope="module")
def wide_gappy():
    """A panel wide enough for the four-wave shard kernel (and so the fused halo prologue), with
    late listings, delistings, NaN days, absent and all-NaN months (walks back in the halo)."""
    from oracle.synth_np import make_panel
    pan = make_panel(96_000, 1_300, seed=23, with_volume=False, late=0.1, delist=0.1,
                     nan_day=0.03, absent_month=0.05, nan_month=0.05, cents=True)
    return _up(pan["P"]), pan["month_start"].astype(np.int64)


@pytest.mark.parametrize("G", [3, 8])
def test_fused_halo_prologue_equals_two_launches(engine, wide_gappy, G):
    """csm_signal_halo (the halo months' prices, state and flags computed in the shard kernel's
    prologue) against csm_shard_halo + csm_signal_shard_halo on every rank of a G-way split:
    flags, PM, M, NR, ids and the end-state record bit for bit; and the whole virtual halo pass
    (fused prologue + shard_fix_cols) against the two-launch pass with the convergence repair
    and against the one-GPU pipeline: M, NR, labels, counts, decile means and long-short."""
    from csmom.distributed import halo_months, halo_slices, virtual_shards_halo
    P, ms = wide_gappy
    N = P.shape[1]
    J, skip = 12, 1
    H = halo_months(J, skip)
    for (d0, d1, hm, F, h0, m0, m1) in halo_slices(ms, G, H):
        Pg = P[d0:d1].contiguous()
        msg = torch.from_numpy(ms[h0:m1 + F + 1] - d0).to("cuda:0")
        msh = msg[hm:hm + (m1 - m0) + 1]
        maxd = int(np.diff(ms[m0:m1 + 1]).max())
        assert engine.halo_fused_ok(N, maxd)
        before, after = h0 > 0, m1 + F < len(ms) - 1
        ids_a = engine.empty((m1 - m0, N), torch.int16)
        ids_b = engine.empty((m1 - m0, N), torch.int16)
        carry, npm, fl_b = engine.shard_halo(Pg, msg, hm, F, J, skip, before=before, after=after)
        PMb, _, Mb, NRb, stb = engine.signal_shard_halo(Pg, msh, maxd, J, skip, carry, npm,
                                                        ids=ids_b)
        PMa, _, Ma, NRa, sta, fl_a = engine.signal_halo(Pg, msg, hm, F, maxd, J, skip,
                                                        before=before, after=after, ids=ids_a)
        assert torch.equal(fl_a, fl_b)
        for x, y in ((PMa, PMb), (Ma, Mb), (NRa, NRb), (sta.t, stb.t)):
            assert bits_equal(x.cpu().numpy(), y.cpu().numpy())
        assert torch.equal(ids_a, ids_b)
    out = engine.pipeline(P, _up(ms), J, skip, 10)
    a = virtual_shards_halo(engine, P, ms, G, J, skip, 10, fused_halo=True)
    b = virtual_shards_halo(engine, P, ms, G, J, skip, 10, fold_repair=True, fused_halo=False)
    assert a[6] > 0   # listed columns went through shard_fix_cols
    for res in (a, b):
        _halo_equal(out, res)
