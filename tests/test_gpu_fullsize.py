"""GPU parity at the BASELINE configs' workload sizes (C3, C4, C5), the bench's own layouts.

C4: the 100,000-asset x 10,000-day panel is generated in HBM exactly as bench.py does and run
through the benchmarked path (csm_pipeline: fused signal with bucket ids -> labels + decile
means -> long-short).  The scan is per asset, so a column subset checked against the oracle
is exact for those columns: month prices, mom_J and next_ret bit for bit on all 100,000 columns
(20,000-column blocks); labels on EVERY date (all 461) are the oracle's qcut of the oracle's
mom_J; counts exact and decile means / long-short within 1e-10 of the oracle's portfolio.
C3: the 5,000 x 6,522-day value-weighted 16-strategy grid with square-root-impact costs, every
(J, K), against the portfolio oracle (rules E1-E5).  C5: SweepRunner.run_bootstrap at the
bench's layout (5,000 assets, 300 months, 16 strategies, turnover + spread costs) in each batch
geometry the bench runs (200 panels on one GPU, 125 per rank on 8, and 100); sampled panels'
summary rows against the oracle stages, and the accounting branch each batch took.
"""
import numpy as np
import pytest
import torch

from conftest import bits_equal, max_rel
from oracle import csmom_oracle as O
from oracle import portfolio_oracle as PO

pytestmark = pytest.mark.gpu
REL = 1e-10


def _labels_ref(rows, n_bins=10):
    out = np.full(rows.shape, -1, dtype=np.int8)
    for t, row in enumerate(rows):
        v = ~np.isnan(row)
        if v.any():
            lab = O.qcut_labels(row[v], n_bins)
            out[t, v] = np.where(np.isnan(lab), -1, lab).astype(np.int8)
    return out


@pytest.fixture(scope="module")
def c4(engine):
    import csmom  # noqa: F401
    from csmom.synth import bday_calendar, make_device_panel
    N, T_d = 100_000, 10_000
    days, ms_h, _ = bday_calendar("1985-01-01", T_d)
    pan = make_device_panel(N, days, ms_h, seed=4 * 1000, device="cuda:0",
                            shard=(0, 1, 4, float(T_d)))          # bench.py's N = 1 panel
    out = engine.pipeline(pan.P, pan.month_start, 12, 1, 10, with_pm=True)
    torch.cuda.synchronize()
    return N, T_d, ms_h, pan, out


@pytest.fixture(scope="module")
def c4_oracle(c4):
    """The oracle's month prices, mom_J and next_ret of ALL 100,000 columns, in blocks of 20,000
    columns (the scan is per asset, so a column block is exact; ~1.6 GB of host panel at a time)."""
    N, T_d, ms_h, pan, out = c4
    T_m = len(ms_h) - 1
    PM_r = np.empty((T_m, N))
    M_r = np.empty((T_m, N))
    NR_r = np.empty((T_m, N))
    for c0 in range(0, N, 20_000):
        c1 = min(N, c0 + 20_000)
        P_h = pan.P[:, c0:c1].contiguous().cpu().numpy()
        PM_r[:, c0:c1], _ = O.month_end(P_h, ms_h)
        _, M_r[:, c0:c1], NR_r[:, c0:c1], _ = O.momentum_scan(PM_r[:, c0:c1], 12, 1)
        del P_h
    return PM_r, M_r, NR_r


def test_c4_columns_bit_exact(c4, c4_oracle):
    """features.py:34-52 + run_demo.py:48 on every one of the 100,000 columns: month price, mom_J
    and next_ret bit for bit against the oracle."""
    N, T_d, ms_h, pan, out = c4
    PM_r, M_r, NR_r = c4_oracle
    assert bits_equal(out.PM.cpu().numpy(), PM_r)
    assert (O.is_absent(out.PM.cpu().numpy()) == O.is_absent(PM_r)).all()
    assert bits_equal(out.M.cpu().numpy(), M_r)
    assert bits_equal(out.NR.cpu().numpy(), NR_r)


def test_c4_labels_every_date_and_means(c4, c4_oracle):
    """run_demo.py:18-29,46,55-67: the labels of all 461 dates are the oracle's qcut of the
    ORACLE's mom_J; counts exact; decile means / long-short within 1e-10 of the oracle's
    portfolio on the oracle's next_ret."""
    N, T_d, ms_h, pan, out = c4
    _, M_r, NR_r = c4_oracle
    T_m = M_r.shape[0]
    assert T_m == 461
    L_ref = _labels_ref(M_r)
    L_h = out.L.cpu().numpy()
    bad = np.nonzero((L_h != L_ref).any(axis=1))[0]
    assert len(bad) == 0, f"label mismatch on dates {bad[:10]}"
    assert np.array_equal(out.NV.cpu().numpy(), (~np.isnan(M_r)).sum(axis=1))
    EW_r, CNT_r, LS_r = O.portfolio_ew(L_ref, NR_r, 10)
    assert np.array_equal(out.CNT.cpu().numpy(), CNT_r)
    ew, ls = out.EW.cpu().numpy(), out.LS.cpu().numpy()
    assert np.array_equal(np.isnan(ew), np.isnan(EW_r)) and max_rel(ew, EW_r) <= REL
    assert np.array_equal(np.isnan(ls), np.isnan(LS_r)) and max_rel(ls, LS_r) <= REL


def test_c4_halo_shards_bench_geometry(engine, c4):
    """The benched 8-way date-shard geometry on the C4 bench panel itself (bench.py --gpus 8
    --shard-mode halo, run here as virtual shards on one device with the collectives replaced
    by stacks): every rank's halo state + k_signal<SH>, the need bits / union list, the listed
    columns' records, fold and repair, and the decile pass of its ~58 rows -- which takes the
    split pass (plan / chunked sweep / finish), while the one-GPU pipeline's 461 rows take the
    merged pass.  M, NR, labels, counts, decile means and long-short bit for bit the one-GPU
    csm_pipeline (features.py:44-52, run_demo.py:18-29,46-67); the listed columns fit the list
    width the rank pass sizes (no fallback)."""
    from csmom.distributed import fallback_cap, halo_slices, halo_months, virtual_shards_halo
    N, T_d, ms_h, pan, out = c4
    G = 8
    rows = [m1 - m0 for (_, _, _, _, _, m0, m1) in halo_slices(np.asarray(ms_h), G,
                                                                 halo_months(12, 1))]
    assert max(rows) * 2 <= engine.cus < 2 * out.L.shape[0]   # split on ranks, merged whole
    M, NR, L, EW, CNT, LS, cnt = virtual_shards_halo(engine, pan.P, ms_h, G, 12, 1, 10)
    assert 1 <= cnt <= fallback_cap(N), cnt                    # the listed-column path ran
    assert bits_equal(M.cpu().numpy(), out.M.cpu().numpy())
    assert bits_equal(NR.cpu().numpy(), out.NR.cpu().numpy())
    assert torch.equal(L, out.L) and torch.equal(CNT, out.CNT)
    assert bits_equal(EW.cpu().numpy(), out.EW.cpu().numpy())
    assert bits_equal(LS.cpu().numpy(), out.LS.cpu().numpy())


def test_c4_default_decile_kernel_agrees(engine, c4):
    """The streaming decile kernel (no ids) on the same mom_J: identical labels and counts."""
    N, T_d, ms_h, pan, out = c4
    L, EW, CNT, NV = engine.deciles(out.M, out.NR, 10, with_nv=True)
    assert torch.equal(L, out.L) and torch.equal(CNT, out.CNT) and torch.equal(NV, out.NV)
    a, b = EW.cpu().numpy(), out.EW.cpu().numpy()
    assert np.array_equal(np.isnan(a), np.isnan(b)) and max_rel(a, b) <= 1e-13


def test_c2_c3_full_panel_bit_exact(engine):
    """C2 / C3's panel (5,000 assets x 6,522 days, every column): the month-end kernel's month
    prices, the time-chunked scan's mom_J / next_ret (+ ids) and the chunked multi-J scan of
    the sweep against the oracle's month-end and scan, bit for bit."""
    from csmom.synth import bday_calendar, make_device_panel
    N, T_d = 5_000, 6_522
    days, ms_h, _ = bday_calendar("2000-01-03", T_d)
    pan = make_device_panel(N, days, ms_h, seed=2 * 1000, device="cuda:0")
    PM, _ = engine.month_end(pan.P, pan.month_start)
    PM_r, _ = O.month_end(pan.P.cpu().numpy(), ms_h)
    assert bits_equal(PM.cpu().numpy(), PM_r)
    T_m = PM.shape[0]
    IDS = engine.empty((T_m, N), torch.int16)
    _, M, NR = engine.momentum_chunked(PM, 12, 1, ids=IDS)
    _, M_r, NR_r, _ = O.momentum_scan(PM_r, 12, 1)
    assert bits_equal(M.cpu().numpy(), M_r) and bits_equal(NR.cpu().numpy(), NR_r)
    outs = engine.momentum_multi(PM, (3, 6, 9, 12), 1, with_ids=True,
                                 chunks=engine.default_chunks(T_m, N, 12, 1))
    for J, (Mq, NRq, _) in zip((3, 6, 9, 12), outs):
        _, Mj, NRj, _ = O.momentum_scan(PM_r, J, 1)
        assert bits_equal(Mq.cpu().numpy(), Mj), J
        assert bits_equal(NRq.cpu().numpy(), NRj), J


# ------------------------------------------------------------------------------------ C3
@pytest.fixture(scope="module")
def c3(engine):
    from csmom.synth import bday_calendar, make_device_panel
    N, T_d = 5_000, 6_522
    days, ms_h, _ = bday_calendar("2000-01-03", T_d)
    seed = 4 * 1000 + 3
    pan = make_device_panel(N, days, ms_h, seed=seed, device="cuda:0")
    g = torch.Generator(device="cuda:0")
    g.manual_seed(seed)
    shares = torch.exp(torch.randn(N, generator=g, device="cuda:0", dtype=torch.float64) + 16.0)
    turn = torch.rand(N, generator=g, device="cuda:0", dtype=torch.float64) * 0.018 + 0.002
    PM, _ = engine.month_end(pan.P, pan.month_start)
    W = PM.abs() * shares
    ADV = W * turn
    return PM, W, ADV


@pytest.mark.parametrize("J", [3, 6, 9, 12])
def test_c3_value_weighted_grid_with_impact_costs(engine, c3, J):
    import csmom
    PM, W, ADV = c3
    cfg = csmom.SweepConfig(Js=(3, 6, 9, 12), Ks=(3, 6, 9, 12), skip=1, aum=1e8)
    _, M, NR = engine.momentum(PM, J, 1)
    L, _, _, _ = engine.deciles(M, None, 10)
    PM_h, W_h, ADV_h = PM.cpu().numpy(), W.cpu().numpy(), ADV.cpu().numpy()
    _, M_r, NR_r, _ = O.momentum_scan(PM_h, J, 1)
    assert bits_equal(M.cpu().numpy(), M_r) and bits_equal(NR.cpu().numpy(), NR_r)
    L_r = O.assign_deciles(M_r, 10)
    assert np.array_equal(L.cpu().numpy(), L_r)
    outs = engine.portfolio_multi(L, NR, 10, Ks=cfg.Ks, W=W, half_spread=cfg.half_spread,
                                  k_impact=cfg.k_impact, aum=cfg.aum, ADV=ADV)
    for K in cfg.Ks:
        ref = PO.portfolio(L_r, NR_r, 10, K=K, W=W_h, half_spread=cfg.half_spread,
                           k_impact=cfg.k_impact, aum=cfg.aum, ADV=ADV_h)
        for f in ("PR", "LS", "TURN", "COST", "NET"):
            g = getattr(outs[K], f).cpu().numpy().reshape(ref[f].shape)
            assert np.array_equal(np.isnan(g), np.isnan(ref[f])), (J, K, f)
            assert max_rel(g, ref[f]) <= REL, (J, K, f, max_rel(g, ref[f]))


def test_c3_sweep_runner_summary(engine, c3):
    """The bench's C3 step (SweepRunner.run_batch with value weights and ADV) gives the summary
    rows of the per-(J, K) device portfolios."""
    import csmom
    PM, W, ADV = c3
    cfg = csmom.SweepConfig(Js=(3, 6, 9, 12), Ks=(3, 6, 9, 12), skip=1, aum=1e8)
    summ, series = csmom.SweepRunner(engine, cfg).run_batch(PM, 1, W=W, ADV=ADV)
    assert tuple(summ.shape) == (1, 16, 7)
    for s, (J, K) in enumerate(cfg.strategies):
        o = series[(J, K)]   # (strided views of the joined outputs)
        c = lambda x: x.contiguous()
        one = engine.summary(c(o.LS), c(o.TURN), c(o.COST), c(o.NET))[0, 0]
        assert bits_equal(summ[0, s].cpu().numpy(), one.cpu().numpy()), (J, K)


def test_c3_bench_step_vs_oracle(engine, c3):
    """The C3 step bench.py times, exactly (bench.py sweep_main's step_defer): month prices ->
    value weights / dollar ADV -> SweepRunner(SweepConfig(Js=Ks=(3, 6, 9, 12), skip=1,
    aum=1e8)).run_batch(PM, 1, W, ADV, defer=True) on its defaults -- the four look-backs
    joined, the chunked multi-J scan with ids, the legs-mode decile pass on ids, the legs-only
    grouped value-weight accounting (k_turnover_vwg) and the device summary.  Every (J, K) row
    of the summary table against the oracle chain (features.py:44-52 scan, run_demo.py:18-29
    qcut, portfolio_oracle's overlapping K-month value-weighted legs with the square-root-impact
    cost of execution_models.py:4-12, the summary of utils.py:8-16): months exact, every other
    field within 1e-10 relative (fp64 sums in another fixed order)."""
    import csmom
    PM, W, ADV = c3
    cfg = csmom.SweepConfig(Js=(3, 6, 9, 12), Ks=(3, 6, 9, 12), skip=1, aum=1e8)
    runner = csmom.SweepRunner(engine, cfg)
    summ, _, flag = runner.run_batch(PM, 1, W=W, ADV=ADV, defer=True)
    torch.cuda.synchronize()
    assert flag is not None and int(flag.item()) == 0   # the legs-only branch the bench times
    got_all = summ.cpu().numpy()
    assert got_all.shape == (1, 16, 7)
    PM_h, W_h, ADV_h = PM.cpu().numpy(), W.cpu().numpy(), ADV.cpu().numpy()
    T_m = PM_h.shape[0]
    for J in cfg.Js:
        _, M_r, NR_r, _ = O.momentum_scan(PM_h, J, cfg.skip)
        L_r = O.assign_deciles(M_r, cfg.n_bins)
        for K in cfg.Ks:
            r = PO.portfolio(L_r, NR_r, cfg.n_bins, K=K, W=W_h, half_spread=cfg.half_spread,
                             k_impact=cfg.k_impact, aum=cfg.aum, ADV=ADV_h)
            x = lambda f: r[f].reshape(1, T_m, 1)
            ref = _summary_rows(x("LS"), x("TURN"), x("COST"), x("NET"))[0, 0]
            got = got_all[0, cfg.strategies.index((J, K))]
            assert np.array_equal(np.isnan(got), np.isnan(ref)), (J, K)
            assert got[0] == ref[0], (J, K, got[0], ref[0])          # months
            m = ~np.isnan(ref)
            err = np.abs(got[m] - ref[m]) / np.maximum(np.abs(ref[m]), 1e-12)
            assert err.max() <= REL, (J, K, float(err.max()))


# ------------------------------------------------------------------------------------ C5
# Geometries of the C5 bench (bench.py --config c5): 1000 panels in device batches of 200 on one
# GPU (the default), 125 panels per rank on 8 ranks (one batch of 125), and batches of 100 (the
# round-4 default).  Whether a batch takes the grouped shared-return accounting (sweep.py
# _boot_batch, "jsg") depends on the portfolio chunk plan at that width, so each geometry is
# checked against the oracle on its own and the branch it took is asserted.
C5_GEOMETRIES = {100: [0, 7, 13, 29, 42, 57, 64, 86, 93, 99],
                 200: [0, 13, 57, 99, 100, 128, 150, 177, 198, 199],
                 125: [0, 7, 31, 62, 63, 64, 88, 100, 117, 124]}


@pytest.fixture(scope="module")
def c5_base(engine):
    from csmom.synth import bday_calendar, make_device_panel
    N, T_d = 5_000, 6_522
    days, ms_h, _ = bday_calendar("2000-01-03", T_d)
    pan = make_device_panel(N, days, ms_h, seed=4 * 1000 + 5, device="cuda:0")
    PM0, _ = engine.month_end(pan.P, pan.month_start)
    R0, _, _ = engine.momentum(PM0, 12, 1, with_ret=True)
    torch.cuda.synchronize()
    return R0, R0.cpu().numpy()


@pytest.fixture(scope="module", params=sorted(C5_GEOMETRIES))
def c5(engine, c5_base, request):
    """One device batch of `batch` panels through SweepRunner.run_bootstrap, as the bench runs
    it; also the accounting branch the batch took."""
    import csmom
    R0, _ = c5_base
    batch = request.param
    cfg = csmom.SweepConfig(Js=(3, 6, 9, 12), Ks=(3, 6, 9, 12), skip=1, aum=1e8)
    runner = csmom.SweepRunner(engine, cfg)
    summ = runner.run_bootstrap(R0, batch, seed=5000, mean_block=6.0, batch=batch)
    torch.cuda.synchronize()
    return cfg, R0, summ.cpu().numpy(), batch, list(runner.boot_paths)


def _oracle_panel_summary(cfg, R_h, b):
    T_m, N = R_h.shape
    src = PO.bootstrap_indices(T_m, 1, 5000, 6.0, b0=b)
    pm = PO.bootstrap_panel(R_h, src).reshape(T_m, N)
    rows = []
    for J in cfg.Js:
        _, M, NR, _ = O.momentum_scan(pm, J, cfg.skip)
        L = O.assign_deciles(M, cfg.n_bins)
        for K in cfg.Ks:
            r = PO.portfolio(L, NR, cfg.n_bins, K=K, half_spread=cfg.half_spread,
                             k_impact=cfg.k_impact, aum=cfg.aum)
            x = lambda f: r[f].reshape(1, T_m, 1)
            rows.append(_summary_rows(x("LS"), x("TURN"), x("COST"), x("NET"))[0, 0])
    return np.stack(rows)


def _summary_rows(LS, TURN, COST, NET, freq=12.0):
    from test_gpu_portfolio import _summary_ref
    return _summary_ref(LS, TURN, COST, NET, freq)


def test_c5_shape_and_branch(engine, c5):
    """Every bench geometry runs one batch, through the grouped shared-return accounting: its
    chunk plan at the batch width equals the plan of the four look-backs side by side (C5: one
    cohort chunk and one turnover chunk either way)."""
    cfg, R0, summ, batch, paths = c5
    assert summ.shape == (batch, 16, 7)
    assert np.isfinite(summ[..., :3]).all()
    assert paths == ["jsg"], paths
    T_m, N = R0.shape
    assert (engine.portfolio_plan(T_m, batch, N, 10, 12)
            == engine.portfolio_plan(T_m, 4 * batch, N, 10, 12))


@pytest.mark.parametrize("k", range(10))
def test_c5_sampled_panels_vs_oracle(c5, c5_base, k):
    """Ten of each batch's bootstrap panels: every (J, K) summary row against the oracle stages
    within north_star's 1e-10 relative (fp64 sums in another order; months exact)."""
    cfg, R0, summ, batch, _ = c5
    b = C5_GEOMETRIES[batch][k]
    ref = _oracle_panel_summary(cfg, c5_base[1], b)
    got = summ[b]
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    assert np.array_equal(got[:, 0], ref[:, 0])                 # months per strategy
    m = ~np.isnan(ref)
    scale = np.maximum(np.abs(ref[m]), 1e-12)
    err = np.abs(got[m] - ref[m]) / scale
    assert err.max() <= 1e-10, (batch, b, float(err.max()))


def test_c5_boot_scan_equals_materialised(engine, c5):
    """The bench path (csm_boot_scan, SweepConfig.boot_scan) against csm_bootstrap ->
    multi-J scan -> decile pass on the whole C5 batch: the summary table bit for bit."""
    import csmom
    from dataclasses import replace
    cfg, R0, summ, batch, _ = c5
    off = csmom.SweepRunner(engine, replace(cfg, boot_scan=False)).run_bootstrap(
        R0, batch, seed=5000, mean_block=6.0, batch=batch).cpu().numpy()
    assert bits_equal(summ, off)


def test_c3_joined_js_equal_per_j(engine, c3):
    """The bench's C3 step joins the four Js into one decile pass and one accounting launch set
    (SweepConfig.join_js): the summary table and every series equal the per-J launches' bit for
    bit (batches of up to four panels share one chunk plan, portfolio.hip pf_plan)."""
    import csmom
    from dataclasses import replace
    PM, W, ADV = c3
    cfg = csmom.SweepConfig(Js=(3, 6, 9, 12), Ks=(3, 6, 9, 12), skip=1, aum=1e8)
    a, sa = csmom.SweepRunner(engine, cfg).run_batch(PM, 1, W=W, ADV=ADV)
    b, sb = csmom.SweepRunner(engine, replace(cfg, join_js=False)).run_batch(PM, 1, W=W, ADV=ADV)
    a, b = a.cpu().numpy(), b.cpu().numpy()
    assert bits_equal(a, b)
    for key in cfg.strategies:
        for f in ("PR", "LS", "TURN", "COST", "NET"):
            x, y = getattr(sa[key], f), getattr(sb[key], f)
            assert x.shape == y.shape, (key, f)
            assert bits_equal(x.cpu().numpy(), y.cpu().numpy()), (key, f)


def test_c3_two_panel_batch_joins_only_on_equal_plans(engine, c3):
    """A 2-panel C3 batch (T_m * B < JOIN_ROWS): the four look-backs side by side would plan
    two turnover chunks against four per J (pf_plan treats batches below four panels as four),
    so the batch is NOT joined and its table equals the per-J launches' bit for bit; the
    single-panel batch (plans equal) is joined."""
    import csmom
    from dataclasses import replace
    PM, W, ADV = c3
    T_m, N = PM.shape
    PM2 = torch.cat([PM, PM * 1.5], 1).contiguous()
    W2 = torch.cat([W, W * 0.5], 1).contiguous()
    ADV2 = torch.cat([ADV, ADV * 0.5], 1).contiguous()
    cfg = csmom.SweepConfig(Js=(3, 6, 9, 12), Ks=(3, 6, 9, 12), skip=1, aum=1e8)
    run = csmom.SweepRunner(engine, cfg)
    assert run._joined(T_m, 1, N)
    assert not run._joined(T_m, 2, N)
    assert engine.portfolio_plan(T_m, 2, N, 10, 12) != engine.portfolio_plan(T_m, 8, N, 10, 12)
    a, _ = run.run_batch(PM2, 2, W=W2, ADV=ADV2)
    b, _ = csmom.SweepRunner(engine, replace(cfg, join_js=False)).run_batch(PM2, 2, W=W2, ADV=ADV2)
    assert bits_equal(a.cpu().numpy(), b.cpu().numpy())
