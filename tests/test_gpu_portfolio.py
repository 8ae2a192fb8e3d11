"""GPU: csm_portfolio (K-overlap, value weights, turnover, costs) and csm_bootstrap against the
portfolio oracle (rules E1..E6).  Bar: the bootstrap's source months and month prices are
bit-exact (integer hashing, sequential fp64 products); portfolio returns, turnover and costs
agree within 1e-10 relative (fp64 sums in a different order)."""
import numpy as np
import pytest
import torch

from conftest import bits_equal, load_golden, max_rel
from oracle import csmom_oracle as O
from oracle import portfolio_oracle as PO

pytestmark = pytest.mark.gpu
REL = 1e-10


def _up(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to("cuda:0")


def _labels(engine, name, J=12, skip=1):
    z = load_golden(name)
    P = z["P"]
    ms = z["month_start"].astype(np.int64)
    PM, _ = engine.month_end(_up(P), _up(ms))
    R, M, NR = engine.momentum(PM, J, skip, with_ret=True)
    L, _, _, _ = engine.deciles(M, None, 10)
    return L, NR, R, PM


def _close(got, ref, what, rel=REL):
    g = got.cpu().numpy() if isinstance(got, torch.Tensor) else got
    assert np.array_equal(np.isnan(g), np.isnan(ref)), what
    m = ~np.isnan(ref)
    scale = np.maximum(np.abs(ref[m]), 1e-12)
    assert (np.abs(g[m] - ref[m]) <= rel * scale + 1e-15).all(), (what, max_rel(g, ref))


@pytest.mark.parametrize("K", [1, 3, 6, 12])
@pytest.mark.parametrize("vw", [False, True])
def test_portfolio_vs_oracle(engine, K, vw):
    L, NR, _, PM = _labels(engine, "c1")
    Lh, NRh = L.cpu().numpy(), NR.cpu().numpy()
    rng = np.random.default_rng(K * 10 + vw)
    T_m, N = Lh.shape
    W = None
    if vw:
        W = np.abs(PM.cpu().numpy()) * rng.uniform(1e5, 1e7, N)   # price x shares
        W[rng.random(W.shape) < 0.01] = np.nan
    ADV = rng.uniform(1e5, 1e8, (T_m, N))
    SIG = rng.uniform(0.005, 0.05, (T_m, N))
    SIG[rng.random(SIG.shape) < 0.02] = np.nan
    ref = PO.portfolio(Lh, NRh, 10, K=K, W=W, aum=5e6, ADV=ADV, SIG=SIG)
    out = engine.portfolio(L, NR, 10, K=K, W=None if W is None else _up(W), aum=5e6,
                           ADV=_up(ADV), SIG=_up(SIG))
    _close(out.PR, ref["PR"], "PR")
    _close(out.LS, ref["LS"], "LS")
    _close(out.TURN, ref["TURN"], "TURN")
    _close(out.COST, ref["COST"], "COST")
    _close(out.NET, ref["NET"], "NET")


def test_portfolio_k1_equal_weight_is_reference_path(engine):
    """K = 1, equal weight, no costs: the same numbers as the fused decile means (the
    reference's run_demo.py:49-67 path) and the golden fixture."""
    z = load_golden("c1")
    L, NR, _, _ = _labels(engine, "c1")
    _, EW, CNT, _ = engine.deciles(*_mom(engine, "c1"), 10)
    out = engine.portfolio(L, NR, 10, K=1, with_costs=False)
    _close(out.PR[:, 0, :], z["J12s1_EW"], "PR vs fixture")
    _close(out.LS[:, 0], z["J12s1_LS"], "LS vs fixture")
    _close(out.PR[:, 0, :], EW.cpu().numpy(), "PR vs k_deciles EW")


def _mom(engine, name):
    z = load_golden(name)
    PM, _ = engine.month_end(_up(z["P"]), _up(z["month_start"].astype(np.int64)))
    _, M, NR = engine.momentum(PM, 12, 1)
    return M, NR


def test_portfolio_batched_panels(engine):
    L, NR, _, _ = _labels(engine, "c1")
    Lh, NRh = L.cpu().numpy(), NR.cpu().numpy()
    perm = np.random.default_rng(3).permutation(Lh.shape[1])
    L3 = np.stack([Lh, Lh[:, perm], Lh[:, ::-1]], axis=1)
    NR3 = np.stack([NRh, NRh[:, perm], NRh[:, ::-1]], axis=1)
    T_m, B, N = L3.shape
    ref = PO.portfolio(L3, NR3, 10, K=6)
    out = engine.portfolio(_up(L3.reshape(T_m, B * N)), _up(NR3.reshape(T_m, B * N)), 10, K=6,
                           B=B)
    _close(out.PR, ref["PR"], "PR")
    _close(out.TURN, ref["TURN"], "TURN")
    _close(out.NET, ref["NET"], "NET")
    # every panel is a permutation of the same cross-sections: identical returns
    pr = out.PR.cpu().numpy()
    assert max_rel(pr[:, 1], pr[:, 0]) <= 1e-12 and max_rel(pr[:, 2], pr[:, 0]) <= 1e-12


def test_portfolio_rejects_bad_args(engine):
    import csmom
    L, NR, _, _ = _labels(engine, "c1")
    with pytest.raises(csmom.CsmError):
        engine.portfolio(L, NR, 7, K=1)          # unsupported n_bins
    with pytest.raises(ValueError):
        engine.portfolio(L, NR, 10, K=1, B=7)    # row width not a multiple of B


@pytest.mark.parametrize("B,b0", [(5, 0), (3, 17)])
def test_bootstrap_bit_exact(engine, B, b0):
    _, _, R, _ = _labels(engine, "c1")
    Rh = R.cpu().numpy()
    T_m, N = Rh.shape
    src, PMb = engine.bootstrap(R, B, b0=b0, seed=5000, mean_block=6.0)
    ref_src = PO.bootstrap_indices(T_m, B, 5000, 6.0, b0=b0)
    assert np.array_equal(src.cpu().numpy().astype(np.int64), ref_src)
    ref = PO.bootstrap_panel(Rh, ref_src)
    got = PMb.cpu().numpy().reshape(T_m, B, N)
    assert (O.is_absent(got) == O.is_absent(ref)).all()
    assert bits_equal(got, ref)


def test_bootstrap_sweep_end_to_end(engine):
    """C5 in miniature: bootstrap panels -> scan -> deciles -> K-overlap portfolios with costs,
    all batched as [T_m][B*N], against the oracle stage by stage."""
    _, _, R, _ = _labels(engine, "c1")
    Rh = R.cpu().numpy()
    T_m, N = Rh.shape
    B = 4
    src, PMb = engine.bootstrap(R, B, b0=100, seed=5000, mean_block=6.0)
    pm_ref = PO.bootstrap_panel(Rh, PO.bootstrap_indices(T_m, B, 5000, 6.0, b0=100))
    for J, K in ((3, 1), (12, 6)):
        _, M, NR = engine.momentum(PMb, J, 1)
        L, _, _, _ = engine.deciles(M.view(T_m * B, N), None, 10)
        L = L.view(T_m, B * N)
        out = engine.portfolio(L, NR, 10, K=K, B=B)
        _, Mr, NRr, _ = O.momentum_scan(pm_ref.reshape(T_m, B * N), J, 1)
        assert bits_equal(M.cpu().numpy(), Mr) and bits_equal(NR.cpu().numpy(), NRr)
        Lr = O.assign_deciles(Mr.reshape(T_m * B, N), 10).reshape(T_m, B, N)
        assert np.array_equal(L.cpu().numpy().reshape(T_m, B, N), Lr)
        ref = PO.portfolio(Lr, NRr.reshape(T_m, B, N), 10, K=K)
        _close(out.PR, ref["PR"], f"PR J{J}K{K}")
        _close(out.NET, ref["NET"], f"NET J{J}K{K}")


def test_sweep_runner_gpu_vs_oracle(engine):
    """SweepRunner on the Engine (bootstrap -> scan -> qcut -> portfolios, batched) against
    the same orchestration on the oracle stages."""
    import csmom
    from test_sweep_gloo import OracleSweepStages
    _, _, R, _ = _labels(engine, "c1")
    cfg = csmom.SweepConfig(Js=(3, 12), Ks=(1, 6), skip=1)
    got = csmom.SweepRunner(engine, cfg).run_bootstrap(R, 5, seed=5000, mean_block=6.0,
                                                       batch=3).cpu().numpy()
    ref = csmom.SweepRunner(OracleSweepStages(), cfg).run_bootstrap(
        R.cpu(), 5, seed=5000, mean_block=6.0, batch=5).numpy()
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    assert np.array_equal(got[..., 0], ref[..., 0])
    m = ~np.isnan(ref)
    assert np.allclose(got[m], ref[m], rtol=1e-9, atol=1e-13)


@pytest.mark.parametrize("n_bins", [2, 5, 20])
def test_portfolio_nbins(engine, n_bins):
    z = load_golden("c1")
    PM, _ = engine.month_end(_up(z["P"]), _up(z["month_start"].astype(np.int64)))
    _, M, NR = engine.momentum(PM, 6, 1)
    L, _, _, _ = engine.deciles(M, None, n_bins)
    ref = PO.portfolio(L.cpu().numpy(), NR.cpu().numpy(), n_bins, K=4)
    out = engine.portfolio(L, NR, n_bins, K=4)
    _close(out.PR, ref["PR"], "PR")
    _close(out.LS, ref["LS"], "LS")
    _close(out.TURN, ref["TURN"], "TURN")


def test_portfolio_wide_panel_single_chunk(engine):
    """Wide batches (many (t, b) rows) take the one-chunk, cohort-loop plan; narrow ones the
    chunked, cohort-parallel plan: both against the oracle."""
    L, NR, _, _ = _labels(engine, "c1")
    Lh, NRh = L.cpu().numpy(), NR.cpu().numpy()
    B = 16
    L16 = np.stack([np.roll(Lh, i, axis=1) for i in range(B)], axis=1)
    NR16 = np.stack([np.roll(NRh, i, axis=1) for i in range(B)], axis=1)
    T_m, _, N = L16.shape
    ref = PO.portfolio(L16, NR16, 10, K=12)
    out = engine.portfolio(_up(L16.reshape(T_m, B * N)), _up(NR16.reshape(T_m, B * N)), 10,
                           K=12, B=B)
    _close(out.PR, ref["PR"], "PR")
    _close(out.TURN, ref["TURN"], "TURN")
    _close(out.NET, ref["NET"], "NET")


@pytest.mark.parametrize("vw", [True, False])
def test_portfolio_multi_shares_cohort_pass(engine, vw):
    """One cohort-sum pass with Kmax serves every K <= Kmax, and one turnover pass every K of
    the set: identical to per-K calls (value weights: f64 path; equal weights: member counts
    in full legs, f64 sums in the first months)."""
    L, NR, _, PM = _labels(engine, "c1")
    W = _up(np.abs(PM.cpu().numpy()) * 1e6) if vw else None
    multi = engine.portfolio_multi(L, NR, 10, Ks=(3, 6, 9, 12), W=W)
    for K, got in multi.items():
        one = engine.portfolio(L, NR, 10, K=K, W=W)
        for f in ("PR", "LS", "TURN", "COST", "NET"):
            assert bits_equal(getattr(got, f).cpu().numpy(), getattr(one, f).cpu().numpy()), (K, f)


@pytest.mark.parametrize("ncols", [500, 498, 497])
@pytest.mark.parametrize("vw", [False, True])
def test_turnover_cell_pairs_vs_oracle_and_per_k(engine, ncols, vw):
    """Turnover / costs with square-root impact on rows of N % 4 == 0, 2 and odd N (the steady
    rows' lanes take 4 or 1 cells and the general rows walk them the same way), through
    k_turn_prep's factors: portfolio_multi over a K set equals per-K calls bit for bit (a row
    switches between the steady and the general launch with the K set) and both match the
    oracle."""
    z = load_golden("c1")
    PM, _ = engine.month_end(_up(np.ascontiguousarray(z["P"][:, :ncols])),
                             _up(z["month_start"].astype(np.int64)))
    _, M, NR = engine.momentum(PM, 12, 1)
    L, _, _, _ = engine.deciles(M, None, 10)
    rng = np.random.default_rng(ncols + vw)
    T_m, N = L.shape
    W = np.abs(PM.cpu().numpy()) * rng.uniform(1e5, 1e7, N) if vw else None
    ADV = rng.uniform(1e5, 1e8, (T_m, N))
    SIG = rng.uniform(0.005, 0.05, (T_m, N))
    SIG[rng.random(SIG.shape) < 0.02] = np.nan
    kw = dict(W=None if W is None else _up(W), aum=5e6, ADV=_up(ADV), SIG=_up(SIG))
    multi = engine.portfolio_multi(L, NR, 10, Ks=(3, 6, 12), **kw)
    for K in (3, 6, 12):
        one = engine.portfolio(L, NR, 10, K=K, **kw)
        for f in ("PR", "LS", "TURN", "COST", "NET"):
            assert bits_equal(getattr(multi[K], f).cpu().numpy(), getattr(one, f).cpu().numpy()), (K, f)
        ref = PO.portfolio(L.cpu().numpy(), NR.cpu().numpy(), 10, K=K, W=W, aum=5e6, ADV=ADV,
                           SIG=SIG)
        for f in ("TURN", "COST", "NET", "LS"):
            _close(getattr(one, f), ref[f], (K, f))


_COHORT_MODES = {"seg": (1, 1), "lds": (0, 1), "reg": (0, 0)}   # (cohort_seg, cohort_lds)


def _with_cohort_mode(engine, mode, fn):
    lib = engine.lib
    seg, lds = _COHORT_MODES[mode]
    try:
        assert lib.csm_tune(b"cohort_seg", seg) == 0 and lib.csm_tune(b"cohort_lds", lds) == 0
        return fn()
    finally:
        lib.csm_tune(b"cohort_seg", 1)
        lib.csm_tune(b"cohort_lds", 1)


@pytest.mark.parametrize("vw", [False, True])
@pytest.mark.parametrize("B", [1, 6])
def test_cohort_variants_deterministic_and_equal(engine, vw, B):
    """The three cohort-sum kernels (label-sorted segment gathers, per-wave LDS atomics,
    register one-hot accumulators): each gives identical bits on repeated runs, and they agree
    within 1e-10 (different summation orders).  B = 6 panels takes the one-chunk plan."""
    L, NR, _, PM = _labels(engine, "c1")
    W = _up(np.abs(PM.cpu().numpy()) * 1e6) if vw else None
    if B > 1:
        T_m, N = L.shape
        rep = lambda x: _up(np.stack([np.roll(x.cpu().numpy(), 7 * i, axis=1) for i in range(B)],
                                     axis=1).reshape(T_m, B * N))
        L, NR = rep(L), rep(NR)
        W = rep(W) if vw else None
    run = lambda: engine.portfolio_multi(L, NR, 10, Ks=(3, 12), W=W, B=B)
    res = {m: (_with_cohort_mode(engine, m, run), _with_cohort_mode(engine, m, run))
           for m in _COHORT_MODES}
    for K in (3, 12):
        for f in ("PR", "LS", "TURN", "NET"):
            z = getattr(res["reg"][0][K], f).cpu().numpy()
            for m, (a, b) in res.items():
                x, y = getattr(a[K], f).cpu().numpy(), getattr(b[K], f).cpu().numpy()
                assert bits_equal(x, y), (m, K, f)
                assert np.array_equal(np.isnan(x), np.isnan(z)) and max_rel(x, z) <= 1e-10, (m, K, f)


@pytest.mark.parametrize("n_bins,ncols", [(3, 500), (20, 500), (30, 500), (10, 497), (5, 498)])
@pytest.mark.parametrize("vw", [False, True])
def test_cohort_seg_vs_oracle_nbins(engine, n_bins, ncols, vw):
    """Segment-gather cohort sums (EW, and VW with invalid weights) with NaN returns against
    the portfolio oracle, for several bin counts (ballot loops unrolled per n_bins) and row
    widths that are not a multiple of 4 (scalar id loads, byte label staging)."""
    z = load_golden("c1")
    PM, _ = engine.month_end(_up(np.ascontiguousarray(z["P"][:, :ncols])),
                             _up(z["month_start"].astype(np.int64)))
    _, M, NR = engine.momentum(PM, 6, 1)
    if n_bins <= 20:
        L, _, _, _ = engine.deciles(M, None, n_bins)
    else:   # beyond csm_deciles' range: random labels with gaps
        Lh = np.random.default_rng(n_bins).integers(-1, n_bins, M.shape).astype(np.int8)
        L = _up(Lh)
    Wh = np.abs(PM.cpu().numpy()) * 1e6
    Wh[::7, ::5] = -1.0   # invalid weights: not members
    Wh[::11, ::3] = np.nan
    if not vw:
        Wh = None
    ref = PO.portfolio(L.cpu().numpy(), NR.cpu().numpy(), n_bins, K=5, W=Wh)
    out = _with_cohort_mode(engine, "seg", lambda: engine.portfolio(
        L, NR, n_bins, K=5, W=None if Wh is None else _up(Wh)))
    _close(out.PR, ref["PR"], "PR")
    _close(out.LS, ref["LS"], "LS")
    _close(out.TURN, ref["TURN"], "TURN")
    _close(out.COST, ref["COST"], "COST")


def _summary_ref(LS, TURN, COST, NET, freq=12.0):
    """NumPy restatement of sweep.summarize per (strategy, panel) (src/utils.py:8-16)."""
    nS, T_m, B = LS.shape
    out = np.full((nS, B, 7), np.nan)
    for q in range(nS):
        for b in range(B):
            x = LS[q, :, b]
            ok = ~np.isnan(x)
            n = ok.sum()
            out[q, b, 0] = n

            def sh(v):
                if n < 2:
                    return np.mean(v) if n else np.nan, np.nan
                m, sd = np.mean(v), np.std(v, ddof=1)
                return m, (m * freq / (sd * np.sqrt(freq)) if sd > 0 else np.nan)
            out[q, b, 1], out[q, b, 2] = sh(x[ok])
            if TURN is not None and n:
                out[q, b, 3] = TURN[q, ok, b].mean()
                out[q, b, 4] = COST[q, ok, b].mean()
                out[q, b, 5], out[q, b, 6] = sh(NET[q, ok, b])
    return out


@pytest.mark.parametrize("costs", [True, False])
def test_summary_kernel(engine, costs):
    """csm_summary against a NumPy restatement: NaN months dropped, an all-NaN panel, a
    one-month panel and a constant panel (Sharpe NaN), several strategies in one launch."""
    rng = np.random.default_rng(3)
    nS, T_m, B = 3, 500, 7
    LS = rng.normal(0.01, 0.05, (nS, T_m, B))
    LS[rng.random(LS.shape) < 0.1] = np.nan
    LS[:, :, 2] = np.nan
    LS[:, :, 3] = np.nan
    LS[:, 17, 3] = 0.02
    LS[:, :, 4] = 0.25          # exact sums: sd == 0 -> Sharpe NaN
    TURN = np.abs(rng.normal(0.3, 0.1, LS.shape))
    COST = TURN * 0.001
    NET = LS - COST
    args = (LS, TURN, COST, NET) if costs else (LS, None, None, None)
    got = engine.summary(*[None if a is None else _up(a) for a in args]).cpu().numpy()
    ref = _summary_ref(*args)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    m = ~np.isnan(ref)
    assert np.allclose(got[m], ref[m], rtol=1e-12, atol=1e-15)
    # one [T_m][B] series is nS = 1
    one = engine.summary(*[None if a is None else _up(a[1]) for a in args]).cpu().numpy()
    assert bits_equal(one[0], got[1])


@pytest.mark.parametrize("mode", ["seg", "lds"])
def test_portfolio_many_rows(engine, mode):
    """More (t, b) rows than a grid's y dimension holds (360 x 203 = 73080 > 65535): the
    flattened grids, and the XCD-ordered segment kernel with a panel count that is not a
    multiple of 8, against the oracle."""
    rng = np.random.default_rng(11)
    T_m, B, N = 360, 203, 48
    Lh = rng.integers(-1, 10, (T_m, B, N)).astype(np.int8)
    NRh = rng.normal(0.0, 0.05, (T_m, B, N))
    NRh[rng.random(NRh.shape) < 0.05] = np.nan
    ref = PO.portfolio(Lh, NRh, 10, K=4)
    out = _with_cohort_mode(engine, mode, lambda: engine.portfolio(
        _up(Lh.reshape(T_m, B * N)), _up(NRh.reshape(T_m, B * N)), 10, K=4, B=B))
    _close(out.PR, ref["PR"], "PR")
    _close(out.TURN, ref["TURN"], "TURN")
    _close(out.NET, ref["NET"], "NET")


@pytest.mark.parametrize("vw", [False, True])
@pytest.mark.parametrize("B,n_bins", [(1, 10), (6, 10), (4, 3), (4, 2), (4, 20), (70, 10)])
def test_legs_only_equals_full(engine, vw, B, n_bins):
    """Legs-only accounting (csm_cohort_sums_legs + csm_portfolio_from_cohorts_legs: only
    deciles 0 and n_bins - 1 sorted and summed, the partials in the two-leg layout) gives the
    full path's LS / TURN / COST / NET bit for bit and its PR on the two legs; the other deciles
    are NaN.  n_bins 2 (both deciles are legs) to 20; 70 panels take the wide long-short."""
    L, NR, _, PM = _labels(engine, "c1")
    if n_bins != 10:
        _, M, NR = engine.momentum(PM, 12, 1)
        L, _, _, _ = engine.deciles(M, None, n_bins)
    T_m, N = L.shape
    W = _up(np.abs(PM.cpu().numpy()) * 1e6) if vw else None
    if B > 1:
        rep = lambda x: _up(np.stack([np.roll(x.cpu().numpy(), 5 * i, axis=1) for i in range(B)],
                                     axis=1).reshape(T_m, B * N))
        L, NR = rep(L), rep(NR)
        W = rep(W) if vw else None
    rng = np.random.default_rng(B)
    ADV = _up(rng.uniform(1e5, 1e8, (T_m, B * N)))
    kw = dict(Ks=(3, 6, 12), W=W, B=B, aum=5e6, ADV=ADV)
    full = engine.portfolio_multi(L, NR, n_bins, **kw)
    legs = engine.portfolio_multi(L, NR, n_bins, legs_only=True, **kw)
    for K in (3, 6, 12):
        for f in ("LS", "TURN", "COST", "NET"):
            assert bits_equal(getattr(legs[K], f).cpu().numpy(), getattr(full[K], f).cpu().numpy()), (K, f)
        a, b = legs[K].PR.cpu().numpy(), full[K].PR.cpu().numpy()
        for d in (0, n_bins - 1):
            assert bits_equal(a[..., d], b[..., d]), (K, d)
        assert np.isnan(a[..., 1:n_bins - 1]).all()


def test_legs_only_falls_back_when_a_leg_column_is_missing(engine):
    """A panel whose top decile never occurs: the long-short rule takes max - min over every
    decile (run_demo.py:60-65), so the legs-only call reruns the full accounting -- the result
    equals the full path bit for bit, PR included -- and the sweep's deferred flag does too."""
    L, NR, _, _ = _labels(engine, "c1")
    Lh = L.cpu().numpy().copy()
    Lh[Lh == 9] = 8
    L2 = _up(Lh)
    full = engine.portfolio_multi(L2, NR, 10, Ks=(3, 12))
    legs = engine.portfolio_multi(L2, NR, 10, Ks=(3, 12), legs_only=True)
    for K in (3, 12):
        for f in ("PR", "LS", "TURN", "COST", "NET"):
            assert bits_equal(getattr(legs[K], f).cpu().numpy(), getattr(full[K], f).cpu().numpy()), (K, f)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    engine.portfolio_multi(L2, NR, 10, Ks=(3, 12), legs_only=True, need_full=flag)
    assert int(flag.item()) == 1
    flag.zero_()
    engine.portfolio_multi(L, NR, 10, Ks=(3, 12), legs_only=True, need_full=flag)
    assert int(flag.item()) == 0


@pytest.mark.parametrize("B,legs,vw,Ks", [(1, False, False, (3, 6, 12)), (1, True, False, (12, 3)),
                                          (16, True, False, (3, 6, 9, 12)),
                                          (16, False, True, (1, 9, 9)), (4, False, True, (12, 2, 5))])
def test_overlap_rows_bit_identical(engine, B, legs, vw, Ks):
    """k_overlap_rows (one thread per (t, b, decile) for every K of the set; trips of 8 ages)
    against k_overlap (one thread per (K, t, b, decile)): PR / LS / TURN / COST / NET bit for
    bit on single-chunk plans (B = 16), repeated and unsorted K sets, legs-only and full
    accounting, equal and value weights; chunked plans (B = 1, 4: C > 1) keep k_overlap in
    both modes."""
    L, NR, _, _ = _labels(engine, "c1")
    T_m, N = L.shape
    if B > 1:
        rep = lambda x: _up(np.stack([np.roll(x.cpu().numpy(), 5 * i, axis=1) for i in range(B)],
                                     axis=1).reshape(T_m, B * N))
        L, NR = rep(L), rep(NR)
    W = None
    if vw:
        g = np.random.default_rng(7)
        W = _up(g.uniform(0.5, 2.0, size=(T_m, B * N)))
    lib = engine.lib
    got = {}
    try:
        for mode in (1, 0):
            assert lib.csm_tune(b"overlap_rows", mode) == 0
            got[mode] = engine.portfolio_multi(L, NR, 10, Ks=Ks, B=B, W=W, legs_only=legs)
    finally:
        lib.csm_tune(b"overlap_rows", 1)
    for K in set(Ks):
        for f in ("PR", "LS", "TURN", "COST", "NET"):
            assert bits_equal(getattr(got[1][K], f).cpu().numpy(), getattr(got[0][K], f).cpu().numpy()), (K, f)


@pytest.mark.parametrize("G,Bg,vw,legs,mode,ncols", [
    (4, 1, True, True, "seg", 500), (4, 1, False, True, "seg", 500), (3, 2, True, False, "seg", 497),
    (2, 3, False, False, "lds", 498), (4, 1, True, False, "reg", 500), (2, 2, True, True, "seg", 498)])
def test_grouped_equals_side_by_side(engine, G, Bg, vw, legs, mode, ncols):
    """csm_cohort_sums_grouped / csm_portfolio_from_cohorts_grouped (labels / next_ret
    group-major [G][T_m][Bg * N], weights / ADV shared by the groups) give the plain-layout
    accounting of the side-by-side panels (weights repeated per group) bit for bit: PR / LS /
    TURN / COST / NET, every cohort kernel, legs-only and full, equal and value weights with
    impact costs, row widths that are not a multiple of 4."""
    z = load_golden("c1")
    PM, _ = engine.month_end(_up(np.ascontiguousarray(z["P"][:, :ncols])),
                             _up(z["month_start"].astype(np.int64)))
    T_m, N = PM.shape
    Lgs, NRgs = [], []
    for g in range(G):   # group g: look-back 3 + 3g on Bg rolled copies of the panel
        _, M, NR = engine.momentum(PM, 3 + 3 * g, 1)
        L, _, _, _ = engine.deciles(M, None, 10)
        roll = lambda x: np.stack([np.roll(x.cpu().numpy(), 5 * p, axis=1) for p in range(Bg)],
                                  axis=1).reshape(T_m, Bg * N)
        Lgs.append(roll(L))
        NRgs.append(roll(NR))
    rng = np.random.default_rng(G * 10 + Bg)
    Wh = np.abs(np.stack([np.roll(PM.cpu().numpy(), 5 * p, axis=1) for p in range(Bg)], axis=1)
                ).reshape(T_m, Bg * N) * rng.uniform(1e5, 1e7, Bg * N)
    Wh[rng.random(Wh.shape) < 0.01] = np.nan
    ADVh = rng.uniform(1e5, 1e8, (T_m, Bg * N))
    W = _up(Wh) if vw else None
    ADV = _up(ADVh)
    kw = dict(Ks=(3, 6, 12), half_spread=0.0005, k_impact=0.1, aum=5e6, legs_only=legs)
    grp = _with_cohort_mode(engine, mode, lambda: engine.portfolio_multi_grouped(
        _up(np.stack(Lgs)), _up(np.stack(NRgs)), 10, W=W, Bg=Bg, ADV=ADV, **kw))
    side = lambda xs: _up(np.concatenate(xs, axis=1))
    plain = _with_cohort_mode(engine, mode, lambda: engine.portfolio_multi(
        side(Lgs), side(NRgs), 10, W=None if W is None else _up(np.tile(Wh, (1, G))), B=G * Bg,
        ADV=_up(np.tile(ADVh, (1, G))), **kw))
    for K in (3, 6, 12):
        for f in ("PR", "LS", "TURN", "COST", "NET"):
            a, b = getattr(grp[K], f).cpu().numpy(), getattr(plain[K], f).cpu().numpy()
            assert a.shape == b.shape and bits_equal(a, b), (K, f)


@pytest.mark.parametrize("B,Ks,ncols", [(1, (3, 6, 9, 12), 500), (16, (3, 6, 9, 12), 500),
                                        (8, (12, 3), 1000), (5, (1, 7, 7), 372),
                                        (3, (3, 6, 9, 12), 4600)])
@pytest.mark.parametrize("key", [b"turn_mask", b"ls_opt"])
def test_turnover_mask_bit_identical(engine, B, Ks, ncols, key):
    """Steady equal-weight legs turnover from the leg bitplanes of the legs label sort
    (k_turnover_ew_mask, popcounts of 64-cell words) against the label-byte path (turn_mask 0),
    and the legs label sort's prefix ranks by v_mbcnt against masked popcounts (ls_opt 0):
    LS / TURN / COST / NET bit for bit -- plain batches and the grouped shared-return path of
    the bootstrap sweep; row widths that end inside a plane word, rows of several cell groups
    per lane."""
    z = load_golden("c1")
    P = z["P"]
    if ncols > P.shape[1]:   # rows wider than a lane's one cell group: tiled columns
        P = np.tile(P, (1, -(-ncols // P.shape[1])))
    PM, _ = engine.month_end(_up(np.ascontiguousarray(P[:, :ncols])),
                             _up(z["month_start"].astype(np.int64)))
    T_m, N = PM.shape
    _, M, NR = engine.momentum(PM, 12, 1)
    L, _, _, _ = engine.deciles(M, None, 10)
    rep = lambda x: _up(np.stack([np.roll(x.cpu().numpy(), 7 * i, axis=1) for i in range(B)],
                                 axis=1).reshape(T_m, B * N))
    L, NR = rep(L), rep(NR)
    lib = engine.lib
    got = {}
    try:
        for mode in (1, 0):
            assert lib.csm_tune(key, mode) == 0
            plain = engine.portfolio_multi(L, NR, 10, Ks=Ks, B=B, legs_only=True)
            grp = engine.portfolio_multi_js_grouped(torch.stack([L, L]), NR, 10, Ks=Ks, B=B,
                                                    legs_only=True)
            got[mode] = (plain, grp)
    finally:
        lib.csm_tune(key, 1)
    for i in range(2):
        for K in set(Ks):
            for f in ("LS", "TURN", "COST", "NET"):
                a = getattr(got[1][i][K], f).cpu().numpy()
                b = getattr(got[0][i][K], f).cpu().numpy()
                assert bits_equal(a, b), (i, K, f)


def test_turnover_planes_follow_the_cohort_pass(engine):
    """The steady legs turnover reads the leg bitplanes only from a workspace whose cohort pass
    wrote them (recorded per workspace in the context), never because the knob says so at
    accounting time: a cohort pass run with turn_mask 0 into a workspace full of garbage,
    then the accounting with turn_mask back at 1, gives the default path's bits (the label
    bytes are read instead of the never-written planes)."""
    import ctypes
    z = load_golden("c1")
    PM, _ = engine.month_end(_up(z["P"]), _up(z["month_start"].astype(np.int64)))
    T_m, N = PM.shape
    _, M, NR = engine.momentum(PM, 12, 1)
    L, _, _, _ = engine.deciles(M, None, 10)
    B, Ks = 8, (3, 6, 9, 12)
    rep = lambda x: _up(np.stack([np.roll(x.cpu().numpy(), 7 * i, axis=1) for i in range(B)],
                                 axis=1).reshape(T_m, B * N))
    L, NR = rep(L), rep(NR)
    ref = engine.portfolio_multi(L, NR, 10, Ks=Ks, B=B, legs_only=True)
    lib = engine.lib
    nbytes = int(lib.csm_portfolio_workspace(T_m, B, N, 10, max(Ks)))
    ws = torch.full((nbytes,), 0xFF, dtype=torch.uint8, device="cuda:0")
    try:
        assert lib.csm_tune(b"turn_mask", 0) == 0
        engine._call("csm_cohort_sums_legs", ctypes.c_void_p(L.data_ptr()),
                     ctypes.c_void_p(NR.data_ptr()), None, T_m, B, N, 10, max(Ks),
                     ctypes.c_void_p(ws.data_ptr()))
    finally:
        assert lib.csm_tune(b"turn_mask", 1) == 0
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    res, _ = engine._from_cohorts(L, None, T_m, B, N, 10, list(Ks), 0.0005, 0.1, 0.0, None,
                                  None, True, ws, True, flag)
    assert int(flag.item()) == 0
    for K in Ks:
        for f in ("LS", "TURN", "COST", "NET"):
            assert bits_equal(getattr(res[K], f).cpu().numpy(),
                              getattr(ref[K], f).cpu().numpy()), (K, f)


def _ls_rule(PR):
    """run_demo.py:57-67 per (month, panel) on the engine's own PR [T_m][B][nb]: D(n-1) - D0 when
    the panel has both legs in some month, else max - min over the deciles holding a value."""
    T_m, B, nb = PR.shape
    LS = np.full((T_m, B), np.nan)
    for b in range(B):
        col = PR[:, b, :]
        both = bool((~np.isnan(col[:, 0])).any() and (~np.isnan(col[:, nb - 1])).any())
        for t in range(T_m):
            e = col[t]
            ok = ~np.isnan(e)
            if not ok.any():
                continue
            LS[t, b] = (e[nb - 1] - e[0]) if both else (e[ok].max() - e[ok].min())
    return LS, both


@pytest.mark.parametrize("legs", [False, True])
def test_long_short_wide_batch_rule(engine, legs):
    """Batches of >= 64 panels form the long-short in two launches (k_ls_flags over month
    blocks, k_ls_rows per output): LS / NET equal the reference rule applied to the engine's
    own PR, bit for bit, on 80 panels where some lack the top or the bottom leg in every month
    (max - min there) or have empty months; legs-only accounting sets the rerun flag for them
    and its rerun is the full path's, bit for bit."""
    rng = np.random.default_rng(5)
    T_m, B, N, nb = 40, 80, 120, 10
    Lh = rng.integers(-1, nb, size=(T_m, B, N)).astype(np.int8)
    Lh[:, 3, :][Lh[:, 3, :] == nb - 1] = nb - 2       # panel 3: no top decile ever
    Lh[:, 11, :][Lh[:, 11, :] == 0] = 1               # panel 11: no bottom decile ever
    Lh[5:9, 17, :] = -1                               # panel 17: four empty months
    NRh = rng.normal(0.01, 0.08, size=(T_m, B, N))
    NRh[rng.random(NRh.shape) < 0.02] = np.nan
    L, NR = _up(Lh.reshape(T_m, B * N)), _up(NRh.reshape(T_m, B * N))
    full = engine.portfolio_multi(L, NR, nb, Ks=(1, 3), B=B)
    for K in (1, 3):
        PR = full[K].PR.cpu().numpy().reshape(T_m, B, nb)
        ref, _ = _ls_rule(PR)
        assert bits_equal(full[K].LS.cpu().numpy().reshape(T_m, B), ref), K
        net = full[K].LS.cpu().numpy() - full[K].COST.cpu().numpy()
        assert bits_equal(full[K].NET.cpu().numpy(), net), K
    if legs:
        flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
        engine.portfolio_multi(L, NR, nb, Ks=(1, 3), B=B, legs_only=True, need_full=flag)
        assert int(flag.item()) == 1
        got = engine.portfolio_multi(L, NR, nb, Ks=(1, 3), B=B, legs_only=True)
        for K in (1, 3):
            for f in ("PR", "LS", "TURN", "COST", "NET"):
                assert bits_equal(getattr(got[K], f).cpu().numpy(),
                                  getattr(full[K], f).cpu().numpy()), (K, f)


@pytest.mark.parametrize("n_bins", [2, 4, 10])
def test_legs_only_equals_full_wide_legs(engine, n_bins):
    """The one-wave legs label sort stages a row's segment in LDS when its two legs hold at most
    2,048 ids and stores it directly otherwise: 3,000-asset rows with n_bins 2 (every ranked cell
    in a leg: the direct stores), 4 and 10 (staged) -- legs-only accounting equals the full path
    bit for bit either way (LS / TURN / COST / NET, PR on the legs)."""
    rng = np.random.default_rng(n_bins)
    T_m, B, N = 60, 3, 3000
    Lh = rng.integers(-1, n_bins, size=(T_m, B, N)).astype(np.int8)
    NRh = rng.normal(0.01, 0.08, size=(T_m, B, N))
    L, NR = _up(Lh.reshape(T_m, B * N)), _up(NRh.reshape(T_m, B * N))
    full = engine.portfolio_multi(L, NR, n_bins, Ks=(1, 3, 12), B=B)
    legs = engine.portfolio_multi(L, NR, n_bins, Ks=(1, 3, 12), B=B, legs_only=True)
    for K in (1, 3, 12):
        for f in ("LS", "TURN", "COST", "NET"):
            assert bits_equal(getattr(legs[K], f).cpu().numpy(), getattr(full[K], f).cpu().numpy()), (K, f)
        a, b = legs[K].PR.cpu().numpy(), full[K].PR.cpu().numpy()
        for d in (0, n_bins - 1):
            assert bits_equal(a[..., d], b[..., d]), (K, d)
