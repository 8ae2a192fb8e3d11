"""GPU: csm_boot_scan (csm_bootstrap fused into the multi-J scan for the bootstrap sweep, C5)
against the materialised path it replaces -- csm_bootstrap -> csm_momentum_multi_ids -- and the
oracle.  Bar: source months, mom_J and bucket ids of every J bit for bit; the shared next_ret
equals each J's next_ret wherever that is defined and on every cell J labels; SweepRunner's
summary table bit for bit with SweepConfig.boot_scan on and off (rules E1-E6,
oracle/portfolio_oracle.py; the scan: src/features.py:44-52, run_demo.py:48)."""
import numpy as np
import pytest
import torch

from conftest import bits_equal
from oracle import csmom_oracle as O
from oracle import portfolio_oracle as PO

pytestmark = pytest.mark.gpu


def _base_returns(engine, N, T_d=2600, seed=11):
    from csmom.synth import bday_calendar, make_device_panel
    days, ms_h, _ = bday_calendar("2000-01-03", T_d)
    pan = make_device_panel(N, days, ms_h, seed=seed, device="cuda:0")
    PM, _ = engine.month_end(pan.P, pan.month_start)
    R, _, _ = engine.momentum(PM, 12, 1, with_ret=True)
    return R.contiguous()


@pytest.mark.parametrize("N,B,b0,Js,skip,ids", [
    (500, 6, 0, (3, 6, 9, 12), 1, True),      # the default grid: compile-time windows
    (5000, 3, 999, (3, 6, 9, 12), 1, True),
    (2000, 5, 37, (3, 12), 1, True),          # generic predicated windows
    (800, 3, 1, (2, 7, 15), 1, False),
    (640, 2, 3, (4,), 0, True),
    (1202, 2, 8, (12, 3, 6, 9), 1, False),    # N % 4 != 0: no ids
    (12, 3, 0, (3, 6, 9, 12), 1, True),
])
def test_boot_scan_equals_materialised(engine, N, B, b0, Js, skip, ids):
    R = _base_returns(engine, N)
    T_m = R.shape[0]
    src, outs, NR, bad = engine.boot_scan(R, B, Js, skip, b0=b0, seed=5000, mean_block=6.0,
                                          with_ids=ids)
    assert int(bad.item()) == 0
    ref_src = PO.bootstrap_indices(T_m, B, 5000, 6.0, b0=b0)
    assert np.array_equal(src.cpu().numpy().astype(np.int64), ref_src)
    _, PMb = engine.bootstrap(R, B, b0=b0, seed=5000, mean_block=6.0)
    ref = engine.momentum_multi(PMb, Js, skip, with_ids=ids)
    nr = NR.cpu().numpy()
    for J, (M, IDS), r in zip(Js, outs, ref):
        assert bits_equal(M.cpu().numpy(), r[0].cpu().numpy()), J
        if ids:
            assert torch.equal(IDS, r[2]), J
        nrj = r[1].cpu().numpy()
        ok = ~np.isnan(nrj)   # wherever J's next_ret is defined
        assert bits_equal(nr[ok], nrj[ok]), J
        on = ~np.isnan(M.cpu().numpy())   # every ranked cell
        assert bits_equal(nr[on], nrj[on]), J
    if N == 500:   # and the oracle's scan of the oracle's panel
        pm = PO.bootstrap_panel(R.cpu().numpy(), ref_src).reshape(T_m, B * N)
        for J, (M, _) in zip(Js, outs):
            _, Mr, _, _ = O.momentum_scan(pm, J, skip)
            assert bits_equal(M.cpu().numpy(), Mr), J


def test_boot_scan_bad_prices_flagged(engine):
    """A return of exactly -1 makes a price 0: outside the shared next_ret's domain, so the
    kernel raises `bad`; SweepRunner then reruns the batch on the materialised path (the same
    table as boot_scan off)."""
    import csmom
    R = _base_returns(engine, 400)
    R[40, 7] = -1.0
    _, _, _, bad = engine.boot_scan(R, 300, (3, 12), 1, b0=0, seed=5000, mean_block=6.0)
    assert int(bad.item()) == 1   # some of 300 panels draw month 40
    on = csmom.SweepConfig(Js=(3, 12), Ks=(3, 12), skip=1)
    off = csmom.SweepConfig(Js=(3, 12), Ks=(3, 12), skip=1, boot_scan=False)
    a = csmom.SweepRunner(engine, on).run_bootstrap(R, 300, batch=300).cpu().numpy()
    b = csmom.SweepRunner(engine, off).run_bootstrap(R, 300, batch=300).cpu().numpy()
    assert bits_equal(a, b)


@pytest.mark.parametrize("legs,ids", [(True, True), (False, True), (True, False)])
def test_sweep_runner_boot_scan_bit_identical(engine, legs, ids):
    import csmom
    R = _base_returns(engine, 1500, seed=12)
    kw = dict(Js=(3, 6, 9, 12), Ks=(3, 6, 9, 12), skip=1, legs_only=legs, decile_ids=ids)
    a = csmom.SweepRunner(engine, csmom.SweepConfig(**kw)).run_bootstrap(
        R, 20, seed=5000, mean_block=6.0, batch=8).cpu().numpy()
    b = csmom.SweepRunner(engine, csmom.SweepConfig(boot_scan=False, **kw)).run_bootstrap(
        R, 20, seed=5000, mean_block=6.0, batch=8).cpu().numpy()
    assert bits_equal(a, b)


@pytest.mark.parametrize("N,B,Js,Ks,n_bins,legs", [
    (1500, 6, (3, 6, 9, 12), (3, 6, 9, 12), 10, True),    # C5's grid: legs, one shared pass
    (1500, 6, (3, 6, 9, 12), (1, 3), 10, False),          # every decile, shared
    (1500, 6, (3, 6, 9, 12), (3, 6, 9, 12), 10, False),   # offsets too many: per-J passes
    (1202, 9, (3, 12), (2, 5), 5, True),                  # N % 4 != 0: the general label sort
    (640, 3, (4,), (6,), 3, False),
])
def test_cohort_sums_js_equal_per_j(engine, N, B, Js, Ks, n_bins, legs):
    """csm_cohort_sums_js (one staged next_ret row for every J) leaves every J's partials and
    the accounting on them bit for bit as csm_cohort_sums(_legs) per J."""
    R = _base_returns(engine, N, seed=13)
    T_m = R.shape[0]
    _, outs, NR, bad = engine.boot_scan(R, B, Js, 1, b0=5, with_ids=False)
    assert int(bad.item()) == 0
    Ls = []
    for M, _ in outs:
        L, _, _, _ = engine.deciles(M.reshape(T_m * B, N), None, n_bins)
        Ls.append(L.reshape(T_m, B * N))
    got = engine.portfolio_multi_js(Ls, NR, n_bins, Ks=Ks, B=B, legs_only=legs)
    for L, (res, stk) in zip(Ls, got):
        ref, rstk = engine.portfolio_multi(L, NR, n_bins, Ks=Ks, B=B, legs_only=legs,
                                           return_stacked=True)
        for f in ("PR", "LS", "TURN", "COST", "NET"):
            assert bits_equal(getattr(stk, f).cpu().numpy(), getattr(rstk, f).cpu().numpy()), f
        assert stk.legs_only == rstk.legs_only


@pytest.mark.parametrize("N,B,Js,Ks,n_bins,legs", [
    (256, 36, (3, 6, 9, 12), (3, 6, 9, 12), 10, True),    # C5's grid: one shared grouped pass
    (256, 36, (3, 6, 9, 12), (1, 3), 10, False),          # every decile, shared
    (256, 36, (3, 6, 9, 12), (3, 6, 9, 12), 10, False),   # offsets too many: the grouped pass
    (202, 40, (3, 12), (2, 5), 5, True),                  # N % 4 != 0: the general label sort
    (1024, 6, (3, 6, 9, 12), (3, 6, 9, 12), 10, True),    # plans differ: TURN / COST within 1e-12
])
def test_cohort_sums_js_grouped_equal_js(engine, N, B, Js, Ks, n_bins, legs):
    """csm_cohort_sums_js_grouped + csm_portfolio_from_cohorts_grouped (the Js' labels
    group-major, one workspace of nJ * B panels, one accounting launch set) give every J's
    outputs bit for bit as portfolio_multi_js where the chunk plans agree (portfolio_plan); with
    different plans the cohort sums (PR / LS) keep their bits and TURN / COST their values."""
    R = _base_returns(engine, N, seed=15)
    T_m = R.shape[0]
    _, outs, NR, bad = engine.boot_scan(R, B, Js, 1, b0=3, with_ids=False)
    assert int(bad.item()) == 0
    nJ = len(Js)
    Lg = torch.empty((nJ, T_m * B, N), dtype=torch.int8, device="cuda:0")
    for q, (M, _) in enumerate(outs):
        Lg[q].copy_(engine.deciles(M.reshape(T_m * B, N), None, n_bins)[0])
    Lg = Lg.view(nJ, T_m, B * N)
    same = engine.portfolio_plan(T_m, B, N, n_bins, max(Ks)) == \
        engine.portfolio_plan(T_m, nJ * B, N, n_bins, max(Ks))
    assert same == (B > 6)   # (714 rows per J: chunked plans; 2856 side by side: one chunk)
    res, stk = engine.portfolio_multi_js_grouped(Lg, NR, n_bins, Ks=Ks, B=B, legs_only=legs,
                                                 return_stacked=True)
    ref = engine.portfolio_multi_js([Lg[q] for q in range(nJ)], NR, n_bins, Ks=Ks, B=B,
                                    legs_only=legs)
    assert stk.legs_only == ref[0][1].legs_only
    for q, (_, rstk) in enumerate(ref):
        for f in ("PR", "LS", "TURN", "COST", "NET"):
            a = getattr(stk, f)[:, :, q * B:(q + 1) * B].cpu().numpy()
            b = getattr(rstk, f).cpu().numpy()
            if same or f in ("PR", "LS"):
                assert bits_equal(a, b), (q, f)
            else:
                assert np.array_equal(np.isnan(a), np.isnan(b)), (q, f)
                assert np.nanmax(np.abs(a - b) / np.maximum(np.abs(b), 1e-300),
                                 initial=0.0) <= 1e-12, (q, f)


@pytest.mark.parametrize("legs", [True, False])
def test_sweep_runner_share_nr_bit_identical(engine, legs):
    """A bootstrap batch above JOIN_ROWS rows takes the shared cohort pass (share_nr): the table
    equals share_nr off and boot_scan off bit for bit."""
    import csmom
    from csmom.sweep import JOIN_ROWS
    R = _base_returns(engine, 1000, seed=14)
    batch = JOIN_ROWS // R.shape[0] + 2
    kw = dict(Js=(3, 6, 9, 12), Ks=(3, 6, 9, 12), skip=1, legs_only=legs)
    run = lambda **o: csmom.SweepRunner(engine, csmom.SweepConfig(**kw, **o)).run_bootstrap(
        R, batch + 3, seed=5000, mean_block=6.0, batch=batch).cpu().numpy()
    a = run()
    assert bits_equal(a, run(share_nr=False))
    assert bits_equal(a, run(boot_scan=False))


def test_cohort_sums_js_rejects_bad_args(engine):
    import csmom
    R = _base_returns(engine, 500, T_d=700)
    _, outs, NR, _ = engine.boot_scan(R, 2, (3, 6, 9, 12), 1, with_ids=False)
    T_m = R.shape[0]
    L = engine.deciles(outs[0][0].reshape(T_m * 2, 500), None, 10)[0].reshape(T_m, 1000)
    with pytest.raises(csmom.CsmError):
        engine.portfolio_multi_js([L] * 5, NR, 10, Ks=(3,), B=2)   # more than 4 J
    with pytest.raises(ValueError):
        engine.portfolio_multi_js([L], NR, 10, Ks=(3,), B=3)       # width not B panels


def test_boot_scan_rejects_bad_args(engine):
    import csmom
    R = _base_returns(engine, 500, T_d=700)
    with pytest.raises(csmom.CsmError):
        engine.boot_scan(R, 2, (3, 6, 9, 12, 3), 1)   # more than 4 J
    with pytest.raises(csmom.CsmError):
        engine.boot_scan(R, 2, (16,), 1)              # J + skip > 16
    R2 = _base_returns(engine, 501, T_d=700)
    with pytest.raises(csmom.CsmError):
        engine.boot_scan(R2, 2, (3,), 1, with_ids=False)   # odd N
