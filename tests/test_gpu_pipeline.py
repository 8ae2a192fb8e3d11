"""GPU parity of the bucket-id pipeline (csm_signal_ids -> csm_deciles_ids, csm_pipeline).

The fused signal kernel writes each mom_J's bucket under a FIXED monotone map
(csrc/csm_common.h csm_fbucket); the decile pass histograms those 2-B ids instead of
streaming mom_J again.  The map only decides how many values share a bucket, so labels,
counts and ranked-row counts must equal the default decile kernel's (and the oracle's,
run_demo.py:18-29) bit for bit on any data, decile means within 1e-10 (they are summed in a
different fixed order).  The stress rows reach every slow path: refinement of a bucket that
holds the whole row, extreme buckets holding huge tails, all-equal rows, +-0.0.
"""
import numpy as np
import pytest
import torch

from conftest import bits_equal, load_golden, max_rel
from oracle import csmom_oracle as O

pytestmark = pytest.mark.gpu
REL = 1e-10


def _up(x, dev="cuda:0"):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def fixed_ids(x):
    """NumPy restatement of csm_fid: bucket of fl(1 + x) at 1024 per octave over [1/16, 16),
    clamped to [0, 8191]; NaN -> 0xFFFF."""
    x = np.asarray(x, dtype=np.float64)
    with np.errstate(invalid="ignore", over="ignore"):
        y = 1.0 + x
    b = y.view(np.int64) >> 42
    k = np.clip(b - (np.float64(1.0 / 16).view(np.int64) >> 42), 0, 8191)
    return np.where(np.isnan(x), 0xFFFF, k).astype(np.uint16)


def _oracle_labels(row, n_bins=10):
    ok = ~np.isnan(row)
    out = np.full(len(row), -1, dtype=np.int8)
    if ok.any():
        lab = O.qcut_labels(row[ok], n_bins)
        out[ok] = np.where(np.isnan(lab), -1, lab).astype(np.int8)
    return out


def _ids_dev(x):
    return _up(fixed_ids(x).view(np.int16))


def test_fixed_map_is_monotone():
    """Host check of the map the kernels share: non-decreasing over a sorted sweep that
    crosses both clamps, every octave boundary and +-0.0."""
    xs = np.sort(np.concatenate([
        np.linspace(-5, 10, 200_001), -np.logspace(-300, 300, 2001), np.logspace(-300, 300, 2001),
        [-np.inf, np.inf, -0.9375, -0.5, 0.0, -0.0, 1.0, 15.0, np.nextafter(-0.9375, 0),
         np.nextafter(15.0, 16)]]))
    ids = fixed_ids(xs).astype(np.int64)
    assert (np.diff(ids) >= 0).all()
    assert ids[0] == 0 and ids[-1] == 8191
    assert fixed_ids(np.array([np.nan]))[0] == 0xFFFF


def _panel(N=20_000, T=900, seed=11):
    from oracle.synth_np import make_panel
    return make_panel(N, T, seed=seed, start="2001-01-02", with_volume=False, nan_day=0.02,
                      absent_month=0.01, nan_month=0.01, cents=True)


def test_signal_ids_equal_fixed_map_of_mom(engine):
    pan = _panel()
    ms_h = pan["month_start"]
    maxd = int(np.diff(ms_h).max())
    P, ms = _up(pan["P"]), _up(ms_h)
    PM, R, M, NR, IDS = engine.signal_ids(P, ms, maxd, 12, 1, with_pm=True, with_ret=True)
    base = engine.signal(P, ms, maxd, 12, 1, with_pm=True, with_ret=True)
    for a, b in zip((PM, R, M, NR), base):
        assert bits_equal(a.cpu().numpy(), b.cpu().numpy())
    m = M.cpu().numpy()
    assert np.array_equal(IDS.cpu().numpy().view(np.uint16), fixed_ids(m))


@pytest.mark.parametrize("J,skip", [(12, 1), (3, 0), (1, 1), (24, 2)])
def test_pipeline_vs_oracle(engine, J, skip):
    """csm_pipeline (one C call) on a 20,000-asset daily panel against the oracle."""
    pan = _panel(seed=7 + J)
    ms_h = pan["month_start"]
    out = engine.pipeline(_up(pan["P"]), _up(ms_h), J, skip, 10, with_ret=True)
    ref = O.pipeline(pan["P"], ms_h, J, skip, 10)
    for k in ("PM", "R", "M", "NR"):
        assert bits_equal(getattr(out, k).cpu().numpy(), ref[k]), k
    assert np.array_equal(out.L.cpu().numpy(), ref["L"])
    assert np.array_equal(out.CNT.cpu().numpy(), ref["CNT"])
    ew, ls = out.EW.cpu().numpy(), out.LS.cpu().numpy()
    assert np.array_equal(np.isnan(ew), np.isnan(ref["EW"])) and max_rel(ew, ref["EW"]) <= REL
    assert np.array_equal(np.isnan(ls), np.isnan(ref["LS"])) and max_rel(ls, ref["LS"]) <= REL


def test_pipeline_equals_stagewise_default_path(engine):
    """The id pipeline and the default signal -> deciles -> long_short agree: labels, counts
    and ranked rows bit for bit, means within 1e-13."""
    pan = _panel(N=24_000, T=700, seed=3)
    ms_h = pan["month_start"]
    maxd = int(np.diff(ms_h).max())
    P, ms = _up(pan["P"]), _up(ms_h)
    out = engine.pipeline(P, ms, 12, 1, 10)
    _, _, M, NR = engine.signal(P, ms, maxd, 12, 1)
    L, EW, CNT, NV = engine.deciles(M, NR, 10, with_nv=True)
    assert torch.equal(out.L, L) and torch.equal(out.CNT, CNT) and torch.equal(out.NV, NV)
    a, b = out.EW.cpu().numpy(), EW.cpu().numpy()
    assert np.array_equal(np.isnan(a), np.isnan(b)) and max_rel(a, b) <= 1e-13


STRESS = ["outlier", "ties", "twoval", "dense_center", "huge_range", "neg_zero", "lognormal",
          "pareto", "all_equal", "single", "empty", "one_bucket_tail", "clamped_low"]


def _stress_row(case, n=200_000):
    rng = np.random.default_rng(abs(hash(case)) % 2**32)
    if case == "outlier":
        x = rng.normal(0, 1e-3, n); x[7] = 1e6
    elif case == "ties":
        x = rng.integers(0, 5, n).astype(float)
    elif case == "twoval":
        x = np.where(rng.random(n) < 0.95, 0.1, 0.2)
    elif case == "dense_center":     # every value in one fixed-map bucket: key refinement
        x = np.concatenate([rng.normal(0, 1e-9, n - 10), rng.normal(0, 1e3, 10)])
    elif case == "huge_range":
        x = rng.normal(0, 1, n) * 10.0 ** rng.integers(-300, 300, n)
    elif case == "neg_zero":
        x = rng.choice(np.array([-0.0, 0.0, 1.0, -1.0, 2.0]), n)
    elif case == "lognormal":
        x = np.exp(rng.normal(0, 3, n)) - 1.0
    elif case == "pareto":
        x = rng.pareto(0.7, n) * np.where(rng.random(n) < 0.5, -1.0, 1.0)
    elif case == "all_equal":
        x = np.full(n, 0.37)
    elif case == "single":
        x = np.full(n, np.nan); x[12345 % n] = 0.5
        return x
    elif case == "empty":
        return np.full(n, np.nan)
    elif case == "lognormal_mild":   # momentum-like: the merged pass takes it
        x = np.exp(rng.normal(0, 0.8, n)) - 1.0
    elif case == "wave_cluster":     # 1500 ties at the median inside wave 0's cells: its list
        x = np.exp(rng.normal(0, 0.8, n)) - 1.0   # of uncertain cells overflows
        idx = np.arange(n)
        x[idx[(idx % 2048) < 256][:1500]] = np.median(x)
    elif case == "one_bucket_tail":  # most of the row above the top clamp (x >= 15)
        x = 15.0 + rng.exponential(1.0, n); x[:1000] = rng.normal(0, 0.1, 1000)
    else:                            # clamped_low: most of the row below -15/16
        x = -0.9375 - rng.random(n) * 0.0625; x[:500] = rng.normal(0.1, 0.2, 500)
    x[rng.random(n) < 0.05] = np.nan
    return x


@pytest.mark.parametrize("case", STRESS)
def test_deciles_ids_stress(engine, case):
    x = _stress_row(case)
    M = _up(x[None, :])
    L, _, _, NV = engine.deciles_ids(M, None, _ids_dev(x[None, :]), 10, with_nv=True)
    assert np.array_equal(L.cpu().numpy()[0], _oracle_labels(x)), case
    assert int(NV.cpu()[0]) == int((~np.isnan(x)).sum())


@pytest.mark.parametrize("n_bins", [2, 3, 4, 5, 10, 20])
def test_deciles_ids_nbins_with_means(engine, n_bins):
    pan = _panel(N=20_000, T=520, seed=n_bins)
    ms_h = pan["month_start"]
    P, ms = _up(pan["P"]), _up(ms_h)
    _, _, M, NR, IDS = engine.signal_ids(P, ms, int(np.diff(ms_h).max()), 6, 1)
    L, EW, CNT, NV = engine.deciles_ids(M, NR, IDS, n_bins, with_nv=True)
    m, nr = M.cpu().numpy(), NR.cpu().numpy()
    refL = O.assign_deciles(m, n_bins)
    assert np.array_equal(L.cpu().numpy(), refL)
    rEW, rCNT, _ = O.portfolio_ew(refL, nr, n_bins)
    assert np.array_equal(CNT.cpu().numpy(), rCNT)
    assert max_rel(EW.cpu().numpy(), rEW) <= REL


def test_deciles_ids_rejects_bad_layout(engine):
    import csmom
    M = torch.zeros((2, 18), dtype=torch.float64, device="cuda:0")   # N % 4 != 0
    ids = torch.zeros((2, 18), dtype=torch.int16, device="cuda:0")
    with pytest.raises(csmom.CsmError):
        engine.deciles_ids(M, None, ids, 10)


def test_pipeline_narrow_rows_fall_back(engine):
    """Rows at or below the narrow-row width (and N % 4 != 0) take signal + deciles without ids:
    same results as the stage-wise calls."""
    z = load_golden("edge")
    for P_h in (z["P"], z["P"][:, :-2]):
        ms_h = z["month_start"].astype(np.int64)
        out = engine.pipeline(_up(P_h), _up(ms_h), 12, 1, 10)
        ref = O.pipeline(P_h, ms_h, 12, 1, 10)
        assert np.array_equal(out.L.cpu().numpy(), ref["L"])
        assert max_rel(out.LS.cpu().numpy(), ref["LS"]) <= REL


MERGE_CASES = STRESS + ["lognormal_mild", "wave_cluster"]


@pytest.fixture
def tune_merge(engine):
    lib = engine.lib
    yield lambda v: lib.csm_tune(b"dec_merge", v)
    lib.csm_tune(b"dec_merge", 1)


@pytest.mark.parametrize("case", MERGE_CASES)
def test_deciles_ids_merged_equals_general(engine, tune_merge, case):
    """The merged decile pass (one sweep of ids + next_ret; the general kernel for the rows it
    leaves) equals the general kernel alone: labels, counts, ranked rows bit for bit, means
    within 1e-13; labels equal the oracle's qcut.  Three rows per case: the case, a mild
    momentum-like row, and the case again with other next_ret."""
    rng = np.random.default_rng(7)
    x = np.stack([_stress_row(case), _stress_row("lognormal_mild"), _stress_row(case)])
    nr = rng.normal(0.01, 0.1, x.shape)
    nr[rng.random(x.shape) < 0.03] = np.nan
    M, NR, IDS = _up(x), _up(nr), _ids_dev(x)
    got = {}
    for v in (1, 0):
        assert tune_merge(v) == 0
        got[v] = engine.deciles_ids(M, NR, IDS, 10, with_nv=True)
    (L1, EW1, C1, N1), (L0, EW0, C0, N0) = got[1], got[0]
    assert torch.equal(L1, L0) and torch.equal(C1, C0) and torch.equal(N1, N0), case
    a, b = EW1.cpu().numpy(), EW0.cpu().numpy()
    assert np.array_equal(np.isnan(a), np.isnan(b)) and max_rel(a, b) <= 1e-13, case
    for r in range(x.shape[0]):
        assert np.array_equal(L1.cpu().numpy()[r], _oracle_labels(x[r])), (case, r)
    rEW, rCNT, _ = O.portfolio_ew(np.stack([_oracle_labels(x[r]) for r in range(3)]), nr, 10)
    assert np.array_equal(C1.cpu().numpy(), rCNT)
    assert max_rel(a, rEW) <= REL


@pytest.mark.parametrize("N", [4_000, 20_000])   # narrow rows: one launch; wide: two
@pytest.mark.parametrize("merge", [1, 0])
def test_deciles_ids_fused_long_short(engine, tune_merge, N, merge):
    """csm_deciles_ids_ls (run_demo.py:46-67 in one launch: the decile pass's last workgroup
    forms the long-short) equals csm_deciles_ids + csm_long_short bit for bit, call after call
    (the context's arrival counter resets itself), with the merged pass and without."""
    pan = _panel(N=N, T=700, seed=N % 31 + merge)
    ms_h = pan["month_start"]
    P, ms = _up(pan["P"]), _up(ms_h)
    _, _, M, NR, IDS = engine.signal_ids(P, ms, int(np.diff(ms_h).max()), 12, 1)
    assert tune_merge(merge) == 0
    L2, EW2, CNT2, NV2 = engine.deciles_ids(M, NR, IDS, 10, with_nv=True)
    ref = engine.long_short(EW2, CNT2).cpu().numpy()
    for _ in range(3):
        LS = engine.empty((M.shape[0],))
        L, EW, CNT, NV = engine.deciles_ids(M, NR, IDS, 10, with_nv=True, LS=LS)
        assert torch.equal(L, L2) and torch.equal(CNT, CNT2) and torch.equal(NV, NV2)
        assert bits_equal(EW.cpu().numpy(), EW2.cpu().numpy())
        assert bits_equal(LS.cpu().numpy(), ref)
    refL = O.assign_deciles(M.cpu().numpy(), 10)
    _, _, LS_r = O.portfolio_ew(refL, NR.cpu().numpy(), 10)
    assert np.array_equal(L.cpu().numpy(), refL) and max_rel(LS.cpu().numpy(), LS_r) <= REL


@pytest.mark.parametrize("case", ["ties", "twoval", "wave_cluster", "lognormal_mild", "empty"])
def test_narrow_fallback_rows_with_long_short(engine, case):
    """Narrow rows the merged pass gives up (ties across edges, a list overflow) take the general
    path in the same workgroup; the fused long-short still sees every row's means."""
    rng = np.random.default_rng(5)
    x = np.stack([_stress_row(case, n=8192), _stress_row("lognormal_mild", n=8192),
                  _stress_row(case, n=8192)])
    nr = rng.normal(0.01, 0.1, x.shape)
    M, NR, IDS = _up(x), _up(nr), _ids_dev(x)
    LS = engine.empty((3,))
    L, EW, CNT, _ = engine.deciles_ids(M, NR, IDS, 10, LS=LS)
    for r in range(3):
        assert np.array_equal(L.cpu().numpy()[r], _oracle_labels(x[r])), (case, r)
    assert bits_equal(LS.cpu().numpy(), engine.long_short(EW, CNT).cpu().numpy())


@pytest.fixture
def tune_split(engine):
    lib = engine.lib
    yield lambda v, pf=0: lib.csm_tune(b"dec_split", v) or lib.csm_tune(b"dec_split_pf", pf)
    lib.csm_tune(b"dec_split", 2)
    lib.csm_tune(b"dec_split_pf", 0)


@pytest.mark.parametrize("case", MERGE_CASES)
def test_deciles_ids_split_equals_merged(engine, tune_split, case):
    """The split decile pass (plan -> chunked sweep -> finish, the general kernel for the rows
    it leaves) against the one-workgroup-per-row merged pass: labels, counts, ranked rows AND
    decile means bit for bit (the merged pass sums in the split pass's chunk order,
    DEC_CHUNK_ORDER), with either split sweep (prefetching / two workgroups per CU); labels
    equal the oracle's."""
    rng = np.random.default_rng(11)
    x = np.stack([_stress_row(case), _stress_row("lognormal_mild"), _stress_row(case)])
    nr = rng.normal(0.01, 0.1, x.shape)
    nr[rng.random(x.shape) < 0.03] = np.nan
    M, NR, IDS = _up(x), _up(nr), _ids_dev(x)
    got = {}
    for v, pf in ((1, 1), (1, 0), (0, 0)):
        assert tune_split(v, pf) == 0
        got[v, pf] = engine.deciles_ids(M, NR, IDS, 10, with_nv=True)
    (L1, EW1, C1, N1), (L0, EW0, C0, N0) = got[1, 1], got[0, 0]
    assert torch.equal(L1, L0) and torch.equal(C1, C0) and torch.equal(N1, N0), case
    assert bits_equal(EW1.cpu().numpy(), EW0.cpu().numpy()), case
    for a, b in zip(got[1, 0], got[1, 1]):
        assert bits_equal(a.cpu().numpy(), b.cpu().numpy()), case
    for r in range(x.shape[0]):
        assert np.array_equal(L1.cpu().numpy()[r], _oracle_labels(x[r])), (case, r)
    L2, _, _, _ = engine.deciles_ids(M, None, IDS, 10)          # labels only (no next_ret)
    assert torch.equal(L2, L1), case


@pytest.mark.parametrize("N,T", [(40_000, 2_200), (16_388, 900), (65_536, 700)])
def test_pipeline_split_equals_merged(engine, tune_split, N, T):
    """The C4 path (csm_pipeline: signal + ids -> decile pass -> long-short) with the split and
    the merged decile pass: labels / counts / means / long-short bit for bit, and the split
    pass's labels equal the oracle's qcut; rows of one, several and a partial chunk."""
    pan = _panel(N=N, T=T, seed=N % 97)
    P, ms = _up(pan["P"]), _up(pan["month_start"])
    got = {}
    for v in (1, 0):
        assert tune_split(v) == 0
        got[v] = engine.pipeline(P, ms, 12, 1, 10)
    a, b = got[1], got[0]
    assert torch.equal(a.L, b.L) and torch.equal(a.CNT, b.CNT) and torch.equal(a.NV, b.NV)
    for k in ("EW", "LS"):
        assert bits_equal(getattr(a, k).cpu().numpy(), getattr(b, k).cpu().numpy()), k
    assert np.array_equal(a.L.cpu().numpy(), O.assign_deciles(a.M.cpu().numpy(), 10))


@pytest.mark.parametrize("cells", [32768, 8192])
def test_chunk_order_merged_equals_split_any_row_count(engine, tune_split, cells):
    """The pass is chosen by the launch's row count (auto: the split pass below n_CU / 2 rows),
    so a long one-GPU panel (merged pass) and its short date slices (split pass) must still give
    the same decile means bit for bit: the 150-month panel ranked in one launch against its
    rows ranked 20 at a time, under the default auto choice, at the default and a small chunk
    width (more chunks per row, odd chunk counts)."""
    lib = engine.lib
    pan = _panel(N=24_000, T=3_300, seed=29)
    P, ms = _up(pan["P"]), _up(pan["month_start"])
    _, _, M, NR, IDS = engine.signal_ids(P, ms, int(np.diff(pan["month_start"]).max()), 12, 1)
    T_m = M.shape[0]
    assert 2 * T_m > engine.cus and 2 * 20 <= engine.cus   # merged whole, split in slices
    try:
        assert lib.csm_tune(b"dec_split_cells", cells) == 0
        assert tune_split(2) == 0
        L, EW, CNT, _ = engine.deciles_ids(M, NR, IDS, 10)
        parts = []
        for t0 in range(0, T_m, 20):
            sl = slice(t0, min(T_m, t0 + 20))
            parts.append(engine.deciles_ids(M[sl].contiguous(), NR[sl].contiguous(),
                                            IDS[sl].contiguous(), 10))
    finally:
        lib.csm_tune(b"dec_split_cells", 32768)
    assert torch.equal(L, torch.cat([p[0] for p in parts]))
    assert torch.equal(CNT, torch.cat([p[2] for p in parts]))
    assert bits_equal(EW.cpu().numpy(), torch.cat([p[1] for p in parts]).cpu().numpy())
    assert np.array_equal(L.cpu().numpy(), O.assign_deciles(M.cpu().numpy(), 10))


def test_pipeline_deciles_repeatable(engine):
    """The wide-row decile pass on ids is deterministic (fixed summation order): two pipeline
    calls give the same bits; labels equal the oracle's on every date."""
    pan = _panel(N=36_000, T=900, seed=21)
    P, ms = _up(pan["P"]), _up(pan["month_start"])
    a = engine.pipeline(P, ms, 12, 1, 10)
    b = engine.pipeline(P, ms, 12, 1, 10)
    for k in ("M", "NR", "EW", "LS"):
        assert bits_equal(getattr(a, k).cpu().numpy(), getattr(b, k).cpu().numpy()), k
    assert torch.equal(a.L, b.L) and torch.equal(a.CNT, b.CNT)
    assert np.array_equal(a.L.cpu().numpy(), O.assign_deciles(a.M.cpu().numpy(), 10))


# ---- sweeps: csm_momentum_multi_ids -> csm_deciles_ids on narrow rows (1024 buckets = ids >> 3)

def _month_panel(N, T_m, seed):
    """Month prices with gaps: absent months, missing prices, late listings."""
    rng = np.random.default_rng(seed)
    r = rng.normal(0.01, 0.08, (T_m, N))
    pm = 20.0 * np.exp(np.cumsum(r, axis=0))
    pm[rng.random((T_m, N)) < 0.02] = np.nan
    absent = rng.random((T_m, N)) < 0.01
    start = rng.integers(0, T_m // 3, N)
    absent |= np.arange(T_m)[:, None] < start[None, :]
    pm[absent] = O.absent_scalar()
    return pm


MJ_REG_DEFAULT = 2


def test_momentum_multi_ids_bit_identical(engine):
    """The id-writing multi-J scan: M / NR equal the plain multi-J scan bit for bit, and every
    id is the fixed map of its mom_J."""
    pm = _month_panel(3_000, 300, 5)
    PM = _up(pm)
    Js = (3, 6, 9, 12)
    lib = engine.lib
    try:
        assert lib.csm_tune(b"mj_reg", 1) == 0
        plain = engine.momentum_multi(PM, Js, 1)
        for mj_reg in (2, 1, 0):   # two assets per lane, one, the LDS ring
            assert lib.csm_tune(b"mj_reg", mj_reg) == 0
            with_ids = engine.momentum_multi(PM, Js, 1, with_ids=True)
            for (M0, NR0), (M1, NR1, IDS) in zip(plain, with_ids):
                assert bits_equal(M1.cpu().numpy(), M0.cpu().numpy()), mj_reg
                assert bits_equal(NR1.cpu().numpy(), NR0.cpu().numpy()), mj_reg
                assert np.array_equal(IDS.cpu().numpy().view(np.uint16), fixed_ids(M0.cpu().numpy()))
            for (M0, NR0), (M1, NR1) in zip(plain, engine.momentum_multi(PM, Js, 1)):
                assert bits_equal(M1.cpu().numpy(), M0.cpu().numpy()), mj_reg
                assert bits_equal(NR1.cpu().numpy(), NR0.cpu().numpy()), mj_reg
    finally:
        lib.csm_tune(b"mj_reg", MJ_REG_DEFAULT)


@pytest.mark.parametrize("width", [4_000, 5_000, 16_384])
def test_deciles_ids_narrow_rows(engine, tune_merge, width):
    """Rows of sweep width through csm_deciles_ids (narrow kernel, the fixed map coarsened to
    1024 buckets): every stress case and momentum-like rows; labels and counts equal the
    oracle's qcut and the streaming kernel's, means within 1e-10; the merged pass equals the
    general kernel alone."""
    rng = np.random.default_rng(width)
    cases = MERGE_CASES + ["lognormal_mild"] * 4
    x = np.stack([_stress_row(c, n=width) for c in cases])
    nr = rng.normal(0.01, 0.1, x.shape)
    nr[rng.random(x.shape) < 0.03] = np.nan
    M, NR, IDS = _up(x), _up(nr), _ids_dev(x)
    got = {}
    for v in (1, 0):
        assert tune_merge(v) == 0
        got[v] = engine.deciles_ids(M, NR, IDS, 10, with_nv=True)
    (L1, EW1, C1, N1), (L0, EW0, C0, N0) = got[1], got[0]
    assert torch.equal(L1, L0) and torch.equal(C1, C0) and torch.equal(N1, N0)
    refL = np.stack([_oracle_labels(x[r]) for r in range(x.shape[0])])
    assert np.array_equal(L1.cpu().numpy(), refL)
    Ls, _, _, _ = engine.deciles(M, None, 10)   # streaming narrow kernel
    assert torch.equal(Ls, L1)
    rEW, rCNT, _ = O.portfolio_ew(refL, nr, 10)
    assert np.array_equal(C1.cpu().numpy(), rCNT)
    a = EW1.cpu().numpy()
    assert np.array_equal(np.isnan(a), np.isnan(rEW)) and max_rel(a, rEW) <= REL
    assert max_rel(a, EW0.cpu().numpy()) <= 1e-13
    Lz, _, _, _ = engine.deciles_ids(M, None, IDS, 10)   # labels only (the sweep's call)
    assert torch.equal(Lz, L1)


def _legs_consistent(full, legs, n_bins):
    """legs-mode labels against exact ones: deciles 0 / n_bins - 1 and NaN cells identical, every
    other ranked cell inside [1, n_bins - 2]."""
    top = n_bins - 1
    assert np.array_equal(full == 0, legs == 0) and np.array_equal(full == top, legs == top)
    assert np.array_equal(full == -1, legs == -1)
    mid = (full > 0) & (full < top)
    assert ((legs[mid] >= 1) & (legs[mid] <= top - 1)).all()


@pytest.mark.parametrize("width", [4_000, 5_000, 16_384, 36_000])
@pytest.mark.parametrize("n_bins", [2, 3, 4, 5, 10, 20])
def test_deciles_ids_legs(engine, width, n_bins):
    """csm_deciles_ids_legs (the sweeps' labels before legs-only accounting): on every stress
    case and momentum-like rows the legs and NaN labels equal csm_deciles_ids's and the oracle's
    qcut, the interior ones lie in [1, n_bins - 2], NV is equal; n_bins < 4: identical labels.
    Narrow rows (merged pass of the 2048-bucket kernel) and a wide one (8192 buckets)."""
    cases = MERGE_CASES + ["lognormal_mild"] * 4
    x = np.stack([_stress_row(c, n=width) for c in cases])
    M, IDS = _up(x), _ids_dev(x)
    Lf, _, _, Nf = engine.deciles_ids(M, None, IDS, n_bins, with_nv=True)
    Ll, _, _, Nl = engine.deciles_ids(M, None, IDS, n_bins, with_nv=True, legs=True)
    assert torch.equal(Nf, Nl)
    if n_bins < 4:
        assert torch.equal(Lf, Ll)
        return
    lf, ll = Lf.cpu().numpy(), Ll.cpu().numpy()
    _legs_consistent(lf, ll, n_bins)
    _legs_consistent(O.assign_deciles(x, n_bins), ll, n_bins)
    if n_bins == 10:   # the legs mode ran: interior labels differ somewhere
        assert (lf != ll).any()


@pytest.mark.parametrize("boot", [False, True])
def test_sweep_legs_labels_same_table(engine, boot):
    """SweepConfig.legs_labels (the decile pass selects only the legs' edges before legs-only
    accounting): the summary table equals legs_labels=False bit for bit -- a month-price batch
    with gaps, and a bootstrap batch (csm_boot_scan)."""
    from csmom.sweep import SweepConfig, SweepRunner
    pm = _month_panel(2_000, 240, 11)
    runs = {}
    for ll in (True, False):
        sr = SweepRunner(engine, SweepConfig(legs_labels=ll))
        if boot:
            R, _, _ = engine.momentum(_up(pm), 12, 1, with_ret=True)
            runs[ll] = sr.run_boot_batch(R.contiguous(), 3, 0)[0]
        else:
            B = 3
            PMb = _up(np.concatenate([pm, pm[:, ::-1], pm * 1.5], axis=1))
            runs[ll] = sr.run_batch(PMb, B)[0]
    assert bits_equal(runs[True].cpu().numpy(), runs[False].cpu().numpy())


def test_sweep_batch_ids_equal_streaming(engine):
    """SweepRunner.run_batch with the id path (default) equals decile_ids=False: the summary
    table bit for bit (the labels are identical, so every later stage is)."""
    import csmom
    from csmom.sweep import SweepConfig, SweepRunner
    pm = _month_panel(2_000, 240, 9)
    B = 3
    PMb = _up(np.concatenate([pm, pm[:, ::-1], pm * 1.5], axis=1))
    a, _ = SweepRunner(engine, SweepConfig()).run_batch(PMb, B)
    b, _ = SweepRunner(engine, SweepConfig(decile_ids=False)).run_batch(PMb, B)
    assert bits_equal(a.cpu().numpy(), b.cpu().numpy())


@pytest.mark.parametrize("N,T,J,skip,n_bins", [(5_000, 6_522, 12, 1, 10), (1_000, 2_600, 3, 0, 5),
                                               (4_004, 1_500, 9, 2, 10)])
def test_chunked_scan_ids_deciles(engine, N, T, J, skip, n_bins):
    """The bench's C2 path (csm_month_end -> csm_momentum_chunked_ids -> csm_deciles_ids on
    narrow rows -> csm_long_short) at C2 size: R / M / NR bit for bit the chunked scan's without
    ids, ids = the fixed map of mom_J, labels / counts = the streaming decile pass's and the
    oracle's qcut on every date, means and long-short within 1e-10 of the oracle's portfolio."""
    pan = _panel(N=N, T=T, seed=23)
    P, ms = _up(pan["P"]), _up(pan["month_start"])
    PM, _ = engine.month_end(P, ms)
    T_m = PM.shape[0]
    C = engine.default_chunks(T_m, N, J, skip)
    assert C > 1
    IDS = engine.empty((T_m, N), torch.int16)
    R1, M1, NR1 = engine.momentum_chunked(PM, J, skip, with_ret=True, ids=IDS)
    R0, M0, NR0 = engine.momentum_chunked(PM, J, skip, with_ret=True)
    for a, b in ((R1, R0), (M1, M0), (NR1, NR0)):
        assert bits_equal(a.cpu().numpy(), b.cpu().numpy())
    Mh = M1.cpu().numpy()
    assert np.array_equal(IDS.cpu().numpy().view(np.uint16), fixed_ids(Mh))
    L, EW, CNT, NV = engine.deciles_ids(M1, NR1, IDS, n_bins, with_nv=True)
    Ls, EWs, CNTs, NVs = engine.deciles(M1, NR1, n_bins, with_nv=True)
    assert torch.equal(L, Ls) and torch.equal(CNT, CNTs) and torch.equal(NV, NVs)
    refL = O.assign_deciles(Mh, n_bins)
    assert np.array_equal(L.cpu().numpy(), refL)
    rEW, rCNT, _ = O.portfolio_ew(refL, NR1.cpu().numpy(), n_bins)
    assert np.array_equal(CNT.cpu().numpy(), rCNT)

    def same(a, b):   # NaN / inf cells equal (cent prices can reach 0: inf next_ret, as pandas)
        fa, fb = np.isfinite(a), np.isfinite(b)
        assert np.array_equal(fa, fb) and np.array_equal(a[~fa], b[~fb], equal_nan=True)
        assert max_rel(a[fa], b[fb]) <= REL
    same(EW.cpu().numpy(), rEW)
    same(EWs.cpu().numpy(), rEW)
    same(engine.long_short(EW, CNT).cpu().numpy(), O.long_short(rEW, rCNT))


def test_chunked_scan_ids_rejects_bad_args(engine):
    import csmom
    PM = engine.empty((30, 1002))
    with pytest.raises(csmom.CsmError):
        engine.momentum_chunked(PM, 12, 1, chunks=2, ids=engine.empty((30, 1002), torch.int16))


@pytest.mark.parametrize("N,T,Js,skip,C", [
    (5_000, 6_522, (3, 6, 9, 12), 1, None),   # C3's panel and grid, default chunks
    (1_000, 2_600, (3, 12), 1, 7),
    (2_002, 1_500, (2, 5, 9), 0, 3),          # N % 4 != 0: no ids
    (640, 2_600, (12, 3, 6, 9), 1, 40),       # chunks shorter than a window
    (1_000, 2_600, (4,), 2, 5),
])
def test_multi_chunked_scan_equals_per_j(engine, N, T, Js, skip, C):
    """csm_momentum_multi_chunked (one summary / fold for max(J) + each J's subset-ffilled
    price, one chunked multi-J scan): every J's M / NR bit for bit the plain per-J scan's, ids the
    fixed map of mom_J."""
    pan = _panel(N=N, T=T, seed=29)
    PM, _ = engine.month_end(_up(pan["P"]), _up(pan["month_start"]))
    T_m = PM.shape[0]
    C = C or engine.default_chunks(T_m, N, max(Js), skip)
    assert C > 1
    ids = N % 4 == 0
    outs = engine.momentum_multi(PM, Js, skip, with_ids=ids, chunks=C)
    for J, o in zip(Js, outs):
        _, M0, NR0 = engine.momentum(PM, J, skip, chunked="never")
        assert bits_equal(o[0].cpu().numpy(), M0.cpu().numpy()), J
        assert bits_equal(o[1].cpu().numpy(), NR0.cpu().numpy()), J
        if ids:
            assert np.array_equal(o[2].cpu().numpy().view(np.uint16), fixed_ids(M0.cpu().numpy())), J


def test_joined_sweep_multi_chunked_equals_per_j(engine):
    """A single-panel sweep batch (C3's joined path) ranks from the chunked multi-J scan's ids:
    the summary table equals the per-J chunked scans' bit for bit."""
    import csmom
    pan = _panel(N=5_000, T=6_522, seed=31)
    PM, _ = engine.month_end(_up(pan["P"]), _up(pan["month_start"]))
    W = PM.abs() * 1e6
    ADV = W * 0.01
    kw = dict(Js=(3, 6, 9, 12), Ks=(3, 6, 9, 12), skip=1, aum=1e8)
    a, _ = csmom.SweepRunner(engine, csmom.SweepConfig(**kw)).run_batch(PM, 1, W=W, ADV=ADV)
    b, _ = csmom.SweepRunner(engine, csmom.SweepConfig(multi_j_scan=False, **kw)).run_batch(
        PM, 1, W=W, ADV=ADV)
    assert bits_equal(a.cpu().numpy(), b.cpu().numpy())


def test_multi_chunked_scan_rejects_bad_args(engine):
    import csmom
    pm = _up(_month_panel(1_000, 120, 5))
    with pytest.raises(csmom.CsmError):
        engine.momentum_multi(pm, (16,), 1, chunks=4)             # max(J) + skip > 16
    with pytest.raises(csmom.CsmError):
        engine.momentum_multi(_up(_month_panel(999, 120, 5)), (3,), 1, chunks=4)   # odd N
