"""GPU parity: the HIP engine (through the C ABI) against the reference's golden fixtures.

Bar: bit-exact for month prices, volumes, ret_1m, mom_J, next_ret and labels; decile means
and long-short within 1e-10 relative (north_star; pandas sums with Kahan in row order, the
engine with a deterministic double-double tree).
"""
import numpy as np
import pytest
import torch

from conftest import bits_equal, golden_tags, load_golden, max_rel, parse_tag
from oracle import csmom_oracle as O

pytestmark = pytest.mark.gpu
REL = 1e-10


def _up(x, dev="cuda:0"):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


@pytest.mark.parametrize("name", ["real_data", "edge", "small", "longwin", "c1"])
def test_fixture_pipeline(engine, name):
    z = load_golden(name)
    P = _up(z["P"])
    V = _up(z["V"]) if "V" in z.files else None
    ms = _up(z["month_start"].astype(np.int64))
    PM, VOL = engine.month_end(P, ms, V)
    pm = PM.cpu().numpy()
    tags = golden_tags(z)
    key = lambda k: k if k in z.files else f"{tags[0]}_{k}"   # real_data prefixes every key
    full = key("PM") in z.files
    assert (O.is_absent(pm) == (z[key("present")] == 0)).all()
    if full:
        assert bits_equal(pm, z[key("PM")])
        if V is not None:
            assert bits_equal(VOL.cpu().numpy(), z[key("VOL")])
    else:
        idx = z["sample_idx"]
        assert bits_equal(pm.reshape(-1)[idx], z["PM_sample"])
    for tag in golden_tags(z):
        J, s = parse_tag(tag)
        R, M, NR = engine.momentum(PM, J, s, with_ret=True, chunked=False)
        L, EW, CNT, NV = engine.deciles(M, NR, 10, with_nv=True)
        LS = engine.long_short(EW, CNT)
        r, m, nr = R.cpu().numpy(), M.cpu().numpy(), NR.cpu().numpy()
        if full:
            assert bits_equal(r, z[key("R")]), tag
            assert bits_equal(m, z[f"{tag}_M"]), tag
            assert bits_equal(nr, z[f"{tag}_NR"]), tag
        else:
            idx = z["sample_idx"]
            assert bits_equal(m.reshape(-1)[idx], z[f"{tag}_M_sample"]), tag
            assert bits_equal(nr.reshape(-1)[idx], z[f"{tag}_NR_sample"]), tag
            import hashlib
            dig = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
            # NaN payloads may differ from pandas' canonical NaN: canonicalise first
            canon = lambda a: np.where(np.isnan(a), np.nan, a)
            assert dig(canon(m)) == str(z[f"{tag}_M_sha256"]), tag
            assert dig(canon(nr)) == str(z[f"{tag}_NR_sha256"]), tag
        assert np.array_equal(L.cpu().numpy(), z[f"{tag}_L"]), tag
        ew = EW.cpu().numpy()
        assert np.array_equal(np.isnan(ew), np.isnan(z[f"{tag}_EW"])), tag
        assert max_rel(ew, z[f"{tag}_EW"]) <= REL, tag
        ls = LS.cpu().numpy()
        assert np.array_equal(np.isnan(ls), np.isnan(z[f"{tag}_LS"])), tag
        assert max_rel(ls, z[f"{tag}_LS"]) <= REL, tag
        keep = ls[~np.isnan(ls)]
        if len(keep):
            assert abs(keep.mean() - float(z[f"{tag}_mean"])) <= REL * abs(float(z[f"{tag}_mean"]))


def test_decile_cases(engine):
    d = load_golden("deciles")
    v, o, lab = d["values"], d["offsets"], d["labels"]
    small = [i for i in range(len(o) - 1) if o[i + 1] - o[i] <= 64]
    W = 64
    M = np.full((len(small), W), np.nan)
    ref = np.full((len(small), W), -1, dtype=np.int8)
    for r, i in enumerate(small):
        x = v[o[i]:o[i + 1]]
        M[r, :len(x)] = x
        li = lab[o[i]:o[i + 1]]
        ref[r, :len(x)] = np.where(np.isnan(li), -1, li).astype(np.int8)
    L, _, _, NV = engine.deciles(_up(M), None, 10, with_nv=True)
    assert np.array_equal(L.cpu().numpy(), ref)
    for i in range(len(o) - 1):
        if o[i + 1] - o[i] <= 64:
            continue
        x = v[o[i]:o[i + 1]]
        n = len(x) + (len(x) & 1)
        row = np.full((1, n), np.nan)
        row[0, :len(x)] = x
        L, _, _, _ = engine.deciles(_up(row), None, 10)
        li = lab[o[i]:o[i + 1]]
        assert np.array_equal(L.cpu().numpy()[0, :len(x)], np.where(np.isnan(li), -1, li).astype(np.int8))


def _oracle_labels(row, n_bins=10):
    ok = ~np.isnan(row)
    out = np.full(len(row), -1, dtype=np.int8)
    if ok.any():
        lab = O.qcut_labels(row[ok], n_bins)
        out[ok] = np.where(np.isnan(lab), -1, lab).astype(np.int8)
    return out


STRESS = ["outlier", "ties", "twoval", "dense_center", "huge_range", "neg_zero", "odd_n",
          "lognormal", "pareto"]


def _stress_row(case, n=200_000):
    rng = np.random.default_rng(hash(case) % 2**32)
    if case == "outlier":
        x = rng.normal(0, 1e-3, n); x[7] = 1e6
    elif case == "ties":
        x = rng.integers(0, 5, n).astype(float)
    elif case == "twoval":
        x = np.where(rng.random(n) < 0.95, 0.1, 0.2)
    elif case == "dense_center":
        x = np.concatenate([rng.normal(0, 1e-9, n - 10), rng.normal(0, 1e3, 10)])
    elif case == "huge_range":
        x = rng.normal(0, 1, n) * 10.0 ** rng.integers(-300, 300, n)
    elif case == "neg_zero":
        x = rng.choice(np.array([-0.0, 0.0, 1.0, -1.0, 2.0]), n)
    elif case == "lognormal":   # momentum after long gaps: the bulk squeezed by the tail
        x = np.exp(rng.normal(0, 3, n)) - 1.0
    elif case == "pareto":
        x = rng.pareto(0.7, n) * np.where(rng.random(n) < 0.5, -1.0, 1.0)
    else:
        n = 100_001
        x = rng.standard_normal(n)
    x[rng.random(n) < 0.05] = np.nan
    return x


@pytest.mark.parametrize("case", STRESS)
def test_decile_stress(engine, case):
    """Cross-sections that overflow the candidate buffer and force key-space refinement."""
    x = _stress_row(case)
    row = x[None, :]
    L, _, _, _ = engine.deciles(_up(row), None, 10)
    assert np.array_equal(L.cpu().numpy()[0], _oracle_labels(x))
    xs = x[:12_000]  # the narrow-row kernel (1024 buckets) on the same pathologies
    Ls, _, _, _ = engine.deciles(_up(xs[None, :]), None, 10)
    assert np.array_equal(Ls.cpu().numpy()[0], _oracle_labels(xs))


@pytest.mark.parametrize("n_bins", [2, 3, 4, 5, 10, 20])
def test_nbins(engine, n_bins):
    z = load_golden("edge")
    P, ms = _up(z["P"]), _up(z["month_start"].astype(np.int64))
    PM, _ = engine.month_end(P, ms)
    _, M, NR = engine.momentum(PM, 3, 0)
    L, EW, CNT, _ = engine.deciles(M, NR, n_bins)
    LS = engine.long_short(EW, CNT)
    m, nr = M.cpu().numpy(), NR.cpu().numpy()
    refL = O.assign_deciles(m, n_bins)
    assert np.array_equal(L.cpu().numpy(), refL)
    rEW, rCNT, rLS = O.portfolio_ew(refL, nr, n_bins)
    assert np.array_equal(CNT.cpu().numpy(), rCNT)
    assert max_rel(EW.cpu().numpy(), rEW) <= REL
    assert bits_equal(np.isnan(LS.cpu().numpy()), np.isnan(rLS))
    assert max_rel(LS.cpu().numpy(), rLS) <= REL


def test_odd_n_scalar_path(engine):
    """N odd selects the scalar (8-B/lane) kernels; results must not change."""
    z = load_golden("edge")
    P = z["P"][:, :-1]
    V = z["V"][:, :-1]
    ms = z["month_start"].astype(np.int64)
    ref = O.pipeline(P, ms, 12, 1, 10, V=V)
    out = engine.run(_up(P), _up(ms), 12, 1, 10, V=_up(V), with_ret=True)
    for k in ("PM", "VOL", "R", "M", "NR"):
        assert bits_equal(getattr(out, k).cpu().numpy(), ref[k]), k
    assert np.array_equal(out.L.cpu().numpy(), ref["L"])
    assert max_rel(out.LS.cpu().numpy(), ref["LS"]) <= REL


@pytest.mark.parametrize("name", ["edge", "longwin", "c1"])
def test_fused_signal_matches_fixtures(engine, name):
    """k_signal (fused month-end + scan) against the reference fixtures, with and without
    the unfused two-kernel path."""
    z = load_golden(name)
    P = _up(z["P"])
    ms_h = z["month_start"].astype(np.int64)
    ms = _up(ms_h)
    maxd = int(np.diff(ms_h).max())
    for tag in golden_tags(z):
        J, s = parse_tag(tag)
        out = engine.run(P, ms, J, s, 10, with_ret=True, max_month_days=maxd, fused=True)
        ref = engine.run(P, ms, J, s, 10, with_ret=True, max_month_days=maxd, fused=False)
        for k in ("PM", "R", "M", "NR", "EW", "LS"):
            assert bits_equal(getattr(out, k).cpu().numpy(), getattr(ref, k).cpu().numpy()), (tag, k)
        assert torch.equal(out.L, ref.L) and torch.equal(out.CNT, ref.CNT) and torch.equal(out.NV, ref.NV)
        assert np.array_equal(out.L.cpu().numpy(), z[f"{tag}_L"]), tag
        if "PM" in z.files:
            assert bits_equal(out.M.cpu().numpy(), z[f"{tag}_M"]), tag
            assert bits_equal(out.NR.cpu().numpy(), z[f"{tag}_NR"]), tag


def test_fused_signal_large_panel_vs_oracle(engine):
    """C2-sized daily panel (5,000 x 6,522 business days): fused path vs the oracle at full
    size -- bit-exact mom/next_ret/labels, EW/LS within 1e-10."""
    from oracle.synth_np import make_panel
    pan = make_panel(5000, 6522, seed=2, start="2000-01-03", with_volume=False)
    ms_h = pan["month_start"]
    P = _up(pan["P"])
    out = engine.run(P, _up(ms_h), 12, 1, 10, max_month_days=int(np.diff(ms_h).max()), fused=True)
    ref = O.pipeline(pan["P"], ms_h, 12, 1, 10)
    assert bits_equal(out.PM.cpu().numpy(), ref["PM"])
    assert bits_equal(out.M.cpu().numpy(), ref["M"])
    assert bits_equal(out.NR.cpu().numpy(), ref["NR"])
    assert np.array_equal(out.L.cpu().numpy(), ref["L"])
    assert np.array_equal(out.CNT.cpu().numpy(), ref["CNT"])
    assert max_rel(out.EW.cpu().numpy(), ref["EW"]) <= REL
    assert max_rel(out.LS.cpu().numpy(), ref["LS"]) <= REL


def test_fused_odd_n_and_variants(engine):
    """Odd N runs the fused kernel with one asset per lane; both assets-per-lane paths give the
    same bits on an even panel."""
    z = load_golden("edge")
    P = z["P"][:, :-1]
    ms_h = z["month_start"].astype(np.int64)
    maxd = int(np.diff(ms_h).max())
    ref = O.pipeline(P, ms_h, 12, 1, 10)
    out = engine.run(_up(P), _up(ms_h), 12, 1, 10, max_month_days=maxd, fused=True)
    for k in ("PM", "M", "NR"):
        assert bits_equal(getattr(out, k).cpu().numpy(), ref[k]), k
    assert np.array_equal(out.L.cpu().numpy(), ref["L"])
    P2, ms2 = _up(z["P"]), _up(ms_h)
    base = engine.signal(P2, ms2, maxd, 12, 1, with_pm=True)
    lib = engine.lib
    try:
        for vec in (1, 2):
            assert lib.csm_tune(b"signal_vec", vec) == 0
            got = engine.signal(P2, ms2, maxd, 12, 1, with_pm=True)
            for a, b in zip(got, base):
                if a is not None:
                    assert bits_equal(a.cpu().numpy(), b.cpu().numpy()), vec
    finally:
        lib.csm_tune(b"signal_vec", 2)
    assert lib.csm_tune(b"nope", 1) != 0


@pytest.mark.parametrize("name", ["edge", "c1"])
def test_signal_block_shapes_bit_identical(engine, name):
    """The fused kernel's two block shapes -- one wave per block with four month buffers, and
    the wide panels' four barrier-free waves with two buffers and raw buffer loads (padding rows
    out of range; partial last block) -- give the same bits, for J = 12 / skip 1 and J = 3 /
    skip 0, and equal the unfused month-end."""
    z = load_golden(name)
    P = z["P"]
    if P.shape[1] % 2:
        P = P[:, :-1]
    ms_h = z["month_start"].astype(np.int64)
    maxd = int(np.diff(ms_h).max())
    Pd, ms = _up(P), _up(ms_h)
    lib = engine.lib
    try:
        for J, skip in ((12, 1), (3, 0)):
            assert lib.csm_tune(b"signal_bwf", 1) == 0
            base = engine.signal(Pd, ms, maxd, J, skip, with_pm=True, with_ret=True)
            assert lib.csm_tune(b"signal_bwf", 4) == 0
            got = engine.signal(Pd, ms, maxd, J, skip, with_pm=True, with_ret=True)
            for a, b in zip(got, base):
                if a is not None:
                    assert bits_equal(a.cpu().numpy(), b.cpu().numpy()), (J, skip)
    finally:
        lib.csm_tune(b"signal_bwf", 0)
    PM, _ = engine.month_end(Pd, ms)
    assert bits_equal(PM.cpu().numpy(), base[0].cpu().numpy())


def test_fused_rejects_long_months(engine):
    import csmom
    P2 = torch.zeros((40, 8), dtype=torch.float64, device="cuda:0")
    ms2 = torch.tensor([0, 40], dtype=torch.int64, device="cuda:0")
    with pytest.raises(csmom.CsmError):
        engine.signal(P2, ms2, 40)       # month longer than 32 days


@pytest.mark.parametrize("name", ["edge", "c1", "small", "real_data"])
def test_narrow_and_wide_decile_kernels_agree(engine, name):
    """Rows of <= 16384 assets take the narrow-row kernel (256 threads, 1024 buckets); forcing
    the wide kernel gives the same labels and counts, means equal to rounding."""
    z = load_golden(name)
    PM, _ = engine.month_end(_up(z["P"]), _up(z["month_start"].astype(np.int64)))
    _, M, NR = engine.momentum(PM, 12, 1)
    lib = engine.lib
    a = engine.deciles(M, NR, 10, with_nv=True)
    try:
        assert lib.csm_tune(b"dec_narrow_max", 0) == 0
        b = engine.deciles(M, NR, 10, with_nv=True)
    finally:
        lib.csm_tune(b"dec_narrow_max", 16384)
    assert torch.equal(a[0], b[0]) and torch.equal(a[2], b[2]) and torch.equal(a[3], b[3])
    ea, eb = a[1].cpu().numpy(), b[1].cpu().numpy()
    assert np.array_equal(np.isnan(ea), np.isnan(eb)) and max_rel(ea, eb) <= 1e-13


@pytest.mark.parametrize("name", ["edge", "c1", "longwin"])
@pytest.mark.parametrize("Js,skip", [((3, 6, 9, 12), 1), ((12,), 1), ((1, 2), 0),
                                     ((24, 48, 12, 5, 7), 2), ((16,), 0), ((14, 2), 2)])
def test_momentum_multi_equals_per_J_scans(engine, name, Js, skip):
    """csm_momentum_multi (one scan, one ring of max(J) + skip factors) equals csm_momentum per
    J bit for bit -- M and the J-dependent NR -- including > 4 look-backs (two launches)."""
    z = load_golden(name)
    PM, _ = engine.month_end(_up(z["P"]), _up(z["month_start"].astype(np.int64)))
    for mj_reg in (2, 1, 0):   # register shift ring (two assets per lane / one) and the LDS ring
        assert engine.lib.csm_tune(b"mj_reg", mj_reg) == 0
        try:
            outs = engine.momentum_multi(PM, Js, skip)
        finally:
            engine.lib.csm_tune(b"mj_reg", 2)
        assert len(outs) == len(Js)
        for J, (M, NR) in zip(Js, outs):
            _, M1, NR1 = engine.momentum(PM, J, skip, chunked=False)
            assert bits_equal(M.cpu().numpy(), M1.cpu().numpy()), (J, mj_reg)
            assert bits_equal(NR.cpu().numpy(), NR1.cpu().numpy()), (J, mj_reg)


def test_sweep_batch_multi_J_scan_equals_per_J(engine):
    """A wide sweep batch (B x N lanes fill the chip) takes the multi-J scan (multi_j_scan, the
    default); its summary table equals the per-J scan path bit for bit."""
    from csmom.sweep import SweepConfig, SweepRunner
    z = load_golden("edge")
    PM, _ = engine.month_end(_up(z["P"]), _up(z["month_start"].astype(np.int64)))
    T_m, N = PM.shape
    B = max(1, -(-140_000 // N))
    PMb = PM.repeat(1, B).contiguous()
    cfg = SweepConfig(multi_j_scan=True)
    run = SweepRunner(engine, cfg)
    a, _ = run.run_batch(PMb, B)

    class PerJ:   # the engine without momentum_multi
        def __init__(self, e):
            self._e = e

        def __getattr__(self, k):
            if k == "momentum_multi":
                raise AttributeError(k)
            return getattr(self._e, k)

    b, _ = SweepRunner(PerJ(engine), cfg).run_batch(PMb, B)
    assert bits_equal(a.cpu().numpy(), b.cpu().numpy())
