"""GPU parity of the one-launch time-chunked signal (csm_signal_chunked, k_signal_tc: C2's
month-end + scan).  Each workgroup reduces one chunk's daily rows to month prices, publishes the
chunk's record, folds the earlier chunks' records (an in-launch hand-off) and scans; the result
must be the unfused csm_month_end -> csm_momentum (features.py:34-52, run_demo.py:48) path bit
for bit: ret_1m, mom_J, next_ret and the fixed-map ids, on panels with late listings,
delistings, absent months and missing days, at every chunk count, on the reference's fixtures,
and under hipGraph replay (the sync words reset themselves)."""
import numpy as np
import pytest
import torch

from conftest import bits_equal, golden_tags, load_golden, parse_tag

pytestmark = pytest.mark.gpu


def _up(x, dev="cuda:0"):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def _panel(N, T, seed, heavy=False):
    from oracle.synth_np import make_panel
    kw = (dict(late=0.3, delist=0.3, nan_day=0.05, absent_month=0.05, nan_month=0.05)
          if heavy else dict(nan_day=0.02, absent_month=0.01, nan_month=0.01))
    return make_panel(N, T, seed=seed, start="2001-01-02", with_volume=False, cents=True, **kw)


def _fixed_ids(x):
    from test_gpu_pipeline import fixed_ids
    return fixed_ids(x)


def _check(engine, P, ms, J, skip, C=None, reps=1):
    T_m = ms.numel() - 1
    maxd = int(torch.diff(ms).max().item())
    PM, _ = engine.month_end(P, ms)
    R0, M0, NR0 = engine.momentum(PM, J, skip, with_ret=True, chunked=False)
    ws = None
    for _ in range(reps):   # the same workspace again: its sync words reset themselves
        R1, M1, NR1, IDS, ws = engine.signal_chunked(P, ms, maxd, J, skip, chunks=C,
                                                     with_ret=True, workspace=ws)
        assert not engine.signal_chunked_timed_out(ws)
        for a, b in ((R1, R0), (M1, M0), (NR1, NR0)):
            assert bits_equal(a.cpu().numpy(), b.cpu().numpy())
        assert np.array_equal(IDS.cpu().numpy().view(np.uint16), _fixed_ids(M1.cpu().numpy()))
    assert ws[16:].numel() > 0 and int(ws[:16].view(torch.int32)[[0, 1]].abs().sum()) == 0
    return M1, NR1, T_m


def test_c2_size_bits_and_chunked_path(engine):
    """C2 (5,000 assets x 6,522 days, J = 12, skip = 1, the default 21 chunks): the unfused
    scan's bits, and the four-launch chunked path's (month_end -> momentum_chunked_ids)."""
    pan = _panel(5_000, 6_522, 23)
    P, ms = _up(pan["P"]), _up(pan["month_start"])
    M1, NR1, T_m = _check(engine, P, ms, 12, 1, reps=2)
    PM, _ = engine.month_end(P, ms)
    ids = engine.empty((T_m, 5_000), torch.int16)
    _, M2, NR2 = engine.momentum_chunked(PM, 12, 1, ids=ids)
    assert bits_equal(M1.cpu().numpy(), M2.cpu().numpy())
    assert bits_equal(NR1.cpu().numpy(), NR2.cpu().numpy())


@pytest.mark.parametrize("N,T,J,skip,C", [(1_000, 2_600, 3, 0, None), (4_004, 1_500, 9, 2, 7),
                                          (2_002, 3_000, 12, 1, 64), (998, 800, 1, 1, 2),
                                          (600, 2_000, 24, 2, None), (514, 2_400, 12, 1, 13),
                                          (256, 300, 12, 1, 1), (2_050, 6_000, 12, 1, 10),
                                          (1_000, 6_000, 12, 1, None), (770, 4_000, 12, 1, 7)])
def test_gappy_panels_every_chunking(engine, N, T, J, skip, C):
    """30 % late listings, 30 % delistings, 5 % absent / all-NaN months and missing days: the
    pending next_ret rows that cross chunk boundaries (written by the chunk with the asset's
    next present row, or NaN by the last chunk), assets absent for whole chunks, one chunk.
    J = 12 / skip = 1 with chunks longer than 14 months (the last three cases) take the
    speculative scan of the idle waves: both of its outcomes -- states equal after month m0 + 13
    (its outputs stand, plus next_ret of m0 + 13 and the last present month's NaN) and unequal
    (the folding lane rescans over them) -- occur on these panels."""
    pan = _panel(N, T, 100 + N, heavy=True)
    _check(engine, _up(pan["P"]), _up(pan["month_start"]), J, skip, C)


@pytest.mark.parametrize("name", ["edge", "c1", "small", "real_data", "longwin"])
def test_fixtures(engine, name):
    """The reference-generated fixtures (tests/golden): M / NR of every tag with J + skip <= 32
    bit for bit (odd N padded with an absent column, which changes no other asset); fixtures
    that keep sampled cells and a digest of the whole panel (C1) are checked through both."""
    z = load_golden(name)
    P = z["P"]
    ms_h = z["month_start"].astype(np.int64)
    if int(np.diff(ms_h).max()) > 23:
        pytest.skip("months longer than 23 day rows: the launch refuses them")
    N = P.shape[1]
    if N % 2:
        from oracle.csmom_oracle import ABSENT_BITS
        pad = np.full((P.shape[0], 1), 0, dtype=np.uint64) + np.uint64(ABSENT_BITS)
        P = np.concatenate([P, pad.view(np.float64)], axis=1)
    Pd, ms = _up(P), _up(ms_h)
    maxd = int(np.diff(ms_h).max())
    tags = golden_tags(z)
    done = 0
    import hashlib
    dig = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    canon = lambda a: np.where(np.isnan(a), np.nan, a)   # (pandas' canonical NaN payload)
    for tag in tags:
        J, s = parse_tag(tag)
        full = f"{tag}_M" in z.files
        if J + s > 32 or not (full or f"{tag}_M_sha256" in z.files):
            continue
        _, M, NR, _, ws = engine.signal_chunked(Pd, ms, maxd, J, s)
        assert not engine.signal_chunked_timed_out(ws)
        m, nr = M.cpu().numpy()[:, :N], NR.cpu().numpy()[:, :N]
        if full:
            assert bits_equal(m, z[f"{tag}_M"]), tag
            assert bits_equal(nr, z[f"{tag}_NR"]), tag
        else:
            idx = z["sample_idx"]
            assert bits_equal(m.reshape(-1)[idx], z[f"{tag}_M_sample"]), tag
            assert bits_equal(nr.reshape(-1)[idx], z[f"{tag}_NR_sample"]), tag
            assert dig(canon(m)) == str(z[f"{tag}_M_sha256"]), tag
            assert dig(canon(nr)) == str(z[f"{tag}_NR_sha256"]), tag
        done += 1
    if not done:
        pytest.skip("no full-panel tag with J + skip <= 32")


def test_graph_replay(engine):
    """Captured as a hipGraph and replayed back to back: every replay the eager bits (the
    ticket and done counters wrap to 0, the last workgroup zeroes the flags)."""
    pan = _panel(3_000, 2_000, 5, heavy=True)
    P, ms = _up(pan["P"]), _up(pan["month_start"])
    maxd = int(np.diff(pan["month_start"]).max())
    _, M0, NR0, I0, ws = engine.signal_chunked(P, ms, maxd, 12, 1)
    M0, NR0, I0 = M0.clone(), NR0.clone(), I0.clone()
    T_m = ms.numel() - 1
    M, NR = engine.empty((T_m, 3_000)), engine.empty((T_m, 3_000))
    I = engine.empty((T_m, 3_000), torch.int16)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        engine.signal_chunked(P, ms, maxd, 12, 1, out=(None, M, NR, I), workspace=ws)
    for reps in (1, 5):
        M.fill_(0.0)
        for _ in range(reps):
            g.replay()
        torch.cuda.synchronize()
        assert not engine.signal_chunked_timed_out(ws)
        assert bits_equal(M.cpu().numpy(), M0.cpu().numpy())
        assert bits_equal(NR.cpu().numpy(), NR0.cpu().numpy())
        assert torch.equal(I, I0)


def test_rejects_bad_args(engine):
    import csmom
    pan = _panel(1_000, 800, 3)
    P, ms = _up(pan["P"]), _up(pan["month_start"])
    with pytest.raises(csmom.CsmError):   # odd N
        engine.signal_chunked(P[:, :999].contiguous(), ms, 23, 12, 1)
    with pytest.raises(csmom.CsmError):   # months longer than 23 day rows
        engine.signal_chunked(P, ms, 24, 12, 1)
    with pytest.raises(csmom.CsmError):   # more than 32 months per chunk
        engine.signal_chunked(P, ms, 23, 12, 1, chunks=1)


def test_handoff_under_uneven_load(engine):
    """The in-launch record hand-off (write-through records, one flag per record, relaxed polls,
    one agent acquire) under uneven load and with consumer caches warm from the previous launch
    of the SAME workspace: two different panels alternate through one workspace while a second
    stream streams 1 GB copies, 24 launches; every result equals its panel's eager result bit
    for bit (a stale record line from the previous launch would change the fold)."""
    pans = [_panel(5_000, 3_000, s, heavy=(s % 2 == 0)) for s in (41, 42)]
    Ps = [_up(p["P"]) for p in pans]
    mss = [_up(p["month_start"]) for p in pans]
    maxd = max(int(np.diff(p["month_start"]).max()) for p in pans)
    refs = []
    for P, ms in zip(Ps, mss):
        _, M, NR, I, _ = engine.signal_chunked(P, ms, maxd, 12, 1)
        refs.append((M.clone(), NR.clone(), I.clone()))
    ws = None
    src = torch.empty(128 * 1024 * 1024, dtype=torch.float64, device="cuda:0").uniform_()
    dst = torch.empty_like(src)
    side = torch.cuda.Stream()
    outs = []
    for it in range(24):
        k = it % 2
        with torch.cuda.stream(side):   # bandwidth pressure on other CUs meanwhile
            dst.copy_(src)
        _, M, NR, I, ws = engine.signal_chunked(Ps[k], mss[k], maxd, 12, 1, workspace=ws,
                                                check=False)
        outs.append((k, M, NR, I))
    torch.cuda.synchronize()
    assert not engine.signal_chunked_timed_out(ws)
    engine.signal_chunked_status(ws)   # (raises on a give-up mark)
    for k, M, NR, I in outs:
        assert bits_equal(M.cpu().numpy(), refs[k][0].cpu().numpy())
        assert bits_equal(NR.cpu().numpy(), refs[k][1].cpu().numpy())
        assert torch.equal(I, refs[k][2])


def test_timeout_is_loud(engine):
    """A workgroup that gives up waiting for an earlier chunk's record (forced here: the
    "tc_spins" knob at 0 gives up at the first trip) must not pass as a correct launch:
    Engine.signal_chunked raises CSM_E_TIMEOUT (csm_signal_chunked_status), an unchecked launch
    leaves the mark for the status call, the report clears it, and the next launch on the same
    workspace is correct bit for bit."""
    import csmom
    from csmom._lib import CSM_E_TIMEOUT
    lib = engine.lib
    pan = _panel(2_000, 1_500, 5)
    P, ms = _up(pan["P"]), _up(pan["month_start"])
    maxd = int(torch.diff(ms).max().item())
    _, M0, NR0, I0, ws = engine.signal_chunked(P, ms, maxd, 12, 1, chunks=4)
    try:
        assert lib.csm_tune(b"tc_spins", 0) == 0
        with pytest.raises(csmom.CsmError) as ei:
            engine.signal_chunked(P, ms, maxd, 12, 1, chunks=4, workspace=ws)
        assert ei.value.status == CSM_E_TIMEOUT
        assert not engine.signal_chunked_timed_out(ws)   # reported once, then cleared
        engine.signal_chunked(P, ms, maxd, 12, 1, chunks=4, workspace=ws, check=False)
        assert engine.signal_chunked_timed_out(ws)       # unchecked: the mark stays
        with pytest.raises(csmom.CsmError) as ei:
            engine.signal_chunked_status(ws)
        assert ei.value.status == CSM_E_TIMEOUT
    finally:
        assert lib.csm_tune(b"tc_spins", 1 << 21) == 0
    _, M, NR, I, ws = engine.signal_chunked(P, ms, maxd, 12, 1, chunks=4, workspace=ws)
    assert bits_equal(M.cpu().numpy(), M0.cpu().numpy())
    assert bits_equal(NR.cpu().numpy(), NR0.cpu().numpy())
    assert torch.equal(I, I0)
