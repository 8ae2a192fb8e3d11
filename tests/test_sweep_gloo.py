"""Sweep sharding on CPU: SweepRunner (the orchestration the GPU ranks run over RCCL) driven with
gloo at world_size 2 and 3 with oracle-backed stages.  Bootstrap panels are keyed by their
global id, so the sharded summary table equals the single-process one (series bit for bit; the
summary reductions to rounding, since they run over differently shaped batches)."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, str(Path(__file__).resolve().parent))
from oracle import csmom_oracle as O  # noqa: E402
from oracle import portfolio_oracle as PO  # noqa: E402


class _PF:
    def __init__(self, **kw):
        self.__dict__.update(kw)


class OracleSweepStages:
    """Engine-shaped sweep stages over the CPU oracles (test-only)."""

    def momentum(self, PM, J=12, skip=1, **kw):
        R, M, NR, _ = O.momentum_scan(PM.numpy(), J, skip)
        return torch.from_numpy(R), torch.from_numpy(M), torch.from_numpy(NR)

    def deciles(self, M, NR=None, n_bins=10, **kw):
        return torch.from_numpy(O.assign_deciles(M.numpy(), n_bins)), None, None, None

    def portfolio(self, L, NR, n_bins=10, K=1, W=None, B=1, with_costs=True, **kw):
        T_m, BN = L.shape
        N = BN // B
        r = PO.portfolio(L.numpy().reshape(T_m, B, N), NR.numpy().reshape(T_m, B, N), n_bins,
                         K=K, W=None if W is None else W.numpy().reshape(T_m, B, N),
                         half_spread=kw.get("half_spread", PO.HALF_SPREAD))
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x))
        return _PF(PR=t(r["PR"]), LS=t(r["LS"]), TURN=t(r["TURN"]) if with_costs else None,
                   COST=t(r["COST"]) if with_costs else None,
                   NET=t(r["NET"]) if with_costs else None)

    def bootstrap(self, R, B, b0=0, seed=5000, mean_block=6.0, **kw):
        T_m, N = R.shape
        src = PO.bootstrap_indices(T_m, B, seed, mean_block, b0=b0)
        pm = PO.bootstrap_panel(R.numpy(), src)
        return torch.from_numpy(src.astype(np.int32)), torch.from_numpy(pm.reshape(T_m, B * N))


def _base_returns():
    from conftest import load_golden
    z = load_golden("edge")
    PM, _ = O.month_end(z["P"], z["month_start"].astype(np.int64))
    R, _, _, _ = O.momentum_scan(PM, 12, 1)
    return torch.from_numpy(R)


def _cfg():
    import csmom
    return csmom.SweepConfig(Js=(3, 6), Ks=(1, 3), skip=1)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_panels, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import csmom
        runner = csmom.SweepRunner(OracleSweepStages(), _cfg())
        tab = runner.run_bootstrap(_base_returns(), n_panels, seed=5000, mean_block=4.0, batch=2)
        q.put((rank, tab.numpy()))
    finally:
        dist.destroy_process_group()


def test_single_process_sweep_matches_per_panel():
    import csmom
    runner = csmom.SweepRunner(OracleSweepStages(), _cfg())
    R = _base_returns()
    tab = runner.run_bootstrap(R, 5, seed=5000, mean_block=4.0, batch=3).numpy()
    assert tab.shape == (5, 4, len(csmom.SUMMARY_FIELDS))
    # panel 3 alone, through the oracle directly
    T_m, N = R.shape
    pm = PO.bootstrap_panel(R.numpy(), PO.bootstrap_indices(T_m, 1, 5000, 4.0, b0=3))[:, 0, :]
    for s, (J, K) in enumerate(_cfg().strategies):
        _, M, NR, _ = O.momentum_scan(pm, J, 1)
        L = O.assign_deciles(M, 10)
        r = PO.portfolio(L, NR, 10, K=K)
        ls = r["LS"][:, 0]
        ls = ls[~np.isnan(ls)]
        assert tab[3, s, 0] == len(ls)
        assert abs(tab[3, s, 1] - ls.mean()) <= 1e-12 * max(1e-12, abs(ls.mean()))
        assert abs(tab[3, s, 2] - O.sharpe(ls, 12)) <= 1e-9 * abs(O.sharpe(ls, 12))


@pytest.mark.parametrize("world", [2, 3])
def test_sweep_shards_gloo(world):
    import csmom
    n_panels = 5
    ref = csmom.SweepRunner(OracleSweepStages(), _cfg()).run_bootstrap(
        _base_returns(), n_panels, seed=5000, mean_block=4.0, batch=2).numpy()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_panels, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, tab in res:  # every rank holds the whole table, equal to the 1-process run
        assert tab.shape == ref.shape
        assert np.array_equal(np.isnan(tab), np.isnan(ref))
        assert np.array_equal(tab[..., 0], ref[..., 0])          # months: exact
        m = ~np.isnan(ref)
        # summary reductions run over differently shaped batches: equal to rounding
        assert np.allclose(tab[m], ref[m], rtol=1e-12, atol=1e-15)


# ------------------------------------------------------------------------------------------------
# (J, K)-grid sharding (SweepRunner.run_batch_sharded, bench C3 at N > 1): every rank holds the
# month panel and runs its contiguous block of the strategy grid; one all-gather of the summary
# blocks.  Oracle stages: the table equals the 1-process run_batch bit for bit.
def _panel_pm():
    from conftest import load_golden
    z = load_golden("edge")
    PM, _ = O.month_end(z["P"], z["month_start"].astype(np.int64))
    return torch.from_numpy(PM)


def _grid_cfg():
    import csmom
    return csmom.SweepConfig(Js=(3, 6, 12), Ks=(1, 3), skip=1)


def _grid_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import csmom
        runner = csmom.SweepRunner(OracleSweepStages(), _grid_cfg())
        tab, series = runner.run_batch_sharded(_panel_pm(), 1)
        q.put((rank, tab.numpy(), sorted(series)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_strategy_shards_gloo(world):
    import csmom
    from csmom.sweep import panel_partition
    ref, _ = csmom.SweepRunner(OracleSweepStages(), _grid_cfg()).run_batch(_panel_pm(), 1)
    ref = ref.numpy()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grid_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    strategies = _grid_cfg().strategies
    for rank, tab, keys in res:   # every rank: the whole table, bit for bit the 1-process one
        assert tab.shape == ref.shape == (1, len(strategies), len(csmom.SUMMARY_FIELDS))
        assert np.array_equal(np.isnan(tab), np.isnan(ref))
        m = ~np.isnan(ref)
        assert np.array_equal(tab[m], ref[m])
        a, b = panel_partition(len(strategies), world)[rank]
        assert keys == sorted(strategies[a:b])                  # its own strategies' series


def test_strategy_shards_single_process_is_run_batch():
    import csmom
    runner = csmom.SweepRunner(OracleSweepStages(), _grid_cfg())
    a, _ = runner.run_batch_sharded(_panel_pm(), 1)
    b, _ = runner.run_batch(_panel_pm(), 1)
    assert np.array_equal(np.isnan(a.numpy()), np.isnan(b.numpy()))
    m = ~np.isnan(b.numpy())
    assert np.array_equal(a.numpy()[m], b.numpy()[m])


def test_stacked_view_or_copy():
    """sweep._stacked: tensors lying back to back in one allocation come back as a view of it
    (the joined sweep's group-major panels, no copy); any other list is stacked into a copy."""
    from csmom.sweep import _stacked
    base = torch.arange(24, dtype=torch.float64).reshape(3, 2, 4)
    v = _stacked(list(base))
    assert v.data_ptr() == base.data_ptr() and torch.equal(v, base)
    parts = [torch.full((2, 4), float(i)) for i in range(3)]
    c = _stacked(parts)
    assert c.shape == (3, 2, 4) and all(torch.equal(c[i], parts[i]) for i in range(3))
    out_of_order = _stacked([base[1], base[0]])
    assert torch.equal(out_of_order, torch.stack([base[1], base[0]]))
    assert out_of_order.data_ptr() != base.data_ptr()
    flat = base.view(6, 4)   # slices of one stacked [rows][N] pass, reshaped
    assert _stacked([flat[0:2], flat[2:4], flat[4:6]]).data_ptr() == base.data_ptr()
