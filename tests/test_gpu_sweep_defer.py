"""GPU: sweep steps without a device sync inside -- SweepRunner.run_batch(defer=True) leaves the
legs flag on the device (bench C3 queues steps back to back), and the bootstrap runner reads
every batch's flags once after the last batch; both give the synchronous tables bit for bit."""
import pytest
import torch

from conftest import bits_equal

pytestmark = pytest.mark.gpu


def _panel(engine, N=1000, T_d=2600, seed=21):
    from csmom.synth import bday_calendar, make_device_panel
    days, ms_h, _ = bday_calendar("2000-01-03", T_d)
    pan = make_device_panel(N, days, ms_h, seed=seed, device="cuda:0")
    PM, _ = engine.month_end(pan.P, pan.month_start)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(seed)
    shares = torch.exp(torch.randn(N, generator=g, device="cuda:0", dtype=torch.float64) + 16.0)
    return PM, shares


@pytest.mark.parametrize("legs", [True, False])
def test_run_batch_deferred_equals_sync(engine, legs):
    """run_batch(defer=True) (bench C3's step: no device sync, the legs flag left on the
    device) gives the synchronous call's table bit for bit, steps queued back to back."""
    import csmom
    PM, shares = _panel(engine)
    cfg = csmom.SweepConfig(Js=(3, 6, 9, 12), Ks=(3, 6, 9, 12), skip=1, aum=1e8, legs_only=legs)
    runner = csmom.SweepRunner(engine, cfg)
    W = PM.abs() * shares
    ADV = W * 0.01
    ref, _ = runner.run_batch(PM, 1, W=W, ADV=ADV)
    acc = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    outs = []
    for _ in range(3):
        summ, _, fl = runner.run_batch(PM, 1, W=W, ADV=ADV, defer=True)
        if fl is not None:
            acc.add_(fl)
        outs.append(summ)
    torch.cuda.synchronize()
    assert int(acc.item()) == 0
    for o in outs:
        assert bits_equal(o.cpu().numpy(), ref.cpu().numpy())


def test_bootstrap_deferred_flags_equal_sync(engine):
    """run_bootstrap reads every batch's flags once after the last batch; the table equals
    run_boot_batch per batch (synchronous) bit for bit."""
    import csmom
    from csmom.sweep import JOIN_ROWS
    PM, _ = _panel(engine, N=800, seed=22)
    R, _, _ = engine.momentum(PM, 12, 1, with_ret=True)
    R = R.contiguous()
    batch = JOIN_ROWS // R.shape[0] + 1
    runner = csmom.SweepRunner(engine, csmom.SweepConfig(Js=(3, 6, 9, 12), Ks=(3, 6, 9, 12),
                                                         skip=1))
    a = runner.run_bootstrap(R, 2 * batch + 3, seed=5000, mean_block=6.0, batch=batch)
    parts = [runner.run_boot_batch(R, min(batch, 2 * batch + 3 - b0), b0, 5000, 6.0)[0]
             for b0 in range(0, 2 * batch + 3, batch)]
    assert bits_equal(a.cpu().numpy(), torch.cat(parts, 0).cpu().numpy())
