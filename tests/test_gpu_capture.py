"""GPU: the C3 sweep step (SweepRunner.run_batch(defer=True), run_demo.py:41-67 per (J, K)) as
a captured hipGraph.

Round 3 captured this step, replayed it once successfully, and then faulted the GPU (illegal
address) in the timed replays of the full 5,000-asset workload.  The turnover launches keep a
work list of general rows in the portfolio workspace: the steady launch appends to it through a
device counter and the general launch walks it.  The counter was reset by hipMemsetAsync before
each steady launch.  If a replay does not reset it, every replay appends behind the previous
replay's entries and the list overruns its capacity (one slot per steady workgroup) after a few
replays -- while eager calls, the first replay and short replay tests stay correct, because
walking a row twice rewrites the same values.

The library now (a) resets the counter with a kernel node (k_zero_i32), (b) never appends past
the list's capacity nor walks past it, and (c) refuses to regrow its own buffers while the stream
is being captured.  test_gen_counter_under_capture records how each reset form behaves across
replays (the counter the general launch read, through csm_tune_ptr("gen_probe")); the full-size
test replays the bench's C3 step three times and checks each summary table bit for bit against
the eager step.
"""
import ctypes

import numpy as np
import pytest
import torch

from conftest import bits_equal

pytestmark = pytest.mark.gpu


def _c3_inputs(engine, N, T_d, seed):
    """bench.py's C3 step inputs: the seeded panel, lognormal shares and daily turnover rates."""
    from csmom.synth import bday_calendar, make_device_panel
    days, ms_h, _ = bday_calendar("2000-01-03", T_d)
    panel = make_device_panel(N, days, ms_h, seed=seed, device=engine.device)
    g = torch.Generator(device=engine.device)
    g.manual_seed(seed)
    shares = torch.exp(torch.randn(N, generator=g, device=engine.device, dtype=torch.float64) + 16.0)
    rate = torch.rand(N, generator=g, device=engine.device, dtype=torch.float64) * 0.018 + 0.002
    return panel, shares, rate


def _c3_step(engine, panel, shares, rate):
    import csmom
    T_m = panel.month_start.numel() - 1
    N = panel.P.shape[1]
    cfg = csmom.SweepConfig(Js=(3, 6, 9, 12), Ks=(3, 6, 9, 12), skip=1, aum=1e8)
    runner = csmom.SweepRunner(engine, cfg)
    PM = engine.empty((T_m, N))

    def step():
        engine.month_end(panel.P, panel.month_start, PM=PM)
        W = PM.abs() * shares
        ADV = W * rate
        summ, _, fl = runner.run_batch(PM, 1, W=W, ADV=ADV, defer=True)
        return summ, fl
    return step


def _capture(step):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):      # warm-up on a side stream, as torch's capture recipe asks
        step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = step()
    return graph, out


def _tune(engine, key, value):
    assert engine.lib.csm_tune(key.encode(), int(value)) == 0


def _probe(engine, t):
    assert engine.lib.csm_tune_ptr(b"gen_probe", ctypes.c_void_p(t.data_ptr() if t is not None
                                                                   else 0)) == 0


@pytest.mark.parametrize("reset", [1, 0])
def test_gen_counter_under_capture(engine, reset):
    """The work-list counter the general turnover launch reads, per graph replay, with the
    counter reset by a kernel (1, the default) or by hipMemsetAsync (0, round 3's form).  The
    kernel form must read the eager count on every replay; both forms must give the eager
    summary table bit for bit (the list is bounded, and walking a row twice rewrites the same
    values).  The memset form's counts are printed: they are the diagnosis DESIGN.md records."""
    panel, shares, rate = _c3_inputs(engine, 1000, 2600, 31)
    step = _c3_step(engine, panel, shares, rate)
    probe = torch.zeros(1, dtype=torch.int32, device=engine.device)
    _tune(engine, "gen_reset", reset)
    _probe(engine, probe)
    try:
        ref, _ = step()
        torch.cuda.synchronize()
        eager_n = int(probe.item())
        ref = ref.cpu().numpy()
        graph, (summ, _) = _capture(step)
        counts = []
        for _ in range(6):
            probe.zero_()
            graph.replay()
            torch.cuda.synchronize()
            counts.append(int(probe.item()))
            assert bits_equal(summ.cpu().numpy(), ref)
        print(f"[gen_reset={reset}] eager count {eager_n}, replay counts {counts}", flush=True)
        assert eager_n > 0
        if reset == 1:
            assert counts == [eager_n] * len(counts)
        del graph
    finally:
        _probe(engine, None)
        _tune(engine, "gen_reset", 1)
        torch.cuda.synchronize()


def test_c3_fullsize_graph_replay_bit_exact(engine):
    """bench.py's C3 workload (5,000 assets x 6,522 bdays, the 16-strategy VW grid with spread +
    sqrt-impact costs) captured as one hipGraph and replayed three times: each replay's summary
    table equals the eager step's bit for bit, and no replay raised the legs flag."""
    panel, shares, rate = _c3_inputs(engine, 5000, 6522, 4 * 1000 + 3)
    step = _c3_step(engine, panel, shares, rate)
    ref, fl = step()
    torch.cuda.synchronize()
    assert fl is None or int(fl.item()) == 0
    ref = ref.cpu().numpy()
    assert np.isfinite(ref[..., 1]).all()
    graph, (summ, flag) = _capture(step)
    for _ in range(3):
        graph.replay()
        torch.cuda.synchronize()
        assert bits_equal(summ.cpu().numpy(), ref)
        assert flag is None or int(flag.item()) == 0
    del graph
    torch.cuda.synchronize()


def test_c3_fullsize_back_to_back_replays(engine):
    """The bench's timed form: 20 replays queued back to back with no sync between them (round
    3's fault came in this loop, after one synced replay), then one sync: the summary table
    equals the eager step's and no legs flag was raised."""
    panel, shares, rate = _c3_inputs(engine, 5000, 6522, 4 * 1000 + 3)
    step = _c3_step(engine, panel, shares, rate)
    ref, _ = step()
    torch.cuda.synchronize()
    ref = ref.cpu().numpy()
    acc = torch.zeros(1, dtype=torch.int32, device=engine.device)

    def step_acc():
        summ, fl = step()
        if fl is not None:
            acc.add_(fl)
        return summ
    graph, summ = _capture(step_acc)
    graph.replay()
    torch.cuda.synchronize()
    acc.zero_()
    for _ in range(20):
        graph.replay()
    torch.cuda.synchronize()
    assert int(acc.item()) == 0
    assert bits_equal(summ.cpu().numpy(), ref)
    del graph
    torch.cuda.synchronize()
