"""CPU: the sweep's per-J chunked scans and streaming narrow decile pass are never captured into a
hipGraph (the round-3 replay fault came from a capture of exactly that joined C3
step, and its cause was never named).  A joined step that would take them while the current
stream is capturing raises before it launches anything; eagerly the same step runs."""
import pytest
import torch

import csmom
from csmom import sweep as sweep_mod


class _Stages:
    """Engine-shaped stub: records which scan / decile entry points a joined step reaches."""

    def __init__(self):
        self.calls = []

    def summary(self, *a, **k):        # marks the device path (joined batches need it)
        raise AssertionError("not reached")

    def momentum(self, PM, J=12, skip=1, **kw):
        self.calls.append(("momentum", J))
        T_m, N = PM.shape
        return None, torch.zeros(T_m, N, dtype=torch.float64), torch.zeros(T_m, N, dtype=torch.float64)

    def deciles(self, M, NR=None, n_bins=10, **kw):
        self.calls.append(("deciles", M.shape[0]))
        return torch.zeros(M.shape, dtype=torch.int8), None, None, None


@pytest.fixture
def capturing(monkeypatch):
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: True)


def _joined_ranked(st, **cfg):
    c = csmom.SweepConfig(Js=(3, 6), Ks=(3,), **cfg)
    r = csmom.SweepRunner(st, c)
    PM = torch.ones(40, 8, dtype=torch.float64)
    assert r._joined(40, 1, 8)
    return list(r._ranked(PM, 1))


def test_joined_per_j_path_refused_under_capture(capturing):
    st = _Stages()
    with pytest.raises(RuntimeError, match="hipGraph"):
        _joined_ranked(st, multi_j_scan=False)
    assert st.calls == []          # refused before any launch


def test_joined_per_j_path_runs_eagerly():
    st = _Stages()
    out = _joined_ranked(st, multi_j_scan=False)
    assert [J for J, _, _ in out] == [3, 6]
    assert st.calls == [("momentum", 3), ("momentum", 6), ("deciles", 80)]


def test_refuse_capture_is_silent_without_capture(monkeypatch):
    monkeypatch.setattr(torch.cuda, "is_available", lambda: False)
    sweep_mod._refuse_capture("x")          # no GPU: nothing to refuse
