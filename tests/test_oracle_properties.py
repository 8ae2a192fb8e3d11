"""Oracle restatement vs the third-party algorithms it restates (pandas qcut, NumPy
percentile / prod), on random inputs -- pins the oracle beyond the fixtures."""
import numpy as np
import pandas as pd
from hypothesis import given, settings, strategies as st

from conftest import bits_equal, load_golden
from oracle import csmom_oracle as O

floats = st.one_of(
    st.floats(-5, 5, allow_nan=False, width=64),
    st.sampled_from([0.0, 0.1, -0.1, 1.0, 0.25]),
)


@settings(max_examples=400, deadline=None)
@given(st.lists(floats, min_size=1, max_size=80), st.sampled_from([2, 3, 4, 5, 10, 20]))
def test_qcut_labels_match_pandas(xs, n_bins):
    x = np.array(xs, dtype=np.float64)
    ref = pd.qcut(pd.Series(x), q=n_bins, labels=False, duplicates="drop").to_numpy(np.float64)
    assert np.array_equal(O.qcut_labels(x, n_bins), ref, equal_nan=True)


@settings(max_examples=200, deadline=None)
@given(st.lists(st.floats(-1e3, 1e3, allow_nan=False, width=64), min_size=1, max_size=50))
def test_qcut_edges_match_numpy_percentile(xs):
    x = np.sort(np.array(xs))
    qt = O.quantile_table(10)
    ref = np.percentile(x, qt * 100.0)  # what pandas calls (quantile_with_mask)
    assert bits_equal(O.qcut_edges(x, qt), ref)


@settings(max_examples=200, deadline=None)
@given(st.lists(st.floats(-0.5, 0.5, allow_nan=False, width=64), min_size=1, max_size=64))
def test_sequential_product_equals_numpy_prod(rs):
    r = np.array(rs)
    acc = 1.0 + r[0]
    for v in r[1:]:
        acc = acc * (1.0 + v)
    assert (acc - 1.0) == (np.prod(1 + r) - 1)


def test_shard_decomposition_exact():
    z = load_golden("edge")
    PM, _ = O.month_end(z["P"], z["month_start"])
    for J, s in [(12, 1), (3, 0), (9, 2), (1, 0)]:
        R, M, NR, _ = O.momentum_scan(PM, J, s)
        for G in (2, 3, 4, 7, 16):
            parts = O.month_ranges(PM.shape[0], G)
            sums = np.stack([O.shard_summary(PM[a:b], J, s) for a, b in parts])
            outs = []
            for g, (a, b) in enumerate(parts):
                stt, npm = O.fold_carry(sums, g, J, s)
                outs.append(O.momentum_scan(PM[a:b], J, s, state=stt, next_pm=npm))
            assert bits_equal(np.concatenate([o[0] for o in outs]), R)
            assert bits_equal(np.concatenate([o[1] for o in outs]), M)
            assert bits_equal(np.concatenate([o[2] for o in outs]), NR)


def test_empty_and_degenerate_cross_sections():
    assert O.qcut_labels(np.array([])).shape == (0,)
    assert np.isnan(O.qcut_labels(np.array([0.3]))).all()
    assert np.isnan(O.qcut_labels(np.full(17, 2.0))).all()
    assert list(O.qcut_labels(np.array([1.0, 2.0, 3.0]))) == [0.0, 4.0, 9.0]
