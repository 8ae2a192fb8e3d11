"""The CPU oracle against the reference's own outputs (golden fixtures, tests/golden/)."""
import hashlib

import numpy as np
import pytest

from conftest import bits_equal, golden_tags, load_golden, parse_tag
from oracle import csmom_oracle as O


def _key(z, k, tags):
    return k if k in z.files else f"{tags[0]}_{k}"


@pytest.mark.parametrize("name", ["real_data", "edge", "small", "longwin"])
def test_oracle_matches_reference(name):
    z = load_golden(name)
    tags = golden_tags(z)
    PM, VOL = O.month_end(z["P"], z["month_start"], z["V"])
    assert bits_equal(PM, z[_key(z, "PM", tags)])
    assert (O.is_absent(PM) == (z[_key(z, "present", tags)] == 0)).all()
    assert bits_equal(VOL, z[_key(z, "VOL", tags)])
    for tag in tags:
        J, s = parse_tag(tag)
        R, M, NR, _ = O.momentum_scan(PM, J, s)
        assert bits_equal(R, z[_key(z, "R", tags)])
        assert bits_equal(M, z[f"{tag}_M"]), tag
        assert bits_equal(NR, z[f"{tag}_NR"]), tag
        L = O.assign_deciles(M, 10)
        assert np.array_equal(L, z[f"{tag}_L"]), tag
        EW, CNT, LS = O.portfolio_ew(L, NR, 10)
        assert bits_equal(EW, z[f"{tag}_EW"]), tag      # Kahan in row order: bit-exact
        assert bits_equal(LS, z[f"{tag}_LS"]), tag
        ls = LS[~np.isnan(LS)]
        assert ls.mean() == float(z[f"{tag}_mean"])
        assert O.sharpe(ls, 12) == float(z[f"{tag}_sharpe"])
        assert bits_equal(np.cumprod(1 + ls), z[f"{tag}_cum"])


def test_real_data_published_numbers():
    """70 months, mean 0.003673964721965685, Sharpe 0.10024098273478031, the
    cumulative curve of results/monthly_mom_cum.png."""
    z = load_golden("real_data")
    PM, _ = O.month_end(z["P"], z["month_start"])
    _, M, NR, _ = O.momentum_scan(PM, 12, 1)
    _, _, LS = O.portfolio_ew(O.assign_deciles(M, 10), NR, 10)
    ls = LS[~np.isnan(LS)]
    cum = np.cumprod(1 + ls)
    assert len(ls) == 70
    assert ls.mean() == 0.003673964721965685
    assert O.sharpe(ls, 12) == 0.10024098273478031
    assert (cum[0], cum.min(), cum.max(), cum[-1]) == (
        0.9701043580579196, 0.38005408951460795, 1.176025718881455, 0.7508682494556713)
    assert "0.003673964721965685" in str(z["printed"])


def test_c1_digests():
    z = load_golden("c1")
    dig = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    PM, _ = O.month_end(z["P"], z["month_start"])
    assert dig(PM) == str(z["PM_sha256"])
    for tag in golden_tags(z):
        J, s = parse_tag(tag)
        R, M, NR, _ = O.momentum_scan(PM, J, s)
        assert dig(R) == str(z["R_sha256"])
        assert dig(M) == str(z[f"{tag}_M_sha256"])
        assert dig(NR) == str(z[f"{tag}_NR_sha256"])
        L = O.assign_deciles(M, 10)
        assert np.array_equal(L, z[f"{tag}_L"])
        EW, _, LS = O.portfolio_ew(L, NR, 10)
        assert bits_equal(EW, z[f"{tag}_EW"])
        assert bits_equal(LS, z[f"{tag}_LS"])


def test_decile_cross_sections():
    d = load_golden("deciles")
    v, o, lab = d["values"], d["offsets"], d["labels"]
    for i in range(len(o) - 1):
        x, ref = v[o[i]:o[i + 1]], lab[o[i]:o[i + 1]]
        ok = ~np.isnan(x)
        out = np.full(len(x), np.nan)
        if ok.any():
            out[ok] = O.qcut_labels(x[ok])
        assert np.array_equal(out, ref, equal_nan=True), i


def test_quantile_table_constants():
    q = O.quantile_table(10)
    assert [float(x).hex() for x in q] == [
        "0x0.0p+0", "0x1.999999999999ap-4", "0x1.999999999999ap-3", "0x1.3333333333334p-2",
        "0x1.999999999999ap-2", "0x1.0000000000000p-1", "0x1.3333333333334p-1",
        "0x1.6666666666666p-1", "0x1.999999999999ap-1", "0x1.ccccccccccccdp-1",
        "0x1.0000000000000p+0"]
