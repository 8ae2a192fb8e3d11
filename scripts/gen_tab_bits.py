"""Bit-identity check of the general turnover rows' age tables (TO_GEN_TAB) against the full
walk: the same legs-only equal-weight accounting with the in-tree library and with a build of
-DTO_GEN_TAB=0 (CSMOM_LIB), printing a sha256 of LS / TURN / COST / NET per K.  Panels with
ramp-up months and an all-NaN month (general rows), K sets around the table width (8)."""
import hashlib
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import csmom  # noqa: E402


def main():
    eng = csmom.Engine(0)
    rng = np.random.default_rng(7)
    T_m, B, N = 120, 16, 4000
    L = rng.integers(-1, 10, size=(T_m, B, N)).astype(np.int8)
    L[30, 3, :] = -1                       # an empty month: K rows after it are general
    L[:5, 5, :] = -1                       # a late start
    NR = rng.normal(0.01, 0.08, size=(T_m, B, N))
    Ld = torch.from_numpy(L.reshape(T_m, B * N)).to("cuda:0")
    NRd = torch.from_numpy(NR.reshape(T_m, B * N)).to("cuda:0")
    h = hashlib.sha256()
    for Ks in ((3, 6, 9, 12), (1, 8, 9), (2, 5, 7, 16), (12, 3)):
        out = eng.portfolio_multi(Ld, NRd, 10, Ks=Ks, B=B, legs_only=True)
        for K in Ks:
            for f in ("LS", "TURN", "COST", "NET"):
                h.update(getattr(out[K], f).cpu().numpy().tobytes())
    print(h.hexdigest())


if __name__ == "__main__":
    main()
