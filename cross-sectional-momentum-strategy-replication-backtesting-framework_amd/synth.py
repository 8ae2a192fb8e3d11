"""Seeded synthetic daily panels generated directly in HBM (bench inputs; 8 GB at C4).

Same conventions as SURVEY.md 8(d): log-returns N(mu_a, sigma_a), mu_a ~ N(3e-4, 2e-4),
sigma_a ~ U(0.01, 0.04), P0 = 100, business-day calendar; masking mix of 5 % late
listings, 5 % early delistings, 1 % NaN days, 0.2 % absent (asset, month) rows and 0.1 %
all-NaN months.  Data generation is plumbing (torch ops), never part of a timed pass.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import pandas as pd
import torch

from ._lib import ABSENT_BITS
from .panel import month_offsets

NAN_BITS = 0x7FF8000000000000


@dataclass
class DevicePanel:
    P: torch.Tensor              # [T_d][N] float64 in HBM
    month_start: torch.Tensor    # [T_m+1] int64 in HBM
    month_start_host: np.ndarray
    days: pd.DatetimeIndex       # (datetime64[D] arrays past pandas' Timestamp range)
    month_end: pd.DatetimeIndex

    @property
    def shape(self):
        return tuple(self.P.shape)


def bday_calendar(start: str, periods: int):
    """pd.bdate_range(start, periods=periods) (Mon-Fri, start rolled forward) with its calendar
    month offsets and 'ME' labels, computed on numpy datetime64[D] so that long weak-scaling
    calendars (8 x 10,000 bdays from 1985 end in 2291) do not overflow pandas' nanosecond
    Timestamps.  Days / labels come back as pd.DatetimeIndex when they fit, else as
    datetime64[D] arrays."""
    d0 = np.busday_offset(np.datetime64(start, "D"), 0, roll="forward")
    days = np.busday_offset(d0, np.arange(periods, dtype=np.int64), roll="forward")
    mkey = days.astype("datetime64[M]")
    change = np.nonzero(mkey[1:] != mkey[:-1])[0] + 1
    ms = np.concatenate([[0], change, [periods]]).astype(np.int64) if periods else \
        np.zeros(1, dtype=np.int64)
    mend = (mkey[ms[:-1]] + 1).astype("datetime64[D]") - np.timedelta64(1, "D")
    if periods == 0 or mend[-1] < np.datetime64("2262-04-01"):
        return (pd.DatetimeIndex(days.astype("datetime64[ns]")), ms,
                pd.DatetimeIndex(mend.astype("datetime64[ns]")))
    return days, ms, mend


def shard_calendar(start: str, periods_total: int, G: int, rank: int):
    """Whole-month date shard `rank` of a G-way split of bdate_range(start, periods_total)."""
    days, ms, mend = bday_calendar(start, periods_total)
    T_m = len(ms) - 1
    base, rem = divmod(T_m, G)
    m0 = rank * base + min(rank, rem)
    m1 = m0 + base + (1 if rank < rem else 0)
    d0, d1 = ms[m0], ms[m1]
    months = [base + (1 if g < rem else 0) for g in range(G)]
    return days[d0:d1], (ms[m0:m1 + 1] - d0).astype(np.int64), mend[m0:m1], months


def make_device_panel(N: int, days: pd.DatetimeIndex, month_start: np.ndarray, seed: int,
                      device, late=0.05, delist=0.05, nan_day=0.01, absent_month=0.002,
                      nan_month=0.001, block_days: int = 512, shard=None) -> DevicePanel:
    """Seeded GBM panel built in HBM.  shard=(rank, world, base_seed, days_per_shard): this
    panel is date shard `rank` of ONE global panel -- per-asset drift / volatility and the
    log-price at every shard boundary come from base_seed (identical on every rank), and the
    shard's path is a Brownian bridge between its two boundary levels, so prices continue
    across shards (independent per-rank panels would jump by e^(sigma*sqrt(T)) at each
    boundary: heavy-tailed momentum for a year after it)."""
    device = torch.device(device)
    T_d = len(days)
    T_m = len(month_start) - 1
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    f64 = dict(dtype=torch.float64, device=device)
    if shard is None:
        mu = torch.randn(N, generator=g, **f64) * 2e-4 + 3e-4
        sig = torch.rand(N, generator=g, **f64) * 0.03 + 0.01
        lvl0, lvl1 = None, None
    else:
        rank, world, base_seed, dps = shard
        gg = torch.Generator(device=device)
        gg.manual_seed(int(base_seed) * 7919 + 17)
        mu = torch.randn(N, generator=gg, **f64) * 2e-4 + 3e-4
        sig = torch.rand(N, generator=gg, **f64) * 0.03 + 0.01
        z = torch.randn(world, N, generator=gg, **f64)
        steps = mu * dps + sig * float(np.sqrt(dps)) * z               # [world][N]
        anchors = torch.cat([torch.zeros(1, N, **f64), torch.cumsum(steps, 0)], 0)
        lvl0, lvl1 = anchors[rank], anchors[rank + 1]
        # the bridge needs the shard's own walk total first: one extra pass of its stream
        gn = torch.Generator(device=device)
        gn.manual_seed(int(seed) * 104729 + 3)
        tot = torch.zeros(N, **f64)
        for d0 in range(0, T_d, block_days):
            d1 = min(T_d, d0 + block_days)
            tot += (torch.randn(d1 - d0, N, generator=gn, **f64) * sig + mu).sum(0)
        gn.manual_seed(int(seed) * 104729 + 3)
        slope = ((lvl1 - lvl0) - tot) / max(T_d, 1)
    if shard is None:
        list_day = torch.where(torch.rand(N, generator=g, **f64) < late,
                               torch.randint(1, max(2, T_d // 2), (N,), generator=g, device=device),
                               torch.zeros(N, dtype=torch.int64, device=device))
        delist_day = torch.where(torch.rand(N, generator=g, **f64) < delist,
                                 torch.randint(max(1, T_d // 2), max(2, T_d), (N,), generator=g,
                                               device=device),
                                 torch.full((N,), T_d, dtype=torch.int64, device=device))
    else:
        # listings and delistings belong to the global panel (an asset delisted in shard r
        # stays delisted in shard r+1), drawn on the global day axis and shifted to this shard
        Dg = int(round(dps * world))
        day0 = int(round(dps * rank))
        lg = torch.where(torch.rand(N, generator=gg, **f64) < late,
                         torch.randint(1, max(2, Dg // 2), (N,), generator=gg, device=device),
                         torch.zeros(N, dtype=torch.int64, device=device))
        dg = torch.where(torch.rand(N, generator=gg, **f64) < delist,
                         torch.randint(max(1, Dg // 2), max(2, Dg), (N,), generator=gg,
                                       device=device),
                         torch.full((N,), Dg, dtype=torch.int64, device=device))
        list_day = lg - day0
        delist_day = torch.where(dg >= Dg, torch.full_like(dg, T_d), dg - day0)
    am = torch.rand(T_m, N, generator=g, **f64) < absent_month      # absent (month, asset)
    nm = torch.rand(T_m, N, generator=g, **f64) < nan_month         # all-NaN (month, asset)
    day_month = torch.from_numpy(
        np.repeat(np.arange(T_m), np.diff(month_start)).astype(np.int64)).to(device)
    P = torch.empty(T_d, N, **f64)
    run = torch.zeros(N, **f64)
    absent = torch.tensor(ABSENT_BITS, dtype=torch.int64, device=device)
    qnan = torch.tensor(NAN_BITS, dtype=torch.int64, device=device)
    for d0 in range(0, T_d, block_days):
        d1 = min(T_d, d0 + block_days)
        if lvl0 is None:
            lr = torch.randn(d1 - d0, N, generator=g, **f64) * sig + mu
        else:
            lr = torch.randn(d1 - d0, N, generator=gn, **f64) * sig + mu + slope
        c = torch.cumsum(lr, 0) + run
        run = c[-1].clone()
        if lvl0 is not None:
            c = c + lvl0
        blk = (100.0 * torch.exp(c)).view(torch.int64)
        dd = torch.arange(d0, d1, device=device)[:, None]
        dm = day_month[d0:d1]
        gone = (dd < list_day[None, :]) | (dd >= delist_day[None, :]) | am[dm]
        nanc = (torch.rand(d1 - d0, N, generator=g, **f64) < nan_day) | nm[dm]
        blk = torch.where(nanc, qnan, blk)
        blk = torch.where(gone, absent, blk)
        P[d0:d1] = blk.view(torch.float64)
        del lr, c, blk, gone, nanc
    ms_dev = torch.from_numpy(np.ascontiguousarray(month_start, dtype=np.int64)).to(device)
    dd = np.asarray(days).astype("datetime64[D]")
    mend = ((dd[np.asarray(month_start[:-1])].astype("datetime64[M]") + 1).astype("datetime64[D]")
            - np.timedelta64(1, "D")) if T_m else dd[:0]
    if T_m == 0 or mend[-1] < np.datetime64("2262-04-01"):
        mend = pd.DatetimeIndex(mend.astype("datetime64[ns]"))
    return DevicePanel(P=P, month_start=ms_dev, month_start_host=np.asarray(month_start),
                       days=days, month_end=mend)


@dataclass
class HaloPanel:
    """Rank `rank`'s rows of a whole-month date split with its lookback halo: P holds the last
    H months of the previous shard, this shard, and the first F months of the next
    (DateShardPipeline.run_halo's input); month_start [H + T_m + F + 1] are day offsets into P."""
    P: torch.Tensor
    month_start: torch.Tensor
    month_start_host: np.ndarray
    H: int
    F: int
    T_m: int                     # this shard's months
    shard_days: int              # this shard's business days (its share of the panel)

    @property
    def shard_month_start(self):
        return self.month_start[self.H:self.H + self.T_m + 1]


def make_halo_panel(N: int, start: str, periods_total: int, world: int, rank: int, H: int,
                    seed_of, base_seed: int, device, days_per_shard: float | None = None,
                    F: int = 3, **kw) -> HaloPanel:
    """Shard `rank` of one global panel (make_device_panel(shard=...), rank r seeded with
    seed_of(r)) with H months of the previous shard and the next shard's first F months: the
    neighbours' panels are generated with their own seeds and sliced, so the halo rows are
    exactly the rows those ranks hold."""
    dps = periods_total / world if days_per_shard is None else days_per_shard

    def shard(r):
        days, ms, _, months = shard_calendar(start, periods_total, world, r)
        return make_device_panel(N, days, ms, seed=seed_of(r), device=device,
                                 shard=(r, world, base_seed, dps), **kw), ms
    me, ms_me = shard(rank)
    parts, mss = [], []
    h = 0
    if rank > 0 and H > 0:
        prev, ms_p = shard(rank - 1)
        h = min(H, len(ms_p) - 1)
        d0 = int(ms_p[len(ms_p) - 1 - h])
        parts.append(prev.P[d0:])
        mss.append(ms_p[len(ms_p) - 1 - h:-1] - d0)
        del prev
    off = sum(int(p.shape[0]) for p in parts)
    parts.append(me.P)
    mss.append(ms_me[:-1] + off)
    off += int(me.P.shape[0])
    f = 0
    if rank < world - 1 and F > 0:
        nxt, ms_n = shard(rank + 1)
        f = min(F, len(ms_n) - 1)
        parts.append(nxt.P[:int(ms_n[f])])
        mss.append(ms_n[:f] + off)
        off += int(ms_n[f])
        del nxt
    F = f
    ms_ext = np.concatenate(mss + [np.array([off], dtype=np.int64)]).astype(np.int64)
    P = torch.cat(parts, 0).contiguous() if len(parts) > 1 else me.P
    del parts, me
    return HaloPanel(P=P, month_start=torch.from_numpy(ms_ext).to(torch.device(device)),
                     month_start_host=ms_ext, H=h, F=F, T_m=len(ms_me) - 1,
                     shard_days=int(ms_me[-1]))
