"""(J, K) strategy sweeps and bootstrap panels (BASELINE configs C3 and C5).

The reference runs one strategy (J = 12, skip = 1, K = 1, equal weight) per call of
`monthly_replication` (run_demo.py:31-79).  A sweep runs a grid of strategies over one or many
panels with the month-end aggregation done once per panel:

  * per J: one scan of the month panel (ret_1m / mom_J / next_ret, features.py:44-52,
    run_demo.py:48) and one qcut pass (run_demo.py:18-29) -- all B panels of a batch at once,
    laid out side by side as [T_m][B*N] (the scan is per asset; the labels are per (month,
    panel) row of N assets);
  * per J: one cohort-sum pass for the largest K (cohort sums do not depend on K), then per
    (J, K) the K-overlap accounting (equal or value weights, turnover, spread +
    square-root-impact costs; rules E1..E5);
  * per (J, K, panel): a summary row (months, mean and Sharpe of the long-short as in
    src/utils.py:8-16 at 12 periods a year, mean turnover, mean cost, mean / Sharpe of net).

Multi-GPU: sweep units are independent.  Bootstrap panels are split across ranks in contiguous
ranges (a panel's bootstrap stream is keyed by its global id, never by the rank); a single
panel's (J, K) grid is split across ranks in contiguous strategy blocks (run_batch_sharded).
Either way the only collective is one all-gather of the summary table at the end.  The stage implementation is
injected (`Engine` on the GPU; the CPU tests drive the same orchestration with gloo and an
oracle-backed adapter).
"""
from __future__ import annotations

import dataclasses
from collections.abc import Mapping
import itertools
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from .distributed import all_gather_stack
from .engine import LEGS_MAX_N

JOIN_ROWS = 4096   # SweepConfig.join_js: batches below this many (month, panel) rows
SUMMARY_FIELDS = ("months", "mean", "sharpe", "turnover", "cost", "net_mean", "net_sharpe")


def _free_bytes(t: torch.Tensor) -> int:
    """Memory available to new tensors on t's device: free device memory plus what torch's
    caching allocator holds reserved but unused (a previous batch's freed panels), so the
    multi-J choice does not flip between batches.  Host tensors: unbounded."""
    if t.is_cuda:
        free, _ = torch.cuda.mem_get_info(t.device)
        cached = torch.cuda.memory_reserved(t.device) - torch.cuda.memory_allocated(t.device)
        return int(free + max(cached, 0))
    return 1 << 62


def _free_bytes_dev(stages) -> int:
    """_free_bytes of the stages' device (the Engine's), unbounded for host stages."""
    dev = getattr(stages, "device", None)
    if dev is None or getattr(dev, "type", "cpu") != "cuda":
        return 1 << 62
    return _free_bytes(torch.empty(0, device=dev))


def strategy_grid(Js=(3, 6, 9, 12), Ks=(3, 6, 9, 12)):
    return [(int(J), int(K)) for J in Js for K in Ks]


def panel_partition(n_panels: int, G: int):
    """Contiguous panel ranges per rank (earlier ranks take the remainder)."""
    base, rem = divmod(n_panels, G)
    out, p0 = [], 0
    for g in range(G):
        p1 = p0 + base + (1 if g < rem else 0)
        out.append((p0, p1))
        p0 = p1
    return out


def summarize(LS: torch.Tensor, TURN, COST, NET, freq: int = 12) -> torch.Tensor:
    """Per-panel summary rows [B][len(SUMMARY_FIELDS)] from [T_m][B] series; NaN months are
    dropped (run_demo.py:67) and the Sharpe ratio is src/utils.py:8-16's."""
    def stats(x):
        ok = ~torch.isnan(x)
        n = ok.sum(0).to(x.dtype)
        xs = torch.where(ok, x, torch.zeros_like(x))
        mean = xs.sum(0) / n
        dev = torch.where(ok, x - mean, torch.zeros_like(x))
        var = (dev * dev).sum(0) / (n - 1)
        sd = torch.sqrt(var)
        sh = torch.where(sd > 0, mean * freq / (sd * freq ** 0.5), torch.full_like(sd, float("nan")))
        return n, mean, sh
    n, mean, sh = stats(LS)
    ok = ~torch.isnan(LS)
    zero = torch.zeros_like(LS)
    if TURN is not None:
        turn = torch.where(ok, TURN, zero).sum(0) / n
        cost = torch.where(ok, COST, zero).sum(0) / n
        _, nmean, nsh = stats(NET)
    else:
        turn = cost = nmean = nsh = torch.full_like(mean, float("nan"))
    return torch.stack([n, mean, sh, turn, cost, nmean, nsh], dim=1)


@dataclass
class SweepConfig:
    Js: tuple = (3, 6, 9, 12)
    Ks: tuple = (3, 6, 9, 12)
    skip: int = 1
    n_bins: int = 10
    half_spread: float = 0.0005
    k_impact: float = 0.1
    aum: float = 0.0
    costs: bool = True
    multi_j_scan: bool = True
    # with the multi-J scan, also write each mom_J's fixed-map bucket ids and rank the batch's
    # rows from them (csm_momentum_multi_ids -> csm_deciles_ids): 2-B ids per cell instead of
    # up to three passes over mom_J; same labels
    decile_ids: bool = True
    # accounting of the two legs only (deciles 0 and n_bins - 1) on rows of <= 7168 assets: the
    # summary table (LS, TURN, COST, NET) is bit for bit the full path's; the per-strategy
    # series' PR then holds the legs (NaN elsewhere; PortfolioOut.legs_only says which form a
    # series has -- wider rows always get every decile).  False: every decile's overlapped
    # return
    legs_only: bool = True
    # with legs_only: the decile pass selects only the legs' edges (csm_deciles_ids_legs --
    # labels 0 / n_bins - 1 exact, the interior ones arbitrary in [1, n_bins - 2]); the same
    # summary table bit for bit
    legs_labels: bool = True
    # bootstrap sweeps (run_bootstrap): csm_boot_scan -- the panel generated in registers and
    # scanned for every J at once, one next_ret panel for every J -- instead of csm_bootstrap ->
    # multi-J scan (same labels and summary table, bit for bit)
    boot_scan: bool = True
    # batches of fewer than JOIN_ROWS (month, panel) rows (C3's single panel): the Js' decile
    # passes and accounting as one launch set over the Js side by side (_account_joined); the
    # same table and series bit for bit (taken only where the side-by-side batch has the chunk
    # plan of one J's batch, _joined; tests/test_gpu_fullsize.py::test_c3_joined_js_equal_per_j)
    join_js: bool = True
    # bootstrap batches: the Js' cohort sums in one pass over the shared next_ret
    # (csm_cohort_sums_js: each month's return row read once for every J; same table bit for bit)
    share_nr: bool = True
    # joined batches: the Js' labels / next_ret read group-major where the stacked scan and
    # decile pass wrote them and the weights / ADV / vol once for every J
    # (portfolio_multi_grouped); False: side-by-side copies (torch.cat / repeat) -- same bits
    grouped: bool = True
    # joined batches: month chunks of the time-chunked multi-J scan (0: Engine.default_chunks;
    # any count gives the same bits -- the fold chains through every earlier chunk)
    scan_chunks: int = 0
    extra: dict = field(default_factory=dict)

    @property
    def strategies(self):
        return strategy_grid(self.Js, self.Ks)


def _refuse_capture(what):
    """The round-3 hipGraph replay fault came from a capture of the joined C3
    step on the per-J chunked scans and the streaming narrow decile pass; its cause was never
    named.  Those launches stay available eagerly (configs outside the multi-J kernels' domain,
    A/B knobs) but are never captured: a joined step that would take them under stream capture
    is refused before it records anything."""
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        raise RuntimeError(f"SweepRunner: {what} are not captured into a hipGraph (DESIGN.md 4.3); "
                           "run this configuration eagerly")


def _legs_labels(c, legs, N):
    """Whether a batch's ids decile pass may label legs only (csm_deciles_ids_legs): the
    legs-only accounting follows (it reads deciles 0 and n_bins - 1 only; a rerun for a panel
    lacking a leg ranks every decile again) and takes rows this wide (LEGS_MAX_N)."""
    return bool(legs) and c.legs_labels and c.n_bins >= 4 and N <= LEGS_MAX_N


def _stacked(ts):
    """The equal-shape tensors `ts` as one [len(ts)][...] tensor: a view when they already lie
    back to back in one allocation (momentum_multi(stacked=True), slices of one stacked decile
    pass), else a stacked copy."""
    t0 = ts[0]
    n = t0.numel() * t0.element_size()
    if all(t.is_contiguous() and t.shape == t0.shape and t.dtype == t0.dtype
           and t.device == t0.device and t.untyped_storage().data_ptr() == t0.untyped_storage().data_ptr()
           and t.data_ptr() == t0.data_ptr() + i * n for i, t in enumerate(ts)):
        return t0.as_strided((len(ts),) + tuple(t0.shape), (t0.numel(),) + tuple(t0.stride()))
    return torch.stack(list(ts))


class _JoinedSeries(Mapping):
    """{(J, K): PortfolioOut} over a joined batch's outputs (panel q * B + b = J q's panel b),
    each entry built on access as strided views; a repeated J maps to its last position, as a
    dict filled in order would."""

    def __init__(self, outs, Js, B):
        self._outs, self._B = outs, B
        self._q = {J: q for q, J in enumerate(Js)}

    def __getitem__(self, key):
        J, K = key
        q, o = self._q[J], self._outs[K]
        sl = slice(q * self._B, (q + 1) * self._B)
        cut = lambda X: None if X is None else X[:, sl]
        return dataclasses.replace(o, PR=cut(o.PR), LS=cut(o.LS), TURN=cut(o.TURN),
                                   COST=cut(o.COST), NET=cut(o.NET))

    def __iter__(self):
        return iter([(J, K) for J in self._q for K in self._outs])

    def __len__(self):
        return len(self._q) * len(self._outs)


class SweepRunner:
    """Runs the (J, K) grid on batches of month panels.

    stages: object with `momentum`, `deciles`, `portfolio`, `bootstrap` (Engine signatures).
    """

    def __init__(self, stages, cfg: SweepConfig | None = None, group=None):
        self.st = stages
        self.cfg = cfg or SweepConfig()
        self.group = group
        self.G = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        # accounting branch of each bootstrap batch run_bootstrap ran, in order: "jsg" (the
        # grouped shared-return launch set), "shared" (one cohort pass, per-J accounting),
        # "per_j" or "materialised" (csm_bootstrap -> run_batch)
        self.boot_paths = []

    def run_batch(self, PMb: torch.Tensor, B: int, W=None, ADV=None, SIG=None, defer=False):
        """PMb [T_m][B*N] month prices of B panels -> summary [B][S][F] and the per-strategy
        long-short series {(J, K): PortfolioOut} (small joined batches: strided views of the
        joined outputs).  defer=True: no device sync -- returns
        (summary, series, need_full) with need_full a device int32 [1] flag (None without the
        legs-only accounting); when it reads non-zero the caller reruns with
        SweepConfig(legs_only=False) (rare: a panel lacks a leg's column).  For hipGraph capture."""
        c = self.cfg
        legs = c.legs_only and hasattr(self.st, "summary")
        flag = torch.zeros(1, dtype=torch.int32, device=PMb.device) if legs else None
        out = self._run_batch(PMb, B, W, ADV, SIG, flag)
        if defer:
            return out[0], out[1], flag
        if legs and int(flag.item()):   # a panel lacks a leg's column: every decile (rare)
            out = self._run_batch(PMb, B, W, ADV, SIG, None)
        return out

    def run_batch_sharded(self, PMb: torch.Tensor, B: int, W=None, ADV=None, SIG=None,
                          defer=False):
        """run_batch with the (J, K) grid split across the ranks (independent
        (panel, J, K) units): every rank holds the month panel, rank r runs only the r-th
        contiguous block of cfg.strategies (its look-backs' scans and decile passes, its holding
        periods' accounting), and ONE all-gather of the [B][S_r][F] summary blocks assembles the
        [B][S][F] table on every rank.  A block's strategies come out bit for bit as in the
        unsharded run: every look-back's scan, labels and accounting are the same launches on
        the same rows, and batches of up to four panels share one chunk plan (portfolio.hip
        pf_plan), so whether four, two or one look-back share a launch does not change a bit.
        Returns (summary, series of this rank's strategies) -- with defer=True also the legs
        flag (device int32 [1], or None), as run_batch(defer=True)."""
        c = self.cfg
        strategies = c.strategies
        S, F = len(strategies), len(SUMMARY_FIELDS)
        s0, s1 = panel_partition(S, self.G)[self.rank]
        mine = strategies[s0:s1]
        flag, series = None, {}
        if mine:
            Js = tuple(dict.fromkeys(J for J, _ in mine))
            Ks = tuple(dict.fromkeys(K for _, K in mine))
            sub = SweepRunner(self.st, dataclasses.replace(c, Js=Js, Ks=Ks))
            if defer:
                summ, series, flag = sub.run_batch(PMb, B, W, ADV, SIG, defer=True)
            else:
                summ, series = sub.run_batch(PMb, B, W, ADV, SIG)
            pos = {jk: i for i, jk in enumerate(sub.cfg.strategies)}
            idx = [pos[jk] for jk in mine]
            if idx != list(range(len(pos))):
                summ = summ[:, idx]
            series = {jk: series[jk] for jk in mine}
        if self.G == 1:
            return (summ, series, flag) if defer else (summ, series)
        width = max(b - a for a, b in panel_partition(S, self.G))
        pad = torch.full((B, width, F), float("nan"), dtype=PMb.dtype, device=PMb.device)
        if mine:
            pad[:, :s1 - s0] = summ
        allp = all_gather_stack(pad, self.group)                   # the one collective
        table = torch.cat([allp[g, :, :b - a] for g, (a, b) in
                           enumerate(panel_partition(S, self.G))], 1)
        return (table, series, flag) if defer else (table, series)

    def _run_batch(self, PMb, B, W, ADV, SIG, flag):
        return self._account(self._ranked(PMb, B, legs=flag is not None), B, W, ADV, SIG, flag)

    def _joined(self, T_m, B, N):
        """Whether a batch this small runs its Js' decile passes and accounting as one launch
        set over the Js side by side (join_js; every J's panels then live at once).  Only where
        the portfolio chunk plan of the nJ * B side-by-side panels is the plan of B panels, so a
        joined batch -- and a strategy-sharded rank joining fewer Js (the plan is monotone in
        the panel count) -- keeps the per-J launches' TURN / COST bits (pf_plan treats batches
        below four panels as four, not wider ones: T_m = 300, B = 2 plans two turnover chunks
        joined against four per J)."""
        c, st = self.cfg, self.st
        if not (c.join_js and hasattr(st, "summary") and len(c.Js) > 1 and T_m * B < JOIN_ROWS):
            return False
        if hasattr(st, "portfolio_plan"):
            Km = max(c.Ks)
            return (st.portfolio_plan(T_m, B, N, c.n_bins, Km)
                    == st.portfolio_plan(T_m, len(c.Js) * B, N, c.n_bins, Km))
        return True

    def _ranked(self, PMb, B, legs=False):
        """(J, L, NR) per J of the grid from the month prices of a batch: one J's ranking
        panels live at a time (small joined batches: every J's scan, then one decile pass over
        the Js' rows stacked).  legs (legs-only accounting follows): the ids decile pass may
        leave the interior deciles inexact (deciles_ids(legs=True))."""
        c, st = self.cfg, self.st
        T_m, BN = PMb.shape
        N = BN // B
        lg = {"legs": True} if _legs_labels(c, legs, N) else {}
        if self._joined(T_m, B, N):
            # every J from one time-chunked scan where it applies (csm_momentum_multi_chunked:
            # C3 scan 0.245 ms for four chunked scans), with the bucket ids for the decile pass
            Cm = (c.scan_chunks or st.default_chunks(T_m, BN, max(c.Js), c.skip)
                  if hasattr(st, "default_chunks") else 1)
            if (c.multi_j_scan and hasattr(st, "momentum_multi") and len(c.Js) <= 4 and Cm > 1
                    and max(c.Js) + c.skip <= 16 and BN % 2 == 0):
                ids = c.decile_ids and hasattr(st, "deciles_ids") and N % 4 == 0
                # (stacked: the Js' mom / next_ret / ids panels back to back, read below as one
                # tensor each -- no concatenation copies)
                MN = st.momentum_multi(PMb, c.Js, c.skip, with_ids=ids, chunks=Cm,
                                       stacked=c.grouped)
            else:
                _refuse_capture("the per-J time-chunked scans")
                ids = False
                MN = [st.momentum(PMb, J, c.skip)[1:] for J in c.Js]
            if not ids:
                _refuse_capture("the streaming narrow decile pass")
            Mcat = _stacked([mo[0] for mo in MN]).view(len(MN) * T_m * B, N)
            if ids:
                Lcat, _, _, _ = st.deciles_ids(
                    Mcat, None, _stacked([mo[2] for mo in MN]).view(len(MN) * T_m * B, N),
                    c.n_bins, **lg)
            else:
                Lcat, _, _, _ = st.deciles(Mcat, None, c.n_bins)
            R = T_m * B
            for q, J in enumerate(c.Js):
                yield J, Lcat[q * R:(q + 1) * R].reshape(T_m, BN), MN[q][1]
            return
        # multi_j_scan (wide batches): every J from one scan of PMb (csm_momentum_multi, the
        # register shift ring: C5 scan stage 30.6 -> 28.9 ms/step; bit-identical per J)
        # The multi-J scan keeps every J's M and NR live at once (2 * len(Js) [T_m][B*N] f64
        # panels, ~10 GB at C5 with batch 100); take it only when that fits in half the free
        # device memory, else scan per J (two panels live at a time).
        multi = None
        ids = (c.decile_ids and hasattr(st, "deciles_ids") and N % 4 == 0)
        need = (2 * PMb.element_size() + (2 if ids else 0)) * len(c.Js) * T_m * BN
        if (c.multi_j_scan and hasattr(st, "momentum_multi") and len(c.Js) > 1
                and st.default_chunks(T_m, BN, max(c.Js), c.skip) == 1
                and max(c.Js) + c.skip <= 64 and need <= _free_bytes(PMb) // 2):
            # by position: Js may repeat
            multi = list(st.momentum_multi(PMb, c.Js, c.skip, with_ids=True) if ids
                         else st.momentum_multi(PMb, c.Js, c.skip))
        for q, J in enumerate(c.Js):   # one J's ranking / portfolio panels live at a time
            IDS = None
            if multi is not None:
                mo, multi[q] = multi[q], None
                M, NR = mo[0], mo[1]
                IDS = mo[2] if ids else None
            else:
                _, M, NR = st.momentum(PMb, J, c.skip)
            if IDS is not None:
                L, _, _, _ = st.deciles_ids(M.reshape(T_m * B, N), None,
                                            IDS.reshape(T_m * B, N), c.n_bins, **lg)
            else:
                _refuse_capture("the streaming narrow decile pass")
                L, _, _, _ = st.deciles(M.reshape(T_m * B, N), None, c.n_bins)
            del M, IDS
            yield J, L.reshape(T_m, BN), NR
            del L, NR

    def _account(self, ranked, B, W, ADV, SIG, flag):
        """Portfolio accounting of every (J, K) from the (J, L, NR) of `ranked` -> summary
        [B][S][F] and the per-strategy series {(J, K): PortfolioOut}."""
        c, st = self.cfg, self.st
        ranked = iter(ranked)
        first = next(ranked)
        if self._joined(first[1].shape[0], B, first[1].shape[1] // B):
            return self._account_joined([first] + list(ranked), B, W, ADV, SIG, flag)
        ranked = itertools.chain([first], ranked)
        rows, series, summ = [], {}, {}
        kw = dict(W=W, B=B, half_spread=c.half_spread, k_impact=c.k_impact, aum=c.aum, ADV=ADV,
                  SIG=SIG, with_costs=c.costs)
        for J, L, NR in ranked:
            if hasattr(st, "summary"):   # device path: one cohort pass for every K of this J,
                if flag is not None:
                    kw2 = dict(kw, legs_only=True, need_full=flag)
                else:
                    kw2 = kw
                outs, stk = st.portfolio_multi(L, NR, c.n_bins, Ks=c.Ks, return_stacked=True, **kw2)
                summ_j = st.summary(stk.LS, stk.TURN, stk.COST, stk.NET)   # summaries on device
                for q, K in enumerate(c.Ks):
                    summ[(J, K)] = summ_j[q]
            elif hasattr(st, "portfolio_multi"):
                outs = st.portfolio_multi(L, NR, c.n_bins, Ks=c.Ks, **kw)
            else:
                outs = {K: st.portfolio(L, NR, c.n_bins, K=K, **kw) for K in c.Ks}
            for K in c.Ks:
                series[(J, K)] = outs[K]
            del L, NR
        for (J, K) in c.strategies:
            if (J, K) in summ:
                rows.append(summ[(J, K)])
            else:
                out = series[(J, K)]
                rows.append(summarize(out.LS, out.TURN, out.COST, out.NET))
        return torch.stack(rows, dim=1), series                  # [B][S][F]

    def _account_joined(self, items, B, W, ADV, SIG, flag):
        """_account for a small batch: the Js' labels / next_ret side by side as nJ * B panels
        (panel q * B + b = J q's panel b; weights / ADV / vol repeated per J), one cohort pass, one
        accounting launch set and one summary launch for the whole (J, K) grid instead of one per
        J -- C3's single-panel rows are latency-bound per launch.  Same rules, same bits as the
        per-J calls (one chunk plan for batches of up to four panels)."""
        c, st = self.cfg, self.st
        nJ = len(items)
        if c.grouped and hasattr(st, "portfolio_multi_grouped"):
            # the Js' label / next_ret panels group-major as the stacked decile pass and scan
            # wrote them, weights / ADV / vol once for every J (csm_*_grouped: the same bits as
            # the side-by-side copies below, without making them)
            Lg = _stacked([it[1] for it in items])
            NRg = _stacked([it[2] for it in items])
            kw = dict(W=W, Bg=B, half_spread=c.half_spread, k_impact=c.k_impact, aum=c.aum,
                      ADV=ADV, SIG=SIG, with_costs=c.costs)
            if flag is not None:
                kw.update(legs_only=True, need_full=flag)
            outs, stk = st.portfolio_multi_grouped(Lg, NRg, c.n_bins, Ks=c.Ks, return_stacked=True,
                                                   **kw)
            del Lg, NRg
        else:
            rep = lambda X: None if X is None else X.repeat(1, nJ)
            L = torch.cat([it[1] for it in items], dim=1)
            NR = torch.cat([it[2] for it in items], dim=1)
            kw = dict(W=rep(W), B=nJ * B, half_spread=c.half_spread, k_impact=c.k_impact,
                      aum=c.aum, ADV=rep(ADV), SIG=rep(SIG), with_costs=c.costs)
            if flag is not None:
                kw.update(legs_only=True, need_full=flag)
            outs, stk = st.portfolio_multi(L, NR, c.n_bins, Ks=c.Ks, return_stacked=True, **kw)
            del L, NR
        summ_all = st.summary(stk.LS, stk.TURN, stk.COST, stk.NET)   # [nK][nJ * B][F]
        return self._joined_table(summ_all, outs, [it[0] for it in items], B)

    def _joined_table(self, summ_all, outs, Js, B):
        """(summary [B][S][F], series) of a joined accounting (panel q * B + b = J q's panel b)
        from its [nK][nJ * B][F] summaries and {K: PortfolioOut}."""
        c = self.cfg
        # per-(J, K) series: strided views of the joined outputs, built when read (C3's step is
        # host-bound: 16 strategies x 5 views a step cost more than the GPU work they describe)
        series = _JoinedSeries(outs, Js, B)
        nK, nJ, F = len(c.Ks), len(Js), summ_all.shape[-1]
        if len(set(Js)) == nJ and len(set(c.Ks)) == nK and Js == [int(J) for J in c.Js]:
            # strategy s = J index * nK + K index (strategy_grid): one permuted copy
            return summ_all.view(nK, nJ, B, F).permute(2, 1, 0, 3).reshape(B, nJ * nK, F), series
        summ = {}
        for q, J in enumerate(Js):
            for k, K in enumerate(c.Ks):
                summ[(J, K)] = summ_all[k, q * B:(q + 1) * B]
        rows = [summ[(J, K)] for (J, K) in c.strategies]
        return torch.stack(rows, dim=1), series                  # [B][S][F]

    def _boot_ok(self, T_m, N, B):
        c = self.cfg
        ids = c.decile_ids and hasattr(self.st, "deciles_ids") and N % 4 == 0
        nJ = len(c.Js)
        # live together: boot_scan's mom_J (+ ids) per J and the shared next_ret, then each J's
        # int8 label panel and portfolio workspace (portfolio_multi_js allocates them at once)
        need = (8 + (2 if ids else 0)) * nJ * T_m * B * N + 8 * T_m * B * N + nJ * T_m * B * N
        lib = getattr(self.st, "lib", None)
        if lib is not None and hasattr(lib, "csm_portfolio_workspace"):
            need += nJ * int(lib.csm_portfolio_workspace(T_m, B, N, c.n_bins, max(c.Ks)))
        return (c.boot_scan and hasattr(self.st, "boot_scan") and N % 2 == 0
                and 1 <= len(c.Js) <= 4 and max(c.Js) + c.skip <= 16
                and need <= _free_bytes_dev(self.st) // 2)

    def run_boot_batch(self, R_base, B, b0, seed=5000, mean_block=6.0):
        """Bootstrap panels b0 .. b0+B-1 through csm_boot_scan (the panel generated in registers,
        every J from one scan, one shared next_ret), then the decile pass and the accounting:
        the summary table equals run_batch on csm_bootstrap's panel bit for bit.  A batch whose
        generated prices leave the shared next_ret's domain (a price not finite and non-zero) is
        rerun that way."""
        out, state, redo = self._boot_batch(R_base, B, b0, seed, mean_block)
        v = int(state.item())
        return redo(v) if v else out

    def _boot_batch(self, R_base, B, b0, seed, mean_block, legs=True):
        """run_boot_batch without the device sync: (out, state, redo) with state a device int32
        [1] (bit 1: a generated price left the shared next_ret's domain, bit 0: a panel lacks a
        leg's column) and redo(int(state)) the batch's final (summary, series)."""
        c, st = self.cfg, self.st
        T_m, N = R_base.shape
        ids = c.decile_ids and hasattr(st, "deciles_ids") and N % 4 == 0
        _, outs, NR, bad = st.boot_scan(R_base, B, c.Js, c.skip, b0=b0, seed=seed,
                                        mean_block=mean_block, with_ids=ids)
        legs = legs and c.legs_only and hasattr(st, "summary")
        flag = torch.zeros(1, dtype=torch.int32, device=NR.device) if legs else None
        lg = {"legs": True} if _legs_labels(c, legs, N) else {}
        # grouped shared-return accounting: the Js' labels written group-major by their decile
        # passes, one cohort pass and ONE accounting launch set for every J -- where the batch's
        # chunk plan is that of the Js' panels side by side, so every table entry keeps its bits
        nJ, Km = len(c.Js), max(c.Ks)
        jsg = (ids and c.share_nr and c.grouped and nJ > 1 and not self._joined(T_m, B, N)
               and hasattr(st, "portfolio_multi_js_grouped") and hasattr(st, "portfolio_plan")
               and st.portfolio_plan(T_m, B, N, c.n_bins, Km)
               == st.portfolio_plan(T_m, nJ * B, N, c.n_bins, Km))
        Lg = torch.empty((nJ, T_m * B, N), dtype=torch.int8, device=NR.device) if jsg else None
        labels = []
        if jsg:   # every J's rows in one decile pass (boot_scan wrote the panels back to back)
            Ms, Is = _stacked([o[0] for o in outs]), _stacked([o[1] for o in outs])
            outs = None
            st.deciles_ids(Ms.view(nJ * T_m * B, N), None, Is.view(nJ * T_m * B, N), c.n_bins,
                           out=(Lg.view(nJ * T_m * B, N), None, None, None), **lg)
            del Ms, Is
        for q, J in enumerate(c.Js):
            if jsg:
                break
            (M, IDS), outs[q] = outs[q], None
            if IDS is not None:
                L, _, _, _ = st.deciles_ids(M.reshape(T_m * B, N), None, IDS.reshape(T_m * B, N),
                                            c.n_bins, **lg)
            else:
                L, _, _, _ = st.deciles(M.reshape(T_m * B, N), None, c.n_bins)
            del M, IDS
            labels.append((J, L.reshape(T_m, B * N), NR))
        shared = False
        if jsg:
            out = self._account_js_grouped(Lg.view(nJ, T_m, B * N), NR, B, flag)
        else:
            shared = (c.share_nr and hasattr(st, "portfolio_multi_js") and len(labels) > 1
                      and not self._joined(T_m, B, N))
            acc = self._account_shared if shared else self._account
            out = acc(labels, B, None, None, None, flag)
        del labels, NR, Lg
        self.boot_paths.append("jsg" if jsg else ("shared" if shared else "per_j"))
        state = bad * 2 + (flag if legs else 0)

        def redo(v):   # holds no panel: a flagged batch is recomputed from its seed
            if v & 2:   # (never on finite returns) the materialised path
                _, PMb = st.bootstrap(R_base, B, b0=b0, seed=seed, mean_block=mean_block)
                return self.run_batch(PMb, B)
            if v & 1:   # a panel lacks a leg's column: every decile (rare)
                o, st2, _ = self._boot_batch(R_base, B, b0, seed, mean_block, legs=False)
                if int(st2.item()) & 2:
                    return redo(2)
                return o
            return None
        return out, state, redo

    def _account_js_grouped(self, Lg, NR, B, flag):
        """_account_shared with the Js' labels group-major (Lg [nJ][T_m][B * N]): one cohort
        pass over the shared next_ret and one accounting launch set for every J
        (portfolio_multi_js_grouped), then one summary launch -- the same table and series."""
        c, st = self.cfg, self.st
        outs, stk = st.portfolio_multi_js_grouped(
            Lg, NR, c.n_bins, Ks=c.Ks, B=B, half_spread=c.half_spread, k_impact=c.k_impact,
            aum=c.aum, with_costs=c.costs, legs_only=flag is not None, need_full=flag,
            return_stacked=True)
        summ_all = st.summary(stk.LS, stk.TURN, stk.COST, stk.NET)   # [nK][nJ * B][F]
        return self._joined_table(summ_all, outs, [int(J) for J in c.Js], B)

    def _account_shared(self, labels, B, W, ADV, SIG, flag):
        """_account for Js that share one next_ret panel (bootstrap batches, no weights / ADV /
        vol): one cohort pass for every J (portfolio_multi_js), then each J's accounting and
        summary -- the same table and series as _account, bit for bit."""
        c, st = self.cfg, self.st
        assert W is None and ADV is None and SIG is None
        NR = labels[0][2]
        outs = st.portfolio_multi_js([L for _, L, _ in labels], NR, c.n_bins, Ks=c.Ks, B=B,
                                     half_spread=c.half_spread, k_impact=c.k_impact, aum=c.aum,
                                     with_costs=c.costs, legs_only=flag is not None,
                                     need_full=flag)
        series, summ = {}, {}
        for (J, _, _), (res, stk) in zip(labels, outs):
            summ_j = st.summary(stk.LS, stk.TURN, stk.COST, stk.NET)
            for q, K in enumerate(c.Ks):
                summ[(J, K)] = summ_j[q]
                series[(J, K)] = res[K]
        rows = [summ[(J, K)] for (J, K) in c.strategies]
        return torch.stack(rows, dim=1), series                  # [B][S][F]

    def run_bootstrap(self, R_base: torch.Tensor, n_panels: int, seed: int = 5000,
                      mean_block: float = 6.0, batch: int = 64):
        """C5: n_panels stationary-bootstrap panels of the base month returns, this rank's
        contiguous share in batches; one all-gather of the summary table.  Returns the full
        [n_panels][S][F] table on every rank."""
        T_m, N = R_base.shape
        p0, p1 = panel_partition(n_panels, self.G)[self.rank]
        S, F = len(self.cfg.strategies), len(SUMMARY_FIELDS)
        mine, pend = [], []
        for b0 in range(p0, p1, batch):
            B = min(batch, p1 - b0)
            if self._boot_ok(T_m, N, B):
                # no sync per batch: the batches' flags are read once after the last launch
                (summ, _), state, redo = self._boot_batch(R_base, B, b0, seed, mean_block)
                pend.append((len(mine), state, redo))
            else:
                _, PMb = self.st.bootstrap(R_base, B, b0=b0, seed=seed, mean_block=mean_block)
                summ, _ = self.run_batch(PMb, B)
                self.boot_paths.append("materialised")
            mine.append(summ)
        if pend:
            states = torch.cat([s for _, s, _ in pend]).tolist()   # one sync for every batch
            for (i, _, redo), v in zip(pend, states):
                if v:   # rare: rerun that batch (materialised panel / every decile)
                    mine[i] = redo(v)[0]
        local = (torch.cat(mine, 0) if mine else
                 torch.empty((0, S, F), dtype=R_base.dtype, device=R_base.device))
        if self.G == 1:
            return local
        width = max(b - a for a, b in panel_partition(n_panels, self.G))
        pad = torch.full((width, S, F), float("nan"), dtype=local.dtype, device=local.device)
        pad[:local.shape[0]] = local
        allp = all_gather_stack(pad, self.group)                   # the one collective
        parts = panel_partition(n_panels, self.G)
        return torch.cat([allp[g, :b - a] for g, (a, b) in enumerate(parts)], 0)
