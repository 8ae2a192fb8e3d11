// deciles_chunked.hip -- the wide-row decile pass on bucket ids (csm_pipeline / csm_deciles_ids,
// rows wider than the narrow-row kernels: C4's 100k-asset dates), as three launches that keep the
// bandwidth-bound sweep load-balanced over the whole chip:
//
//   k_dec_hist   one workgroup per date: 8192-bucket histogram of the fixed-map ids (2 B per
//                cell), ranked count n, exclusive prefix, and for every bin edge k the bucket
//                range [rlo_k, rhi_k] holding its order statistics (edge 0: the minimum's
//                bucket, edge n_bins: the maximum's).  When the ranges are pairwise disjoint (no
//                two edges can then be equal) every cell outside them has a label fixed by its
//                bucket alone -- the map is monotone -- and the cells inside the interior ranges
//                are exactly the candidates of the order statistics.  Otherwise (ties across
//                edges, tiny rows, oversized candidate sets) the row is flagged for the general
//                kernel (deciles.inc PRE mode), as the merged pass did.
//   k_dec_sweep  a grid of (chunk, date) workgroups, 8192 cells each: ids + next_ret read once,
//                labels of the certain cells written four per word, their next_ret summed per
//                label (fixed per-lane order, then a fixed two-sum tree) into a per-chunk
//                partial, the uncertain cells appended to per-wave index lists.
//   k_dec_finish one workgroup per date: mom_J and next_ret of the listed cells (~0.2 % of a
//                row), counting selection of the order statistics inside each range, NumPy's
//                lerp for the edges, exact labels of the listed cells, their sums; the per-label
//                totals = the chunk partials in chunk order + the listed cells' (deterministic).
//
// Labels / counts / ranked rows are bit-identical to the streaming kernel and to the merged pass
// (the same exact order statistics and edges); decile means differ from theirs only by
// summation order (<= 1e-13 relative; pandas' own Kahan sums agree with each within 1e-10).
// Reference: run_demo.py:18-29,46 (per-date pd.qcut, duplicates='drop'), :49-55 (dropna, mean).
#include "csm_common.h"

#define DC_HB 8192          // = CSM_FB_BUCKETS: the fixed map's ids, no coarsening
#define DC_HIST_THREADS 512
#define DC_SWEEP_THREADS 256
#define DC_FIN_THREADS 256
#define DC_CAP 2048         // candidates per row (cells of the interior ranges)
#define DC_LW 256           // list entries per wave and chunk
#define DC_REC 192          // ints per row record

// row record (int32 offsets)
#define R_N 0
#define R_TOTAL 1
#define R_RLO 4
#define R_RHI (R_RLO + MAXQ)
#define R_PRE (R_RHI + MAXQ)
#define R_CNT (R_PRE + MAXQ)
#define R_OFF (R_CNT + MAXQ)
#define R_RP (R_OFF + MAXQ)   // residual ranks (inside the range) of edge k's two order statistics
#define R_RQ (R_RP + MAXQ)
static_assert(R_RQ + MAXQ <= DC_REC, "row record");

namespace {

__device__ __forceinline__ int bucket_of_rank(const uint32_t* pre, int64_t r) {
  int lo = 0, hi = DC_HB - 1;   // last bucket b with prefix[b] <= r
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((int64_t)pre[mid] <= r) lo = mid; else hi = mid - 1;
  }
  return lo;
}

}  // namespace

// ------------------------------------------------------------------------------ k_dec_hist
template <int NB>
__global__ __launch_bounds__(DC_HIST_THREADS, 2) void k_dec_hist(const uint16_t* __restrict__ IDS,
                                                               int64_t N, QTab qt,
                                                               int32_t* __restrict__ REC,
                                                               int32_t* __restrict__ FLG) {
  __shared__ uint32_t hist[DC_HB];
  __shared__ uint32_t wtot[DC_HIST_THREADS / 64];
  __shared__ int64_t red[DC_HIST_THREADS / 64];
  const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int b = tid; b < DC_HB; b += DC_HIST_THREADS) hist[b] = 0;
  __syncthreads();
  const uint16_t* irow = IDS + (int64_t)t * N;
  int64_t cnt = 0;
  {
    const int64_t step = 4 * DC_HIST_THREADS;
    constexpr int HU = 8;
    for (int64_t i0 = 4 * (int64_t)tid; i0 < N; i0 += HU * step) {
      uint2 pk[HU];
#pragma unroll
      for (int u = 0; u < HU; ++u) {
        const int64_t i = i0 + u * step;
        pk[u] = i < N ? *reinterpret_cast<const uint2*>(irow + i) : make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
      }
#pragma unroll
      for (int u = 0; u < HU; ++u) {
        const uint32_t id[4] = {pk[u].x & 0xFFFFu, pk[u].x >> 16, pk[u].y & 0xFFFFu, pk[u].y >> 16};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const bool ok = id[k] != CSM_FB_NAN;
          cnt += ok ? 1 : 0;
          if (ok) atomicAdd(&hist[id[k]], 1u);
        }
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_down(cnt, o, 64);
  if (lane == 0) red[wid] = cnt;
  __syncthreads();
  int64_t n = 0;
#pragma unroll
  for (int w = 0; w < DC_HIST_THREADS / 64; ++w) n += red[w];
  // exclusive prefix of the histogram in place: per-thread sums of 16 buckets, a wave scan,
  // then the wave totals
  {
    constexpr int per = DC_HB / DC_HIST_THREADS;
    uint32_t loc[per], s = 0;
#pragma unroll
    for (int j = 0; j < per; ++j) { loc[j] = hist[tid * per + j]; s += loc[j]; }
    uint32_t inc = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(inc, o, 64);
      if (lane >= o) inc += v;
    }
    if (lane == 63) wtot[wid] = inc;
    __syncthreads();
    uint32_t run = inc - s;
    for (int w = 0; w < wid; ++w) run += wtot[w];
#pragma unroll
    for (int j = 0; j < per; ++j) { hist[tid * per + j] = run; run += loc[j]; }
    __syncthreads();
  }
  if (wid != 0) return;
  // wave 0, lane k <= NB: edge k's bucket range
  int32_t* rec = REC + (int64_t)t * DC_REC;
  const int k = lane;
  bool ok = true;
  int rl = 0, rh = 0, pre = 0, cn = 0, rp = 0, rq = 0;
  if (n > 0 && k <= NB) {
    if (k == 0) {
      rl = rh = bucket_of_rank(hist, 0);
    } else if (k == NB) {
      rl = rh = bucket_of_rank(hist, n - 1);
    } else {
      const double v = (double)(n - 1) * qt.q[k];
      if (!(v < (double)(n - 1))) {
        ok = false;
      } else {
        const double p = floor(v);
        const int64_t pi = (int64_t)p;
        const int64_t ph = (v - p != 0.0) ? pi + 1 : pi;
        if (pi < 1 || ph > n - 2) {
          ok = false;
        } else {
          rl = bucket_of_rank(hist, pi);
          rh = bucket_of_rank(hist, ph);
          pre = (int)hist[rl];
          cn = (int)((rh + 1 < DC_HB ? (int64_t)hist[rh + 1] : n) - pre);
          rp = (int)(pi - pre);
          rq = (int)(ph - pre);
        }
      }
    }
  }
  const int nl = __shfl_down(rl, 1, 64);
  if (n > 0 && k < NB && !(rh < nl)) ok = false;   // ranges pairwise disjoint and increasing
  int inc = (k <= NB) ? cn : 0;
  const int own = inc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(inc, o, 64);
    if (lane >= o) inc += v;
  }
  const int total = __shfl(inc, 63, 64);
  const uint64_t bad = __ballot(k <= NB && !ok);
  const bool fast = n == 0 || (bad == 0 && total <= DC_CAP);
  if (k <= NB) {
    rec[R_RLO + k] = rl;
    rec[R_RHI + k] = rh;
    rec[R_PRE + k] = pre;
    rec[R_CNT + k] = cn;
    rec[R_OFF + k] = inc - own;
    rec[R_RP + k] = rp;
    rec[R_RQ + k] = rq;
  }
  if (lane == 0) {
    rec[R_N] = (int32_t)n;
    rec[R_TOTAL] = total;
    FLG[t] = fast ? 0 : 1;   // 1: the general kernel ranks this row
  }
}

// ----------------------------------------------------------------------------- k_dec_sweep
// Chunk (blockIdx.x) of date t (blockIdx.y): ITER groups of 4 cells per lane, all loads issued
// before any is used.  The bucket -> label table of the row is rebuilt in LDS from the record's
// ranges (8 KB; one barrier), so a cell's label is one LDS byte read.
template <int NB, int ITER>
__global__ __launch_bounds__(DC_SWEEP_THREADS) void k_dec_sweep(
    const uint16_t* __restrict__ IDS, const double* __restrict__ NR, int64_t N,
    const int32_t* __restrict__ REC, int32_t* __restrict__ FLG, int8_t* __restrict__ L,
    double* __restrict__ PART, int32_t* __restrict__ LCNT, uint32_t* __restrict__ LIST) {
  constexpr int NW = DC_SWEEP_THREADS / 64;
  constexpr int64_t CH = (int64_t)ITER * 4 * DC_SWEEP_THREADS;
  __shared__ __attribute__((aligned(16))) int8_t tab[DC_HB];
  // per-lane label sums in LDS, one private column per lane: a cell adds with one ds_add_f64 /
  // ds_add_u32 (no return, no contention, the lane's cells in program order -- so the same
  // rounding as sequential adds, deterministic) instead of NB compare / select / fma per cell
  // in registers, which made the sweep VALU-bound
  __shared__ double acc[NB][DC_SWEEP_THREADS];
  __shared__ uint32_t acn[NB][DC_SWEEP_THREADS];
  __shared__ double wh[NW][NB], wlo[NW][NB];
  __shared__ int wc[NW][NB];
  const int c = blockIdx.x, t = blockIdx.y, C = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (FLG[t]) return;   // the general kernel ranks this row
  const int32_t* rec = REC + (int64_t)t * DC_REC;
  const int64_t i0 = (int64_t)c * CH + 4 * tid;
  const int64_t i_end = min(N, (int64_t)(c + 1) * CH);
  const uint16_t* irow = IDS + (int64_t)t * N;
  const double* nrow = NR + (int64_t)t * N;
  int8_t* lrow = L + (int64_t)t * N;
  // every load of the chunk in flight first
  uint2 pk[ITER];
  double2 ra[ITER], rb[ITER];
#pragma unroll
  for (int u = 0; u < ITER; ++u) {
    const int64_t i = i0 + (int64_t)u * 4 * DC_SWEEP_THREADS;
    pk[u] = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
    ra[u] = rb[u] = make_double2(0.0, 0.0);
    if (i < i_end) {
      pk[u] = *reinterpret_cast<const uint2*>(irow + i);
      ra[u] = *reinterpret_cast<const double2*>(nrow + i);
      rb[u] = *reinterpret_cast<const double2*>(nrow + i + 2);
    }
  }
  // bucket -> label table meanwhile: the ranges are sorted and disjoint; inside edge 0's /
  // edge NB's range the label is 0 / NB - 1, inside an interior range -3 (uncertain), between
  // ranges j - 1 and j: j - 1.  Each thread owns 32 consecutive buckets.
  {
    constexpr int PT = DC_HB / DC_SWEEP_THREADS;
    const int b0 = tid * PT;
    int j = 0;   // ranges wholly below the current bucket
    while (j <= NB && rec[R_RHI + j] < b0) ++j;
    uint32_t w = 0;
#pragma unroll 4
    for (int o = 0; o < PT; ++o) {
      const int b2 = b0 + o;
      while (j <= NB && rec[R_RHI + j] < b2) ++j;
      int lab = j - 1;
      if (j <= NB && rec[R_RLO + j] <= b2) lab = j == 0 ? 0 : (j == NB ? NB - 1 : -3);
      w |= (uint32_t)(uint8_t)(int8_t)lab << (8 * (o & 3));
      if ((o & 3) == 3) { reinterpret_cast<uint32_t*>(tab + b0)[o >> 2] = w; w = 0; }
    }
  }
  __syncthreads();
  const int64_t wl = ((int64_t)t * C + c) * NW + wid;   // this wave's list
  uint32_t* list = LIST + wl * DC_LW;
  const uint64_t lt = (1ull << lane) - 1ull;
  int lc = 0;   // wave-uniform list length
#pragma unroll
  for (int d = 0; d < NB; ++d) { acc[d][tid] = 0.0; acn[d][tid] = 0u; }
#pragma unroll
  for (int u = 0; u < ITER; ++u) {
    const int64_t i = i0 + (int64_t)u * 4 * DC_SWEEP_THREADS;
    const uint32_t id[4] = {pk[u].x & 0xFFFFu, pk[u].x >> 16, pk[u].y & 0xFFFFu, pk[u].y >> 16};
    const double rs[4] = {ra[u].x, ra[u].y, rb[u].x, rb[u].y};
    int lab[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) lab[q] = id[q] == CSM_FB_NAN ? -1 : (int)tab[id[q]];
    const uint32_t w = (uint32_t)(uint8_t)lab[0] | ((uint32_t)(uint8_t)lab[1] << 8) |
                       ((uint32_t)(uint8_t)lab[2] << 16) | ((uint32_t)(uint8_t)lab[3] << 24);
    if (i < i_end) *reinterpret_cast<uint32_t*>(lrow + i) = w;   // uncertain bytes: finish
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (lab[q] >= 0 && rs[q] == rs[q]) {
        atomicAdd(&acc[lab[q]][tid], rs[q]);
        atomicAdd(&acn[lab[q]][tid], 1u);
      }
    }
    // uncertain cells into the wave's list, (group, cell, lane) order: deterministic
    const bool any = lab[0] == -3 || lab[1] == -3 || lab[2] == -3 || lab[3] == -3;
    if (__ballot(any)) {   // wave-uniform, rare
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool un = lab[q] == -3;
        const uint64_t mk = __ballot(un);
        const int pos = lc + __popcll(mk & lt);
        if (un && pos < DC_LW) list[pos] = (uint32_t)(i + q);
        lc += __popcll(mk);
      }
    }
  }
  const bool ovf = lc > DC_LW;
  if (lane == 0) LCNT[wl] = ovf ? 0 : lc;
  if (ovf && lane == 0) FLG[t] = 1;   // (idempotent) the general kernel re-ranks the row
  // per-label partial sums of the chunk: wave trees (two-sum), waves in order
#pragma unroll
  for (int d = 0; d < NB; ++d) {
    double h = acc[d][tid], l = 0.0;
    int cc = (int)acn[d][tid];
    for (int o = 32; o > 0; o >>= 1) {
      const double h2 = __shfl_down(h, o, 64), l2 = __shfl_down(l, o, 64);
      const int c2 = __shfl_down(cc, o, 64);
      const double s2 = h + h2, bb = s2 - h;
      const double err = (h - (s2 - bb)) + (h2 - bb);
      h = s2; l = (l + l2) + err; cc += c2;
    }
    if (lane == 0) { wh[wid][d] = h; wlo[wid][d] = l; wc[wid][d] = cc; }
  }
  __syncthreads();
  if (tid < NB) {
    const int d = tid;
    double h = 0.0, l = 0.0;
    int cc = 0;
#pragma unroll
    for (int w2 = 0; w2 < NW; ++w2) {
      const double h2 = wh[w2][d], s2 = h + h2, bb = s2 - h;
      const double err = (h - (s2 - bb)) + (h2 - bb);
      h = s2; l = (l + wlo[w2][d]) + err; cc += wc[w2][d];
    }
    double* p = PART + (((int64_t)t * C + c) * NB + d) * 3;
    p[0] = h;
    p[1] = l;
    p[2] = (double)cc;
  }
}

// ---------------------------------------------------------------------------- k_dec_finish
template <int NB>
__global__ __launch_bounds__(DC_FIN_THREADS) void k_dec_finish(
    const double* __restrict__ M, const double* __restrict__ NR, int64_t N, int C, QTab qt,
    const int32_t* __restrict__ REC, const int32_t* __restrict__ FLG, int8_t* __restrict__ L,
    const double* __restrict__ PART, const int32_t* __restrict__ LCNT,
    const uint32_t* __restrict__ LIST, double* __restrict__ EW, int32_t* __restrict__ CNT,
    int32_t* __restrict__ NV) {
  constexpr int NWS = DC_SWEEP_THREADS / 64;   // lists per chunk
  constexpr int NWF = DC_FIN_THREADS / 64;
  __shared__ uint32_t ent[DC_CAP];
  __shared__ double xv[DC_CAP], rv[DC_CAP], cand[DC_CAP];
  __shared__ uint8_t ck[DC_CAP];
  __shared__ int lofs[65];
  __shared__ int fill[MAXQ], roff[MAXQ], rcnt[MAXQ], rrp[MAXQ], rrq[MAXQ];
  __shared__ double aval[MAXQ], bval[MAXQ], bins[MAXQ];
  __shared__ double wh[NWF][NB], wlo[NWF][NB];
  __shared__ int wc[NWF][NB];
  const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (FLG[t]) return;   // the general kernel ranks this row
  const int32_t* rec = REC + (int64_t)t * DC_REC;
  const int64_t n = rec[R_N];
  if (NV && tid == 0) NV[t] = (int32_t)n;
  const double* row = M + (int64_t)t * N;
  const double* nrow = NR + (int64_t)t * N;
  int8_t* lrow = L + (int64_t)t * N;
  if (tid <= NB) {
    fill[tid] = 0;
    roff[tid] = rec[R_OFF + tid];
    rcnt[tid] = rec[R_CNT + tid];
    rrp[tid] = rec[R_RP + tid];
    rrq[tid] = rec[R_RQ + tid];
  }
  // the row's lists, (chunk, wave) order, compacted into ent[]
  const int nl = C * NWS;
  for (int l0 = 0; l0 < nl; l0 += 64) {   // block-uniform trip count
    if (wid == 0) {
      const int l = l0 + lane;
      const int cl = l < nl ? LCNT[(int64_t)t * nl + l] : 0;
      int inc = cl;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(inc, o, 64);
        if (lane >= o) inc += v;
      }
      const int base = l0 == 0 ? 0 : lofs[64];
      __builtin_amdgcn_wave_barrier();
      lofs[lane] = base + inc - cl;
      if (lane == 63) lofs[64] = base + inc;
    }
    __syncthreads();
    for (int l = l0 + wid; l < min(nl, l0 + 64); l += NWF) {   // one wave per list
      const int cl = LCNT[(int64_t)t * nl + l];
      const int o = lofs[l - l0];
      const uint32_t* src = LIST + ((int64_t)t * nl + l) * DC_LW;
      for (int j = lane; j < cl; j += 64)
        if (o + j < DC_CAP) ent[o + j] = src[j];
    }
    __syncthreads();
  }
  const int ne = min(lofs[64], DC_CAP);   // == the row's candidate total (checked by k_dec_hist)
  int rhi[NB + 1];
#pragma unroll
  for (int k = 0; k <= NB; ++k) rhi[k] = rec[R_RHI + k];
  // mom_J and next_ret of the listed cells (all loads in flight), the values into their
  // range's candidate slots
  for (int p = tid; p < ne; p += DC_FIN_THREADS) {
    const uint32_t idx = ent[p];
    const double x = row[idx];
    rv[p] = nrow[idx];
    xv[p] = x;
    const int b = csm_fbucket(x);
    int j = 0;
#pragma unroll
    for (int k = 0; k <= NB; ++k) j += rhi[k] < b ? 1 : 0;   // x lies in interior range j
    const int q = roff[j] + atomicAdd(&fill[j], 1);
    cand[q] = x;
    ck[q] = (uint8_t)j;
  }
  __syncthreads();
  // order statistics inside each range by counting selection (ties broken by slot position):
  // the member whose rank equals the target's residual rank
  for (int p = tid; p < ne; p += DC_FIN_THREADS) {
    const int k = ck[p];
    const int off = roff[k], cntk = rcnt[k];
    const int i = p - off;
    const double x = cand[p];
    int rank = 0;
    for (int j = 0; j < cntk; ++j) {
      const double y = cand[off + j];
      rank += (y < x || (y == x && j < i)) ? 1 : 0;
    }
    if (rank == rrp[k]) aval[k] = x;
    if (rank == rrq[k]) bval[k] = x;
  }
  __syncthreads();
  // interior edges (NumPy _lerp); edge 0 / n_bins (min / max) never decide a listed cell's label
  if (tid > 0 && tid < NB) {
    const int k = tid;
    const double v = (double)(n - 1) * qt.q[k];
    const double p = floor(v);
    const double g = v - p;
    const double a = aval[k];
    const double b = (g != 0.0) ? bval[k] : a;
    const double d = b - a;
    bins[k] = (g >= 0.5) ? (b - d * (1.0 - g)) : (a + d * g);
  }
  __syncthreads();
  double eb[NB > 1 ? NB - 1 : 1];
#pragma unroll
  for (int k = 1; k < NB; ++k) eb[k - 1] = bins[k];
  double hs[NB];
  int cn[NB];
#pragma unroll
  for (int d = 0; d < NB; ++d) { hs[d] = 0.0; cn[d] = 0; }
  // labels of the listed cells (searchsorted-left over the edges: every listed cell is above
  // edge 0 and below edge n_bins), next_ret summed in list order
  for (int p = tid; p < ne; p += DC_FIN_THREADS) {
    const double x = xv[p];
    int lab = 0;
#pragma unroll
    for (int k = 1; k < NB; ++k) lab += eb[k - 1] < x ? 1 : 0;
    lrow[ent[p]] = (int8_t)lab;
    const double r = rv[p];
    const bool ok = r == r;
#pragma unroll
    for (int d = 0; d < NB; ++d) {
      const bool h = ok && lab == d;
      hs[d] = fma(h ? 1.0 : 0.0, ok ? r : 0.0, hs[d]);
      cn[d] += h ? 1 : 0;
    }
  }
#pragma unroll
  for (int d = 0; d < NB; ++d) {
    double h = hs[d], l = 0.0;
    int cc = cn[d];
    for (int o = 32; o > 0; o >>= 1) {
      const double h2 = __shfl_down(h, o, 64), l2 = __shfl_down(l, o, 64);
      const int c2 = __shfl_down(cc, o, 64);
      const double s2 = h + h2, bb = s2 - h;
      const double err = (h - (s2 - bb)) + (h2 - bb);
      h = s2; l = (l + l2) + err; cc += c2;
    }
    if (lane == 0) { wh[wid][d] = h; wlo[wid][d] = l; wc[wid][d] = cc; }
  }
  __syncthreads();
  if (tid < NB) {
    const int d = tid;
    double h = 0.0, l = 0.0;
    int cc = 0;
    auto add = [&](double h2, double l2, int c2) {
      const double s2 = h + h2, bb = s2 - h;
      const double err = (h - (s2 - bb)) + (h2 - bb);
      h = s2; l = (l + l2) + err; cc += c2;
    };
    for (int c = 0; c < C; ++c) {   // the chunks' certain cells, in chunk order
      const double* pp = PART + (((int64_t)t * C + c) * NB + d) * 3;
      add(pp[0], pp[1], (int)pp[2]);
    }
#pragma unroll
    for (int w2 = 0; w2 < NWF; ++w2) add(wh[w2][d], wlo[w2][d], wc[w2][d]);   // the listed cells
    const double sum = h + l;
    EW[(int64_t)t * NB + d] = cc > 0 ? sum / (double)cc : qnan();
    if (CNT) CNT[(int64_t)t * NB + d] = cc;
  }
}

// ------------------------------------------------------------------------------- launcher
#define DC_ITER 8   // 8 x 1024 cells per sweep workgroup (C4: 13 chunks x 461 dates)

size_t deciles_chunked_workspace(int T_m, int64_t N) {
  const int64_t CH = (int64_t)DC_ITER * 4 * DC_SWEEP_THREADS;
  const int64_t C = (N + CH - 1) / CH;
  const int64_t NWS = DC_SWEEP_THREADS / 64;
  size_t b = 0;
  auto al = [](size_t x) { return (x + 255) / 256 * 256; };
  b = al(b + (size_t)T_m * DC_REC * 4);                  // REC
  b = al(b + (size_t)T_m * C * 20 * 3 * 8);              // PART (NB <= 20)
  b = al(b + (size_t)T_m * C * NWS * 4);                 // LCNT
  b = al(b + (size_t)T_m * C * NWS * DC_LW * 4);         // LIST
  return b;
}

template <int NB>
void launch_deciles_chunked(int T_m, hipStream_t st, const double* M, const double* NR, int64_t N,
                            const QTab& q, int8_t* L, double* EW, int32_t* CNT, int32_t* NV,
                            const uint16_t* ids, int32_t* flg, void* ws) {
  const int64_t CH = (int64_t)DC_ITER * 4 * DC_SWEEP_THREADS;
  const int C = (int)((N + CH - 1) / CH);
  const int64_t NWS = DC_SWEEP_THREADS / 64;
  auto al = [](size_t x) { return (x + 255) / 256 * 256; };
  char* w = (char*)ws;
  size_t o = 0;
  int32_t* REC = (int32_t*)(w + o); o = al(o + (size_t)T_m * DC_REC * 4);
  double* PART = (double*)(w + o); o = al(o + (size_t)T_m * C * 20 * 3 * 8);
  int32_t* LCNT = (int32_t*)(w + o); o = al(o + (size_t)T_m * C * NWS * 4);
  uint32_t* LIST = (uint32_t*)(w + o);
  hipLaunchKernelGGL((k_dec_hist<NB>), dim3(T_m), dim3(DC_HIST_THREADS), 0, st, ids, N, q, REC, flg);
  hipLaunchKernelGGL((k_dec_sweep<NB, DC_ITER>), dim3(C, T_m), dim3(DC_SWEEP_THREADS), 0, st, ids, NR,
                     N, (const int32_t*)REC, flg, L, PART, LCNT, LIST);
  hipLaunchKernelGGL((k_dec_finish<NB>), dim3(T_m), dim3(DC_FIN_THREADS), 0, st, M, NR, N, C, q,
                     (const int32_t*)REC, (const int32_t*)flg, L, (const double*)PART,
                     (const int32_t*)LCNT, (const uint32_t*)LIST, EW, CNT, NV);
}

#define INST(NB)                                                                              \
  template void launch_deciles_chunked<NB>(int, hipStream_t, const double*, const double*,     \
                                           int64_t, const QTab&, int8_t*, double*, int32_t*,    \
                                           int32_t*, const uint16_t*, int32_t*, void*);
INST(2)
INST(3)
INST(4)
INST(5)
INST(10)
#undef INST
