// portfolio.hip -- portfolio accounting beyond the reference's K = 1 equal-weight case
// (rules E1..E6 in oracle/portfolio_oracle.py and DESIGN.md 8).
//
//   k_cohort       one workgroup per (asset chunk c, holding month t, panel b[, cohort k]):
//                  decile partial sums of w * next_ret and w over the chunk's members of the
//                  cohort formed at t - k whose next_ret[t] is valid (E1), plus the chunk's
//                  formation totals of the two legs (k = 0)
//   k_turnover     one workgroup per (asset chunk, t, b): aggregate leg weights of the K
//                  overlapping cohorts at t and t - 1, |dw| summed into turnover and into the
//                  spread + square-root-impact cost of src/execution_models.py:4-12 (E4, E5)
//   k_overlap      one thread per (K, t, b, decile): chunk partials summed in chunk order,
//                  cohort means -> overlapped decile returns (E2), turnover / cost totals
//   k_ls           64 panels per workgroup: the reference's long-short rule
//                  (run_demo.py:60-67) per panel (E3), net = long-short - cost
//
// Chunking: narrow panels (few (t, b) rows) split each row over asset chunks, and wide ones
// run one chunk, so every launch has thousands of workgroups; partial sums go to a workspace
// and are combined in a fixed order.
//   k_bootstrap_*  stationary month bootstrap with a counter-based splitmix64 stream (E6)
//
// Panels are batched as [T_m][B][N] rows (B cross-sections per month), the sweep layout.
// Everything is HBM/latency-bound integer + fp64 work (no MFMA).  Reductions are per-lane
// fp64 partial sums combined by a fixed shuffle tree and then in wave order, so results are
// deterministic run to run.
#include "csm_common.h"

#include <string.h>

#include <algorithm>

#define PF_THREADS 256
#define PF_WAVES (PF_THREADS / 64)
#define PF_CHUNK_MIN 256     // assets per chunk, at least one per thread
#define PF_PLAN_MIN_B 4      // chunk plans of smaller batches are those of 4 panels (pf_plan)
#define TO_MAXK 240

__device__ __forceinline__ double wave_sum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}
__device__ __forceinline__ int wave_sumi(int v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}

// member weight of a cell with label `lab` for decile d (0 if not a member)
__device__ __forceinline__ double member_w(int lab, int d, const double* W, int64_t o) {
  if (lab != d) return 0.0;
  if (!W) return 1.0;
  const double w = W[o];
  return (w > 0.0 && w < INFINITY) ? w : 0.0;  // NaN fails w > 0
}

// Row addressing of a batch's input panels.  The B = G * Bg panels of a batch (row tb = t * B + b
// of every workspace and output array) may hold their labels / next_ret group-major,
// [G][T_m][Bg][N] -- G look-backs' label panels one block each, as the joined sweep's decile pass
// writes them (no side-by-side copy) -- and their weights / ADV / vol once for all the groups,
// [T_m][Bg][N] (no per-group copies).  The plain layout, [T_m][B][N] for both, is G = 1.
struct PanAddr {
  int B, Bg;        // panels of the batch, panels per group
  int64_t N;
  int64_t gl, ml;   // labels / next_ret: group stride, month stride (cells)
  int64_t mw;       // weights / ADV / vol: month stride (one block for every group)
  int64_t ngl;      // next_ret: group stride (gl, or 0: one next_ret block for every group)
  __host__ __device__ int64_t lrow(int t, int b) const {
    const int g = b / Bg;
    return (int64_t)g * gl + (int64_t)t * ml + (int64_t)(b - g * Bg) * N;
  }
  __host__ __device__ int64_t nrow(int t, int b) const {
    const int g = b / Bg;
    return (int64_t)g * ngl + (int64_t)t * ml + (int64_t)(b - g * Bg) * N;
  }
  __host__ __device__ int64_t wrow(int t, int b) const {
    const int g = b / Bg;
    return (int64_t)t * mw + (int64_t)(b - g * Bg) * N;
  }
};
static PanAddr pan_plain(int B, int64_t N) {
  return PanAddr{B, B, N, 0, (int64_t)B * N, (int64_t)B * N, 0};
}
static PanAddr pan_grouped(int G, int Bg, int T_m, int64_t N, bool shared_nr = false) {
  const int64_t gl = (int64_t)T_m * Bg * N;
  return PanAddr{G * Bg, Bg, N, gl, (int64_t)Bg * N, (int64_t)Bg * N, shared_nr ? 0 : gl};
}

// -------------------------------------------------------------------------------- E1
// Cohort sums do not depend on the holding period: a pass with Kmax cohorts serves every
// K <= Kmax (the sweep runs one pass per J for all its K).  Per-lane decile accumulators
// live in registers (predicated adds; SW > 0 doubles as "the cohort has a valid member",
// weights being > 0, so no count is kept).
template <int NB, bool VW>
__global__ __launch_bounds__(PF_THREADS) void k_cohort(
    const int8_t* __restrict__ L, const double* __restrict__ NR, const double* __restrict__ W,
    int T_m, int B, int64_t N, int K, int C, int64_t CH, int kpar, double* __restrict__ SWRp,
    double* __restrict__ SWp, double* __restrict__ FWp, PanAddr pa) {
  __shared__ double red[PF_WAVES][2 * NB + 2];
  const int c = (int)(blockIdx.x % (unsigned)C);
  const int tb = (int)(blockIdx.x / (unsigned)C);
  const int t = tb / B, b = tb - t * B;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t a0 = (int64_t)c * CH;
  const int64_t a1 = a0 + CH < N ? a0 + CH : N;
  const int64_t rt = pa.nrow(t, b);   // next_ret row of month t
  const int k_lo = kpar ? (int)blockIdx.z : 0, k_hi = kpar ? k_lo + 1 : K;
  for (int k = k_lo; k < k_hi; ++k) {
    const int s = t - k;
    const int64_t ob = (((int64_t)tb * K + k) * C + c) * NB;
    if (s < 0) {
      if (tid < NB) { SWRp[ob + tid] = 0.0; SWp[ob + tid] = 0.0; }
      continue;
    }
    const int64_t rs = pa.lrow(s, b), rw = pa.wrow(s, b);
    double swr[NB], sw[NB];
    uint32_t cnt[NB];   // equal weight: the weight sum is a count
#pragma unroll
    for (int d = 0; d < NB; ++d) { swr[d] = 0.0; sw[d] = 0.0; cnt[d] = 0; }
    double ft = 0.0, fb = 0.0;
    // CU cells per lane per trip, all loads issued before the first use (memory-level
    // parallelism; a one-cell loop waits out a full memory round trip per cell)
    constexpr int CU = 8;
    for (int64_t i0 = a0 + tid; i0 < a1; i0 += CU * PF_THREADS) {
      int lab[CU];
      double r[CU], wx[CU];
#pragma unroll
      for (int u = 0; u < CU; ++u) {
        const int64_t i = i0 + (int64_t)u * PF_THREADS;
        const bool in = i < a1;
        lab[u] = in ? (int)L[rs + i] : -1;
        r[u] = in ? NR[rt + i] : 0.0;
        if (VW) wx[u] = in ? W[rw + i] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < CU; ++u) {
        double w = 1.0;
        if (VW) w = (wx[u] > 0.0 && wx[u] < INFINITY) ? wx[u] : 0.0;   // invalid: not a member
        if (k == 0) {
          ft += lab[u] == NB - 1 ? w : 0.0;
          fb += lab[u] == 0 ? w : 0.0;
        }
        // a cell with no valid return (or weight) joins no decile sum; the one-hot factor
        // hd in {0, 1} makes each decile one select + one fma: fma(1, x, s) rounds exactly
        // like s + x and fma(0, x, s) == s, so the sums equal plain conditional adds
        const bool ok = r[u] == r[u] && (!VW || w > 0.0);
        const int lb = ok ? lab[u] : -1;
        const double wr = ok ? (VW ? w * r[u] : r[u]) : 0.0;   // fma(0, NaN, s) would be NaN
#pragma unroll
        for (int d = 0; d < NB; ++d) {
          const bool h = lb == d;
          const double hd = h ? 1.0 : 0.0;
          swr[d] = fma(hd, wr, swr[d]);
          if (VW) sw[d] = fma(hd, w, sw[d]);
          else cnt[d] += h ? 1u : 0u;
        }
      }
    }
#pragma unroll
    for (int d = 0; d < NB; ++d) {
      const double x = wave_sum(swr[d]), y = wave_sum(VW ? sw[d] : (double)cnt[d]);
      if (lane == 0) { red[wid][d] = x; red[wid][NB + d] = y; }
    }
    if (k == 0) {
      const double x = wave_sum(ft), y = wave_sum(fb);
      if (lane == 0) { red[wid][2 * NB] = x; red[wid][2 * NB + 1] = y; }
    }
    __syncthreads();
    if (tid < NB) {
      double x = 0.0, y = 0.0;
      for (int w2 = 0; w2 < PF_WAVES; ++w2) { x += red[w2][tid]; y += red[w2][NB + tid]; }
      SWRp[ob + tid] = x;
      SWp[ob + tid] = y;
    }
    if (k == 0 && tid < 2) {
      double x = 0.0;
      for (int w2 = 0; w2 < PF_WAVES; ++w2) x += red[w2][2 * NB + tid];
      FWp[((int64_t)tb * C + c) * 2 + tid] = x;   // leg 0 = top, 1 = bottom
    }
    __syncthreads();  // red is reused by the next cohort
  }
}

// Cohort sums with per-wave LDS accumulators: cells in the outer loop, the K cohort ages in
// the inner loop, and one LDS float atomic per (cell, age) into the wave's own [age][decile]
// slot instead of n_bins predicated fmas.  The slots are private to a wave, so only lanes of
// one instruction ever meet at an address, and the waves' slots are combined in wave order.
// Used when Kmax * n_bins fits (<= AC_MAXKD slots).
#define AC_MAXKD 384
template <int NB, bool VW>
__global__ __launch_bounds__(PF_THREADS) void k_cohort_lds(
    const int8_t* __restrict__ L, const double* __restrict__ NR, const double* __restrict__ W,
    int T_m, int B, int64_t N, int K, int C, int64_t CH, double* __restrict__ SWRp,
    double* __restrict__ SWp, double* __restrict__ FWp, PanAddr pa) {
  __shared__ double acc_r[PF_WAVES][AC_MAXKD];   // sum of w * r per (age, decile)
  __shared__ double acc_w[PF_WAVES][AC_MAXKD];   // sum of w (equal weight: the count)
  __shared__ double red[PF_WAVES][2];
  const int c = (int)(blockIdx.x % (unsigned)C);
  const int tb = (int)(blockIdx.x / (unsigned)C);
  const int t = tb / B, b = tb - t * B;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int KD = K * NB;
  for (int i = lane; i < KD; i += 64) { acc_r[wid][i] = 0.0; acc_w[wid][i] = 0.0; }
  const int64_t a0 = (int64_t)c * CH;
  const int64_t a1 = a0 + CH < N ? a0 + CH : N;
  const int64_t rt = pa.lrow(t, b), rtw = pa.wrow(t, b), rtn = pa.nrow(t, b);
  const int kmax = t + 1 < K ? t + 1 : K;   // ages with a formation month s = t - k >= 0
  double ft = 0.0, fb = 0.0;
  double* ar = acc_r[wid];
  double* aw = acc_w[wid];
  __syncthreads();
  const int64_t rowstep = pa.ml, rowstepw = pa.mw;   // one month back
  for (int64_t a = a0 + tid; a < a1; a += PF_THREADS) {
    const double r = NR[rtn + a];
    const bool rv = r == r;
    // ages in groups of KU: the group's label (and weight) loads are issued before use
    constexpr int KU = 4;
    for (int k0 = 0; k0 < kmax; k0 += KU) {
      int lab[KU];
      double wx[KU];
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        const int k = k0 + u;
        const int64_t o = rt - (int64_t)k * rowstep + a;
        lab[u] = k < kmax ? (int)L[o] : -1;
        if (VW) wx[u] = k < kmax ? W[rtw - (int64_t)k * rowstepw + a] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        const int k = k0 + u;
        double w = 1.0;
        if (VW) w = (wx[u] > 0.0 && wx[u] < INFINITY) ? wx[u] : 0.0;
        if (k == 0) {
          ft += lab[u] == NB - 1 ? w : 0.0;
          fb += lab[u] == 0 ? w : 0.0;
        }
        if (lab[u] >= 0 && rv && (!VW || w > 0.0)) {
          const int slot = k * NB + lab[u];
          atomicAdd(ar + slot, VW ? w * r : r);
          atomicAdd(aw + slot, w);
        }
      }
    }
  }
  const double x1 = wave_sum(ft), y1 = wave_sum(fb);
  if (lane == 0) { red[wid][0] = x1; red[wid][1] = y1; }
  __syncthreads();
  for (int i = tid; i < K * NB; i += PF_THREADS) {
    const int k = i / NB, d = i - k * NB;
    double x = 0.0, y = 0.0;
    for (int w2 = 0; w2 < PF_WAVES; ++w2) { x += acc_r[w2][i]; y += acc_w[w2][i]; }
    const int64_t ob = (((int64_t)tb * K + k) * C + c) * NB + d;
    SWRp[ob] = k < kmax ? x : 0.0;
    SWp[ob] = k < kmax ? y : 0.0;
  }
  if (tid < 2) {
    double x = 0.0;
    for (int w2 = 0; w2 < PF_WAVES; ++w2) x += red[w2][tid];
    FWp[((int64_t)tb * C + c) * 2 + tid] = x;
  }
}

// Cohort sums from label-sorted formation rows.  k_label_sort turns each formation row (s, b)
// into a stable counting sort of its members by decile (asset ids as uint16, segment offsets,
// and for value weights the sanitised weights in the same order), plus the row's formation
// leg totals.  k_cohort_seg then holds the return row of month t in LDS and, per (age k,
// decile d) segment of the row formed at t - k, gathers the members' returns: no per-decile
// selects and no atomics, one LDS read per (cell, age).  A row's sort is read by the K months
// that hold it (from L2 / MALL).  Chunks split every segment by position, and the partials are
// combined in chunk order like the other cohort kernels'.  Used for N <= SEG_MAXN.
// id rows are padded: every segment starts on a 4-id (8-byte) boundary and its last word is
// filled with the sentinel id N (LDS slot N of the staged return row holds NaN, so a sentinel
// contributes nothing): the gather loop needs no per-element bounds test.  Row stride:
__host__ __device__ __forceinline__ int64_t seg_stride(int64_t N) { return ((N + 3) & ~3LL) + 128; }
#define SEG_MAXN 7168   // VW sort stages 9 bytes per cell in LDS: <= 64 KB per workgroup
// LEGS: only the two legs (deciles 0 and NB - 1) are sorted -- the sweeps' long-short needs
// nothing else -- the other deciles get empty segments.
template <int NB, bool VW, bool LEGS = false>
__global__ __launch_bounds__(PF_THREADS) void k_label_sort(
    const int8_t* __restrict__ L, const double* __restrict__ W, int64_t N, int C,
    uint16_t* __restrict__ PERM, int32_t* __restrict__ OFF, double* __restrict__ WSRT,
    double* __restrict__ FWp, PanAddr pa) {
  auto is_leg = [](int d) { return !LEGS || d == 0 || d == NB - 1; };
  const int64_t PS = seg_stride(N);
  // the row is staged in LDS first (all loads in flight at once), then both passes read LDS
  extern __shared__ double wl[];                  // VW: weights [N], then labels [N]
  int8_t* ll = VW ? (int8_t*)(wl + N) : (int8_t*)wl;
  __shared__ int cnts[PF_WAVES][NB];
  __shared__ double red[PF_WAVES][2];
  const int64_t row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int rt = (int)(row / pa.B), rb = (int)(row - (int64_t)rt * pa.B);
  const int8_t* Lr = L + pa.lrow(rt, rb);
  const double* Wr = VW ? W + pa.wrow(rt, rb) : nullptr;
  if (!VW && (N & 3) == 0) {   // 4-byte aligned rows: word loads
    const uint32_t* L4 = (const uint32_t*)Lr;
    uint32_t* l4 = (uint32_t*)ll;
    const int nw = (int)(N >> 2);
#pragma unroll 4
    for (int i = tid; i < nw; i += PF_THREADS) l4[i] = L4[i];
  } else {
#pragma unroll 4
    for (int a = tid; a < (int)N; a += PF_THREADS) {
      int lab = (int)Lr[a];
      if (VW) {
        const double w = Wr[a];
        wl[a] = w;
        if (!(w > 0.0 && w < INFINITY)) lab = -1;   // no valid weight: not a member
      }
      ll[a] = (int8_t)lab;
    }
  }
  __syncthreads();
  const int64_t Q = ((N + PF_WAVES - 1) / PF_WAVES + 63) / 64 * 64;   // wave quarter, whole tiles
  const int64_t q0 = wid * Q, q1 = q0 + Q < N ? q0 + Q : N;
  int cnt[NB];
#pragma unroll
  for (int d = 0; d < NB; ++d) cnt[d] = 0;
  for (int64_t a0 = q0; a0 < q1; a0 += 64) {
    const int64_t a = a0 + lane;
    const int lab = a < q1 ? (int)ll[a] : -1;
#pragma unroll
    for (int d = 0; d < NB; ++d)
      if (is_leg(d)) cnt[d] += __popcll(__ballot(lab == d));
  }
  if (lane == 0) {
#pragma unroll
    for (int d = 0; d < NB; ++d) cnts[wid][d] = cnt[d];
  }
  __syncthreads();
  int base[NB];
  int run = 0;
#pragma unroll
  for (int d = 0; d < NB; ++d) {
    int before = 0, tot = 0;
    for (int w2 = 0; w2 < PF_WAVES; ++w2) {
      const int v = cnts[w2][d];
      before += w2 < wid ? v : 0;
      tot += v;
    }
    base[d] = run + before;
    if (tid == 0) OFF[row * (NB + 1) + d] = run;
    const int r4 = (tot + 3) & ~3;
    if (tid == d)   // sentinel ids in the segment's last word
      for (int p = run + tot; p < run + r4; ++p) {
        PERM[row * PS + p] = (uint16_t)N;
        if (VW) WSRT[row * PS + p] = 0.0;
      }
    run += r4;
  }
  if (tid == 0) OFF[row * (NB + 1) + NB] = run;
  // pass 2: a lane's rank among the lanes of its tile with the same label from bit-sliced
  // ballots (one per label bit, not one per label); the running segment positions live in
  // this wave's LDS row, bumped by the last lane of each label group
  __shared__ int wbase[PF_WAVES][NB];
  if (lane == 0) {
#pragma unroll
    for (int d = 0; d < NB; ++d) wbase[wid][d] = base[d];
  }
  constexpr int NBITS = NB <= 2 ? 1 : NB <= 4 ? 2 : NB <= 8 ? 3 : NB <= 16 ? 4 : 5;
  const uint64_t lt = (1ull << lane) - 1ull;
  double ft = 0.0, fb = 0.0;
  for (int64_t a0 = q0; a0 < q1; a0 += 64) {
    const int64_t a = a0 + lane;
    int lab = a < q1 ? (int)ll[a] : -1;
    if (LEGS && !is_leg(lab)) lab = -1;
    uint64_t same;
    if (LEGS) {   // two labels: one ballot each
      const uint64_t m0 = __ballot(lab == 0), m1 = __ballot(lab == NB - 1);
      same = lab == 0 ? m0 : m1;
    } else {
      same = __ballot(lab >= 0);
#pragma unroll
      for (int bb = 0; bb < NBITS; ++bb) {
        const bool bit = (lab >> bb) & 1;
        const uint64_t m = __ballot(bit);
        same &= bit ? m : ~m;
      }
    }
    int pos = -1;
    if (lab >= 0) {
      const int r = __popcll(same & lt);
      const int b0 = wbase[wid][lab];
      pos = b0 + r;
      if (r == __popcll(same) - 1) wbase[wid][lab] = b0 + r + 1;   // last of its group
    }
    if (pos >= 0) {
      PERM[row * PS + pos] = (uint16_t)a;
      if (VW) {
        const double w = wl[a];
        WSRT[row * PS + pos] = w;
        ft += lab == NB - 1 ? w : 0.0;
        fb += lab == 0 ? w : 0.0;
      }
    }
  }
  if (VW) {
    const double x = wave_sum(ft), y = wave_sum(fb);
    if (lane == 0) { red[wid][0] = x; red[wid][1] = y; }
    __syncthreads();
  }
  for (int i = tid; i < 2 * C; i += PF_THREADS) {   // leg totals in chunk 0, zeros elsewhere
    const int c = i >> 1, leg = i & 1;
    double v = 0.0;
    if (c == 0) {
      if (VW) {
        for (int w2 = 0; w2 < PF_WAVES; ++w2) v += red[w2][leg];
      } else {
        const int d = leg == 0 ? NB - 1 : 0;
        for (int w2 = 0; w2 < PF_WAVES; ++w2) v += (double)cnts[w2][d];
      }
    }
    FWp[(row * C + c) * 2 + leg] = v;
  }
}

// Legs-only label sort for equal weights, ONE WAVE PER FORMATION ROW (4 rows per workgroup, no
// block barriers): 4-label words per lane, leg counts by SWAR byte compares, then ranks from
// one ballot per byte lane and leg -- the same ascending-asset segments, sentinels, offsets and
// leg totals as k_label_sort<NB, false, true>, so every later sum is bit-identical.  N % 4 == 0.
__device__ __forceinline__ uint32_t byte_eq0(uint32_t z) {   // 0x80 in each byte of z that is 0
  return ~(((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z) & 0x80808080u;
}
// LM (nullable): the row's leg bitplanes [rows][2][nwm] uint64, nwm = 4 ceil(N / 256) -- plane 0
// the top decile (NB - 1), plane 1 decile 0 -- for the steady equal-weight turnover rows
// (k_turnover_ew_mask): the ballots themselves, word 4 g + e holding cell 4 (64 g + l) + e at
// bit l (a fixed order of each 256-cell group, the same in every row; the counts it serves do
// not depend on the order).
// LSO: prefix ranks by v_mbcnt (fewer VALU operations per label word than the popcount of the
// masked ballot; the same values)
// LS_STAGE: a row whose two legs hold at most LS_CAP ids (sentinels included) builds its segment
// in the wave's LDS slice and stores it once, as 8-byte words of consecutive positions, instead
// of each lane storing its own 2-byte ids a few positions apart (those stores were 280 of 1020
// us per C5 batch, -DLS_NOSTORE timing); larger rows store directly.  The same ids at the same
// positions.
#ifndef LS_STAGE
#define LS_STAGE 1
#endif
#define LS_CAP 2048
template <int NB, bool LSO = false>
__global__ __launch_bounds__(PF_THREADS) void k_label_sort_legs_ew(
    const int8_t* __restrict__ L, int64_t N, int C, int64_t rows, uint16_t* __restrict__ PERM,
    int32_t* __restrict__ OFF, double* __restrict__ FWp, PanAddr pa,
    uint64_t* __restrict__ LM = nullptr, int64_t nwm = 0) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * PF_WAVES + (threadIdx.x >> 6);
  if (row >= rows) return;   // no barriers below
  const int64_t PS = seg_stride(N);
  const int rt0 = (int)(row / pa.B);
  const uint32_t* L4 =
      reinterpret_cast<const uint32_t*>(L + pa.lrow(rt0, (int)(row - (int64_t)rt0 * pa.B)));
  const int nw = (int)(N >> 2);
  const uint32_t topw = (uint32_t)(NB - 1) * 0x01010101u;
  const uint64_t lt = (1ull << lane) - 1ull;
  // the whole row in registers (N <= SEG_MAXN: at most LS_RW words per lane), every load in
  // flight at once, read once for both passes
  constexpr int LS_RW = (SEG_MAXN / 4 + 63) / 64;
  uint32_t vr[LS_RW];
#pragma unroll
  for (int k = 0; k < LS_RW; ++k) {
    const int wi = k * 64 + lane;
    vr[k] = wi < nw ? L4[wi] : 0xFFFFFFFFu;
  }
  // (held in registers for the second pass: without this the compiler re-issues the label
  // loads there -- a second read of the row -- to save registers)
#pragma unroll
  for (int k = 0; k < LS_RW; ++k) asm volatile("" : "+v"(vr[k]));
  int nb0 = 0, nt0 = 0;   // per-lane counts: bottom (decile 0), top (decile NB - 1)
#pragma unroll
  for (int k = 0; k < LS_RW; ++k) {
    nb0 += __popc(byte_eq0(vr[k]));
    nt0 += __popc(byte_eq0(vr[k] ^ topw));
  }
  for (int o = 32; o > 0; o >>= 1) { nb0 += __shfl_xor(nb0, o, 64); nt0 += __shfl_xor(nt0, o, 64); }
  const int rb = (nb0 + 3) & ~3, rt = (nt0 + 3) & ~3;
  uint16_t* Pr = PERM + row * PS;
  if (lane <= NB) OFF[row * (NB + 1) + lane] = lane == 0 ? 0 : (lane < NB ? rb : rb + rt);
#if LS_STAGE
  __shared__ __attribute__((aligned(16))) uint16_t stg[PF_WAVES][LS_CAP];
  uint16_t* sp = stg[threadIdx.x >> 6];
  const bool staged = rb + rt <= LS_CAP;   // (wave-uniform)
  if (staged) {
    if (lane < rb - nb0) sp[nb0 + lane] = (uint16_t)N;               // sentinel ids
    if (lane < rt - nt0) sp[rb + nt0 + lane] = (uint16_t)N;
  } else {
    if (lane < rb - nb0) Pr[nb0 + lane] = (uint16_t)N;
    if (lane < rt - nt0) Pr[rb + nt0 + lane] = (uint16_t)N;
  }
#else
  if (lane < rb - nb0) Pr[nb0 + lane] = (uint16_t)N;               // sentinel ids
  if (lane < rt - nt0) Pr[rb + nt0 + lane] = (uint16_t)N;
#endif
  for (int i = lane; i < 2 * C; i += 64) {   // leg totals in chunk 0 (leg 0 = top), zeros elsewhere
    const int c = i >> 1, leg = i & 1;
    FWp[(row * C + c) * 2 + leg] = c == 0 ? (double)(leg == 0 ? nt0 : nb0) : 0.0;
  }
  int pb = 0, pt = rb;   // next position of each leg's segment
  // plane words 4 k + e (the ballots of byte e of group k) collect in lane 4 (k % 16) + e and
  // leave as one 512-byte store per plane every 16 groups
  uint64_t pw_t = 0, pw_b = 0;
#pragma unroll
  for (int k = 0; k < LS_RW; ++k) {
    if (k * 64 >= nw) break;
    const int wi = k * 64 + lane;
    const uint32_t v = vr[k];
    const uint32_t eb = byte_eq0(v), et = byte_eq0(v ^ topw);
    int bb = pb, bt = pt;   // this lane's first position of each leg
    int totb = 0, tott = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint64_t mb = __ballot((eb >> (8 * e + 7)) & 1u), mt = __ballot((et >> (8 * e + 7)) & 1u);
      if constexpr (LSO) {   // set bits of the ballot below this lane: v_mbcnt (2 ops)
        bb += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mb, 0u));
        bt += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mt >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mt, 0u));
      } else {
        bb += __popcll(mb & lt);
        bt += __popcll(mt & lt);
      }
      totb += __popcll(mb);
      tott += __popcll(mt);
      pw_t = lane == 4 * (k & 15) + e ? mt : pw_t;
      pw_b = lane == 4 * (k & 15) + e ? mb : pw_b;
    }
    if (LM && ((k & 15) == 15 || (k + 1) * 64 >= nw)) {   // (wave-uniform)
      const int64_t w = 4 * (k & ~15) + lane;
      if (w < nwm && lane < 4 * ((k & 15) + 1)) {
        LM[(row * 2) * nwm + w] = pw_t;
        LM[(row * 2 + 1) * nwm + w] = pw_b;
      }
    }
#if LS_STAGE
    if (staged) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {   // lane-major then byte order = ascending asset id
        const uint16_t a = (uint16_t)(4 * wi + e);
        if ((eb >> (8 * e + 7)) & 1u) sp[bb++] = a;
        if ((et >> (8 * e + 7)) & 1u) sp[bt++] = a;
      }
    } else
#endif
    {
#pragma unroll
      for (int e = 0; e < 4; ++e) {   // lane-major then byte order = ascending asset id
        const uint16_t a = (uint16_t)(4 * wi + e);
        if ((eb >> (8 * e + 7)) & 1u) Pr[bb++] = a;
        if ((et >> (8 * e + 7)) & 1u) Pr[bt++] = a;
      }
    }
    pb += totb;
    pt += tott;
  }
#if LS_STAGE
  if (staged) {   // the whole segment out: 4 ids per 8-byte store, consecutive lanes
    __builtin_amdgcn_wave_barrier();
    const int nw8 = (rb + rt) >> 2;
    const uint64_t* s8 = reinterpret_cast<const uint64_t*>(sp);
    uint64_t* d8 = reinterpret_cast<uint64_t*>(Pr);
    for (int i = lane; i < nw8; i += 64) d8[i] = s8[i];
    __builtin_amdgcn_wave_barrier();
  }
#endif
}

// 16-lane groups, one (age, decile) segment per group at a time: a short reduction (4 steps)
// per segment instead of a 64-lane one, and four segments per wave instruction.  The segment
// offsets of all K formation rows are fetched into LDS with the return row, and a group reads
// its segment's ids as 8-byte words (4 ids), up to 8 words per lane in flight, so one round
// trip to L2 covers a typical segment.
#define SEG_G 16
#define SEG_MAXKD 512   // K * (n_bins + 1) offsets staged in LDS
// LEGS: the (age, leg) segments only (ND = 2 per age: deciles 0 and NB - 1); the partial
// slots of the other deciles are not written (k_overlap skips them).
#define SEG_STAGE_U 12
// SJ: the label-sorted segments of up to SEG_MAXJ look-backs J that share one next_ret panel
// (the bootstrap sweep's shared next_ret, csm_boot_scan): the month's return row is staged once
// and the segments of every J walked from it -- one read of next_ret instead of one per J.  Each
// J's sums come out bit for bit as from its own launch (same segments, groups and order).
#define SEG_MAXJ 4
struct SegJ {
  const uint16_t* PERM[SEG_MAXJ];
  const int32_t* OFF[SEG_MAXJ];
  double* SWR[SEG_MAXJ];
  double* SW[SEG_MAXJ];
  int n;
};
#ifndef SEG_PANEL_MAJOR
#define SEG_PANEL_MAJOR 1
#endif
template <int NB, bool VW, bool LEGS = false>
__global__ __launch_bounds__(PF_THREADS) void k_cohort_seg(
    const double* __restrict__ NR, SegJ sj, const double* __restrict__ WSRT, int T_m, int B,
    int64_t N, int K, int C, int Cs, int xcd, int stage2, PanAddr pa, int Bo) {
  constexpr int ND = LEGS ? 2 : NB;   // segments per age
  auto dec_of = [](int e) { return LEGS ? (e ? NB - 1 : 0) : e; };
  // LEGS: the partials in the two-leg layout [rows][K][C][2] (leg 0 = decile 0, leg 1 = decile
  // NB - 1): the accounting reads 2 of every 2 values, not 2 of every NB, and the leg partials
  // of a (row, age) are one 16-B pair instead of two stores NB * 8 B apart
  constexpr int SW_W = LEGS ? 2 : NB;   // partials per (row, age, chunk)
  // the return row of month t (N values), NaN at slot N
  extern __shared__ __attribute__((aligned(16))) double rl[];
  // then each J's K * (NB + 1) segment offsets, in the same dynamic allocation: sized to the
  // launch, so a 5k-asset row's workgroup needs 40.5 KB and four fit a CU (a fixed 2 KB table
  // made 3)
  // (LEGS: only the two legs' segment bounds, as u16 -- offsets are row positions <= SEG_MAXN:
  // four per age, so four J's tables still leave four 5k-asset workgroups per CU)
  typedef typename std::conditional<LEGS, uint16_t, int32_t>::type OffT;
  constexpr int OE = LEGS ? 4 : NB + 1;   // offsets per age
  OffT* offs_all = reinterpret_cast<OffT*>(rl + N + 1);
  int c = 0;
  int64_t tb;
  int t;
  if (xcd) {   // C == 1
    // XCD-aware order: workgroups go round-robin to the 8 XCDs, so workgroup id -> (t, b)
    // keeps panel b on XCD b % 8.  SEG_PANEL_MAJOR (default): an XCD's workgroups take one
    // panel's months in order, then its next panel, so the K formation rows (member ids) a
    // month re-reads were read by the months just before it, in that XCD's L2 (else: the
    // XCD's panels for one month, then the next month -- the L2 then also holds the return
    // rows of ~Bx other panels between two uses of a formation row).
    const int id = (int)blockIdx.x, x = id & 7, j = id >> 3;
    const int Bx = (B + 7) >> 3;
#if SEG_PANEL_MAJOR
    const int bj = j / T_m;
    t = j - bj * T_m;
    const int b = x + 8 * bj;
#else
    t = j / Bx;
    const int b = x + 8 * (j - t * Bx);
#endif
    if (b >= B || t >= T_m || j >= Bx * T_m) return;
    tb = (int64_t)t * B + b;
  } else {
    c = (int)(blockIdx.x % (unsigned)C);
    tb = blockIdx.x / (unsigned)C;
    t = (int)(tb / B);
  }
  const int tid = threadIdx.x;
  const int grp = tid / SEG_G, sl = tid % SEG_G;
  const int kmax = t + 1 < K ? t + 1 : K;
  // the segment rows and cohort partials of panel b: row t * Bo + b of the workspace (Bo = B;
  // the shared-return grouped pass: Bo = nJ * B, J q's panels at rows q * B + b via sj's bases)
  const int64_t tbo = (int64_t)t * Bo + (tb - (int64_t)t * B);
  const int KD = K * OE;
  if (c >= Cs) {   // chunks beyond the Cs working ones only hold zeros
    for (int jq = 0; jq < sj.n; ++jq)
      for (int g = tid; g < K * ND; g += PF_THREADS) {
        const int k = g / ND, e = g - k * ND;
        const int64_t ob = ((tbo * K + k) * C + c) * SW_W + (LEGS ? e : dec_of(e));
        sj.SWR[jq][ob] = 0.0;
        sj.SW[jq][ob] = 0.0;
      }
    return;
  }
  const double* NRr = NR + pa.nrow(t, (int)(tb - (int64_t)t * B));
  for (int jq = 0; jq < sj.n; ++jq)
    for (int i = tid; i < kmax * OE; i += PF_THREADS) {
      const int k = i / OE, e = i - k * OE;
      const int es = LEGS ? (e < 2 ? e : NB - 3 + e) : e;   // legs: bounds 0, 1, NB - 1, NB
      offs_all[jq * KD + i] = (OffT)sj.OFF[jq][(tbo - (int64_t)k * Bo) * (NB + 1) + es];
    }
  if ((N & 1) == 0 && stage2) {
    // 16-B loads, up to SEG_STAGE_U per lane issued before any LDS store: a 6144-value row
    // in flight at once (row starts are 16-B aligned for even N)
    const int NP = (int)(N >> 1);
    const double2* src = reinterpret_cast<const double2*>(NRr);
    double2* dst = reinterpret_cast<double2*>(rl);
    for (int i0 = tid; i0 < NP; i0 += PF_THREADS * SEG_STAGE_U) {
      double2 v[SEG_STAGE_U];
#pragma unroll
      for (int u = 0; u < SEG_STAGE_U; ++u) {
        const int i = i0 + u * PF_THREADS;
        v[u] = i < NP ? src[i] : make_double2(0.0, 0.0);
      }
#pragma unroll
      for (int u = 0; u < SEG_STAGE_U; ++u) {
        const int i = i0 + u * PF_THREADS;
        if (i < NP) dst[i] = v[u];
      }
    }
  } else {
#pragma unroll 8
    for (int a = tid; a < (int)N; a += PF_THREADS) rl[a] = NRr[a];
  }
  if (tid == 0) rl[N] = qnan();
  __syncthreads();
  for (int jq = 0; jq < sj.n; ++jq) {   // every J sharing the staged row, in order
  const uint16_t* PERM = sj.PERM[jq];
  const OffT* offs = offs_all + jq * KD;
  double* __restrict__ SWRp = sj.SWR[jq];
  double* __restrict__ SWp = sj.SW[jq];
  // working chunk c < Cs owns the segments g = c (mod Cs) whole and writes zeros for the
  // others (exact under the chunk-order sum of k_overlap); each working chunk stages the
  // whole return row, so Cs stays small
  for (int g = tid; g < K * ND && Cs > 1; g += PF_THREADS) {
    if (g % Cs == c) continue;
    const int k = g / ND, e = g - k * ND;
    const int64_t ob = ((tbo * K + k) * C + c) * SW_W + (LEGS ? e : dec_of(e));
    SWRp[ob] = 0.0;
    SWp[ob] = 0.0;
  }
  const int64_t PS = seg_stride(N);
  const uint64_t SENT = (uint64_t)N * 0x0001000100010001ull;   // four sentinel ids
  const int gstep = (PF_THREADS / SEG_G) * Cs;
  // one segment: its row's id words [w0, w1), its sorted weights; zeros when its cohort is
  // not formed
  struct Seg {
    int64_t w0, w1, ob;
    const uint64_t* P8;
    const double* Ws;
    bool live;
  };
  auto seg_at = [&](int g) {
    Seg q;
    const int k = g / ND, d = dec_of(g - k * ND);
    q.ob = ((tbo * K + k) * C + c) * SW_W + (LEGS ? g - k * ND : d);
    q.live = k < kmax;
    const int64_t srow = tbo - (int64_t)(q.live ? k : 0) * Bo;
    const int oi = LEGS ? k * 4 + (d == 0 ? 0 : 2) : k * (NB + 1) + d;
    q.w0 = q.live ? (int64_t)offs[oi] >> 2 : 0;
    q.w1 = q.live ? (int64_t)offs[oi + 1] >> 2 : 0;
    q.P8 = (const uint64_t*)(PERM + srow * PS);
    q.Ws = VW ? WSRT + srow * PS : nullptr;
    return q;
  };
  constexpr int U = 8;
  // ids of one trip (U words of 4 ids per lane) of a segment, from word w on
  auto load_trip = [&](const Seg& q, int64_t w, uint64_t* v) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t x = w + u * SEG_G;
      v[u] = x < q.w1 ? q.P8[x] : SENT;
    }
  };
  auto use_trip = [&](const Seg& q, int64_t w, const uint64_t* v, double& sr, double& sw, int& n) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const double x = rl[(v[u] >> (16 * e)) & 0xffffu];
        if (x == x) {
          if (VW) {
            const double wt = q.Ws[(w + u * SEG_G) * 4 + e];
            sr += wt * x;
            sw += wt;
          } else {
            sr += x;
            ++n;
          }
        }
      }
    }
  };
  auto finish = [&](const Seg& q, double sr, double sw, int n) {
#pragma unroll
    for (int o = SEG_G / 2; o > 0; o >>= 1) {
      sr += __shfl_xor(sr, o, SEG_G);
      if (VW) sw += __shfl_xor(sw, o, SEG_G);
      else n += __shfl_xor(n, o, SEG_G);
    }
    if (sl == 0) {
      SWRp[q.ob] = q.live ? sr : 0.0;
      SWp[q.ob] = q.live ? (VW ? sw : (double)n) : 0.0;
    }
  };
  // two segments per group at a time: both segments' first trips of ids are in flight
  // together (a typical segment is one trip), then any further trips one by one
  for (int g = c + grp * Cs; g < K * ND; g += 2 * gstep) {
    const bool two = g + gstep < K * ND;
    const Seg q1 = seg_at(g), q2 = seg_at(two ? g + gstep : g);
    const int64_t a1 = q1.w0 + sl, a2 = q2.w0 + sl;
    uint64_t v1[U], v2[U];
    load_trip(q1, a1, v1);
    if (two) load_trip(q2, a2, v2);
    double sr1 = 0.0, sw1 = 0.0, sr2 = 0.0, sw2 = 0.0;
    int n1 = 0, n2 = 0;
    use_trip(q1, a1, v1, sr1, sw1, n1);
    for (int64_t w = a1 + U * SEG_G; w < q1.w1; w += U * SEG_G) {
      load_trip(q1, w, v1);
      use_trip(q1, w, v1, sr1, sw1, n1);
    }
    if (two) {
      use_trip(q2, a2, v2, sr2, sw2, n2);
      for (int64_t w = a2 + U * SEG_G; w < q2.w1; w += U * SEG_G) {
        load_trip(q2, w, v2);
        use_trip(q2, w, v2, sr2, sw2, n2);
      }
    }
    finish(q1, sr1, sw1, n1);
    if (two) finish(q2, sr2, sw2, n2);
  }
  }   // J
}

// ------------------------------------------------------------------------------ E4, E5
// w_u = (1/K_u) sum over the non-empty cohorts s in (u-K, u] of omega_s, omega_s[a] =
// W[s][a] / total_s.  When both windows of months t and t-1 are full (K non-empty cohorts
// each), w_t - w_{t-1} = (omega_t - omega_{t-K}) / K: two label reads per leg instead of 2K.
// One launch serves up to TO_MAXQ holding periods (a sweep's K values): a cell's month-t
// label / weight is loaded once and its month t-K_q ones for every q in the same trip.  The
// per-cohort inverse totals (chunk partials summed in chunk order) are staged in LDS, so the
// inner loop multiplies.
#define TO_MAXQ 4
struct KSet {
  int n;
  int K[TO_MAXQ];
};

// labels of CW consecutive cells (CW = 4: one 4-byte load, the row offset being 4-aligned)
template <int CW>
__device__ __forceinline__ void load_labels(const int8_t* __restrict__ p, int* lab) {
  if constexpr (CW == 4) {
    const uint32_t v = *(const uint32_t*)p;
#pragma unroll
    for (int e = 0; e < 4; ++e) lab[e] = (int)(int8_t)(v >> (8 * e));
  } else {
    lab[0] = (int)*p;
  }
}

__device__ __forceinline__ double valid_w(double x) { return (x > 0.0 && x < INFINITY) ? x : 0.0; }

// GEN = false: the steady rows only (every (K, leg) window full), GEN = true: the others (the
// first months, empty cohorts); two launches so the steady kernel keeps few registers.  The
// steady launch (one workgroup per (chunk, row)) appends the (chunk, row) ids it leaves to a
// work list; the general launch is a small persistent grid that walks that list (every
// workgroup reaches the list's end), so the steady rows cost it nothing.
// Per-row turnover factors for the steady equal-weight launch, computed once per row instead
// of in every workgroup's prologue (two barriers and a dependent load round each): one thread
// per row (t, b) forms, with the prologue's own arithmetic, inv_s = 1 / (leg total of the
// cohort formed at s) for s = t and s = t - K_q, sk = 1 / K_u of month t, and the telescoping
// mask (bit 2q + leg: the windows of months t and t - 1 hold as many non-empty cohorts, K_t ==
// K_{t-1} -- both full, or an empty formation month inside both -- so w_t - w_{t-1} =
// (omega_t - omega_{t-K}) / K_t: the common cohorts cancel, and only the month-t and month t-K
// labels enter, as in every steady row; month t - K must exist, t >= K).
// TPv [rows][TP_STRIDE]: per leg [inv_t, inv_{t-K_0..3}], then sk [q][leg].
#define TP_STRIDE (2 * (TO_MAXQ + 1) + 2 * TO_MAXQ)
#define TP_THREADS 64   // one thread per row: small grids, so 64-thread workgroups spread wide
#define TP_U 16          // formation months' totals loaded together (all in flight)
// TPm bit: no cohort of the row's windows has a member (a panel's first months).  Every charge
// of such a row is +0.0, so k_turn_prep writes its TURN / COST partials (0.0, the bits the
// general launch would write) and neither turnover launch takes the row.
#define TP_EMPTY 0x80000000u
__global__ __launch_bounds__(TP_THREADS) void k_turn_prep(const double* __restrict__ FWt, int T_m,
                                                          int B, KSet ks, double* __restrict__ TPv,
                                                          uint32_t* __restrict__ TPm,
                                                          int32_t* __restrict__ gen_count,
                                                          int Ct, double* __restrict__ TURNp,
                                                          double* __restrict__ COSTp) {
  const int64_t tb = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tb == 0 && gen_count) *gen_count = 0;   // the general-row work list, for the steady launch
  if (tb >= (int64_t)T_m * B) return;
  const int t = (int)(tb / B), b = (int)(tb - (int64_t)t * B);
  int kq = 0;
  for (int q = 0; q < ks.n; ++q) kq = ks.K[q] > kq ? ks.K[q] : kq;
  int k1[TO_MAXQ][2], k0[TO_MAXQ][2];
  double* tp = TPv + tb * TP_STRIDE;
#pragma unroll
  for (int q = 0; q < TO_MAXQ; ++q) k1[q][0] = k1[q][1] = k0[q][0] = k0[q][1] = 0;
  for (int j0 = 0; j0 <= kq; j0 += TP_U) {
    double fv[TP_U][2];
#pragma unroll
    for (int u = 0; u < TP_U; ++u) {
      const int s = t - (j0 + u);
      const bool ok = j0 + u <= kq && s >= 0;
#pragma unroll
      for (int li = 0; li < 2; ++li) fv[u][li] = ok ? FWt[((int64_t)s * B + b) * 2 + li] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < TP_U; ++u) {
      const int j = j0 + u;
      if (j > kq) break;
#pragma unroll
      for (int li = 0; li < 2; ++li) {
        const double tot = 0.0 + fv[u][li];
        const double v = tot > 0.0 ? 1.0 / tot : 0.0;
        if (j == 0) tp[li * (TO_MAXQ + 1)] = v;
#pragma unroll
        for (int q = 0; q < TO_MAXQ; ++q) {
          if (q >= ks.n) break;
          const int K = ks.K[q];
          if (j == K) tp[li * (TO_MAXQ + 1) + 1 + q] = v;
          k1[q][li] += (j < K && v > 0.0) ? 1 : 0;
          k0[q][li] += (j >= 1 && j <= K && t >= 1 && v > 0.0) ? 1 : 0;
        }
      }
    }
  }
  uint32_t m = 0;
#pragma unroll
  for (int q = 0; q < TO_MAXQ; ++q) {
    if (q >= ks.n) break;
    const bool has_tk = t >= ks.K[q];   // month t - K exists: the steady rows read its labels
#pragma unroll
    for (int li = 0; li < 2; ++li) {
      tp[2 * (TO_MAXQ + 1) + 2 * q + li] = k1[q][li] > 0 ? 1.0 / (double)k1[q][li] : 0.0;
      m |= (has_tk && k1[q][li] == k0[q][li]) ? (1u << (2 * q + li)) : 0u;
    }
  }
  // a member in some formation month of the windows: the windows of the longest K cover every
  // age 0..kq (month t's ages 0..K-1, month t-1's 1..K)
  bool any = false;
#pragma unroll
  for (int q = 0; q < TO_MAXQ; ++q)
    if (q < ks.n) any = any || k1[q][0] > 0 || k1[q][1] > 0 || k0[q][0] > 0 || k0[q][1] > 0;
  if (!any && TURNp) {
    m = TP_EMPTY;
    const int64_t rows = (int64_t)T_m * B;
    for (int q = 0; q < ks.n; ++q)
      for (int c = 0; c < Ct; ++c) {
        TURNp[((int64_t)q * rows + tb) * Ct + c] = 0.0;
        COSTp[((int64_t)q * rows + tb) * Ct + c] = 0.0;
      }
  }
  TPm[tb] = m;
}

// TO_GEN_TAB: the general equal-weight rows' non-full legs from per-row tables of the ages
// 0..TB-1 / 1..TB (TB = TO_GEN_TB) plus a walk over the ages >= TB, instead of a walk over every
// age (the same sums)
#ifndef TO_GEN_TAB
#define TO_GEN_TAB 1
#endif
#ifndef TO_GEN_TB
#define TO_GEN_TB 8
#endif
template <bool VW, bool IMP, bool GEN, bool BM = false>
__device__ __forceinline__ void turnover_body(
    int bid, const int8_t* __restrict__ L, const double* __restrict__ W,
    const double* __restrict__ FWp, int T_m, int B, int64_t N, KSet ks, int Kmax, int n_bins,
    int Cf, int64_t CH, int Ct, double half_spread, double k_impact, double aum,
    const double* __restrict__ ADV, const double* __restrict__ SIG, double* __restrict__ TURNp,
    double* __restrict__ COSTp, int32_t* __restrict__ gen_list, int32_t* __restrict__ gen_count,
    PanAddr pa, const double* __restrict__ TPv = nullptr,
    const uint32_t* __restrict__ TPm = nullptr) {
  const int c = bid % Ct;
  const int tb = bid / Ct;
  const int rows = T_m * B;
  const int t = tb / B, b = tb - t * B;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  __shared__ double inv[2][TO_MAXK + 1];      // [leg][j]: 1/total of cohort s = t - j (0 = empty)
  __shared__ double sk[TO_MAXQ][2][2];        // [q][leg][month t, t-1]: 1/K_u (0 if none)
  __shared__ int full[TO_MAXQ][2];
  // steady rows with k_turn_prep's factors: no prologue, the row's label (and weight) loads
  // start at once (the factors are per-row uniforms, read where they are used)
  const bool pre = !GEN && TPm != nullptr;
  if (!pre) {
  for (int j = tid; j <= Kmax; j += PF_THREADS) {
    const int s = t - j;
#pragma unroll
    for (int li = 0; li < 2; ++li) {
      double tot = 0.0;
      if (s >= 0)
        for (int cc = 0; cc < Cf; ++cc) tot += FWp[(((int64_t)s * B + b) * Cf + cc) * 2 + li];
      // (called with the folded totals, Cf = 1)
      inv[li][j] = tot > 0.0 ? 1.0 / tot : 0.0;
    }
  }
  __syncthreads();
  if (tid < 2 * ks.n) {
    const int q = tid >> 1, li = tid & 1, K = ks.K[q];
    int k1 = 0, k0 = 0;
    for (int j = 0; j < K; ++j) k1 += inv[li][j] > 0.0 ? 1 : 0;                    // month t
    for (int j = 1; j <= K; ++j) k0 += (t >= 1 && inv[li][j] > 0.0) ? 1 : 0;        // month t-1
    sk[q][li][0] = k1 > 0 ? 1.0 / (double)k1 : 0.0;
    sk[q][li][1] = k0 > 0 ? 1.0 / (double)k0 : 0.0;
    full[q][li] = (t >= K && k1 == k0) ? 1 : 0;   // telescoping (k_turn_prep's mask bit)
  }
  __syncthreads();
  }
  const int64_t a0 = (int64_t)c * CH;
  const int64_t a1 = a0 + CH < N ? a0 + CH : N;
  // labels at rt (one month back: rowstep), weights / ADV / vol at rtw (rowstepw)
  const int64_t rt = pa.lrow(t, b), rtw = pa.wrow(t, b);
  const int64_t rowstep = pa.ml, rowstepw = pa.mw;
  const int nq = ks.n;
  const int dtop = n_bins - 1;
  // Equal weight (any cost model without impact): |w_t - w_{t-1}| of a cell in a full leg is
  // inv0 (member at t only), invK (at t - K only), |inv0 - invK| (both) or 0, so a full leg's
  // turnover is three member counts.  Counts are exact integers (both legs packed in one
  // 32-bit word: a chunk holds < 65536 cells); f64 sums only for legs that are not full (the
  // first months) and for value weights.  Every path gives a (K, leg) the same value, so a
  // K's result does not depend on the other K of the set.
  constexpr bool CNT = !VW && !IMP;
  double turn[TO_MAXQ], cost[TO_MAXQ];
  uint32_t s1 = 0, s0[TO_MAXQ], sb[TO_MAXQ];   // packed counts: leg 0 (top) low half, leg 1 high
#pragma unroll
  for (int q = 0; q < TO_MAXQ; ++q) { turn[q] = 0.0; cost[q] = 0.0; s0[q] = 0; sb[q] = 0; }
  // sra = sqrt(AUM / ADV) of the cell (< 0: no ADV, spread only), once per cell: the impact of
  // a trade of dw is sqrt(dw) * sra, one square root per (q, leg) and no division (the same
  // value as sqrt(dw * AUM / ADV) to a few ulps)
  auto cell_sra = [&](double adv) { return (IMP && adv > 0.0) ? sqrt(aum / adv) : -1.0; };
  auto charge = [&](int q, double dw, double sra, double unit_sig) {
    turn[q] += dw;
    if (IMP) {
      double unit = half_spread;
      if (sra >= 0.0) {
        const double im = k_impact * unit_sig * (sqrt(dw) * sra);
        unit = unit + ((im == im) ? im : 0.0);
      }
      cost[q] += dw * unit;
    }
  };
  bool all_full = true;
  if (pre) {
    const uint32_t need = (1u << (2 * nq)) - 1u;   // bit 2q + leg
    if (TPm[tb] & TP_EMPTY) return;   // k_turn_prep wrote its partials
    all_full = (TPm[tb] & need) == need;
  } else {
    for (int q = 0; q < nq; ++q) all_full = all_full && full[q][0] && full[q][1];
  }
  if (all_full == GEN) {   // the other launch's row
    if (!GEN && gen_list && tid == 0) {   // onto its work list (capacity: one slot per workgroup
      const int slot = atomicAdd(gen_count, 1);   // of this launch; a counter that was not reset
      if (slot < rows * Ct) gen_list[slot] = bid;   // can never write past it)
    }
    return;
  }
  if (!GEN && CNT && (N & 3) == 0) {
    // steady state, 4 cells per lane per word (SWAR byte compares on the label words)
    const uint32_t topw = (uint32_t)dtop * 0x01010101u;
    auto beq = [](uint32_t z) {   // 0x80 in each byte of z that is zero
      return ~(((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z) & 0x80808080u;
    };
    // (TU = 5: a 5k-asset row's label words all in flight in one trip; counts are exact
    // integers, so the trip shape does not change a result)
    constexpr int TU = 5;
    for (int64_t a = a0 + 4 * tid; a < a1; a += 4 * TU * PF_THREADS) {
      uint32_t w1[TU], w0[TU][TO_MAXQ];
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        const int64_t x = a + (int64_t)u * 4 * PF_THREADS;
        const bool in = x < a1;
        w1[u] = in ? *(const uint32_t*)(L + rt + x) : 0xFFFFFFFFu;
#pragma unroll
        for (int q = 0; q < TO_MAXQ; ++q)
          w0[u][q] = (in && q < nq) ? *(const uint32_t*)(L + rt - (int64_t)ks.K[q] * rowstep + x)
                                    : 0xFFFFFFFFu;
      }
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        const uint32_t e1t = beq(w1[u] ^ topw), e10 = beq(w1[u]);
        s1 += __popc(e1t) + (__popc(e10) << 16);
#pragma unroll
        for (int q = 0; q < TO_MAXQ; ++q) {
          if (q >= nq) break;
          const uint32_t e0t = beq(w0[u][q] ^ topw), e00 = beq(w0[u][q]);
          s0[q] += __popc(e0t) + (__popc(e00) << 16);
          sb[q] += __popc(e1t & e0t) + (__popc(e10 & e00) << 16);
        }
      }
    }
  } else if (!GEN) {
    // steady state (value weights or impact costs): w_t - w_{t-1} needs the month-t and month
    // t-K_q labels only; TU cells per lane per trip (stride PF_THREADS), all loads in flight.
    // The row's factors (1 / leg totals of months t and t - K_q, 1 / K_u) from k_turn_prep
    // (row-uniform loads) or the prologue's LDS tables -- the same values.
    double f1[2], f0[TO_MAXQ][2], fs[TO_MAXQ][2];
    {
      const double* tp = pre ? TPv + (int64_t)tb * TP_STRIDE : nullptr;
#pragma unroll
      for (int li = 0; li < 2; ++li) {
        f1[li] = pre ? tp[li * (TO_MAXQ + 1)] : inv[li][0];
#pragma unroll
        for (int q = 0; q < TO_MAXQ; ++q) {
          const bool on = q < nq;
          f0[q][li] = !on ? 0.0 : pre ? tp[li * (TO_MAXQ + 1) + 1 + q] : inv[li][ks.K[q]];
          fs[q][li] = !on ? 0.0 : pre ? tp[2 * (TO_MAXQ + 1) + 2 * q + li] : sk[q][li][0];
        }
      }
    }
    constexpr int TU = 2;
    for (int64_t i0 = a0 + tid; i0 < a1; i0 += TU * PF_THREADS) {
      int l1[TU], l0[TU][TO_MAXQ];
      double x1[TU], x0[TU][TO_MAXQ], adv[TU], sg[TU];
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        const int64_t a = i0 + (int64_t)u * PF_THREADS;
        const bool in = a < a1;
        l1[u] = in ? (int)L[rt + a] : -1;
        x1[u] = (VW && in) ? W[rtw + a] : 1.0;
#pragma unroll
        for (int q = 0; q < TO_MAXQ; ++q) {
          const bool use = in && q < nq;
          const int64_t kq = use ? (int64_t)ks.K[q] : 0;
          l0[u][q] = use ? (int)L[rt - kq * rowstep + a] : -1;
          x0[u][q] = (VW && use) ? W[rtw - kq * rowstepw + a] : 1.0;
        }
        adv[u] = (IMP && in) ? ADV[rtw + a] : 0.0;
        sg[u] = (IMP && SIG && in) ? SIG[rtw + a] : 0.02;
      }
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        const double vw1 = VW ? valid_w(x1[u]) : 1.0;
        const double unit_sig = sg[u] == sg[u] ? sg[u] : 0.02;
        const double sra = cell_sra(adv[u]);
#pragma unroll
        for (int q = 0; q < TO_MAXQ; ++q) {
          if (q >= nq) break;
          const double vw0 = VW ? valid_w(x0[u][q]) : 1.0;
#pragma unroll
          for (int li = 0; li < 2; ++li) {
            const int d = li == 0 ? dtop : 0;
            const double w1 = (l1[u] == d ? vw1 : 0.0) * f1[li];
            const double w0 = (l0[u][q] == d ? vw0 : 0.0) * f0[q][li];
            charge(q, fabs(w1 - w0) * fs[q][li], sra, unit_sig);
          }
        }
      }
    }
  } else if (GEN) {
    // general rows: one pass over the ages j <= max K_q per cell, the age loads unrolled so
    // they are in flight together; w_t and w_{t-1} sums for every (q, leg) at once.  Cells go
    // to lanes as in the steady paths (4 consecutive per lane when N % 4 == 0), so a row's
    // sums have the same order whichever path it takes.
    int kq = 0;
    for (int q = 0; q < nq; ++q) kq = ks.K[q] > kq ? ks.K[q] : kq;
    const int cw = (CNT && (N & 3) == 0) ? 4 : 1;   // the steady paths' cells per lane
    const int jmax = kq < t ? kq : t;   // ages with a formation month s = t - j >= 0
    if (CNT && kq <= 31) {
      // equal weight: a cell's leg memberships over the ages are two bit masks; the sums of
      // inverse totals take the member ages only (ascending age, the same order and values as
      // the dense loop below)
      const uint32_t topw = (uint32_t)dtop * 0x01010101u;
      auto beq = [](uint32_t z) { return ~(((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z) & 0x80808080u; };
      // ages whose cohort is empty on both legs contribute nothing (their bits add inv 0.0,
      // and a leg with an empty age in either window is not full, so its counts are unused):
      // their label loads are skipped (the first months of a panel: most ages are empty)
      uint32_t amask = 0;
      for (int j = 0; j <= jmax; ++j) amask |= (inv[0][j] != 0.0 || inv[1][j] != 0.0) ? 1u << j : 0u;
      // the (q, leg) pairs whose windows are full (counts, like the steady rows) as a row-uniform
      // bit mask, read once
      uint32_t fullm = 0;
      for (int q = 0; q < nq; ++q)
        fullm |= (full[q][0] ? 1u : 0u) << (2 * q) | (full[q][1] ? 1u : 0u) << (2 * q + 1);
      const bool anyfree = fullm != (1u << (2 * nq)) - 1u;
#if TO_GEN_TAB
      // legs that are not full take x1 / x0 from per-row tables for the ages 0..TB-1 / 1..TB
      // (each entry the ascending sum of inv over its member ages: the walk's own additions,
      // the +0.0 of a non-member age being exact for these non-negative sums), and walk only the
      // ages >= TB: pairs with K_q <= TB are charged straight from the tables
      constexpr int TB = TO_GEN_TB, TN = 1 << TO_GEN_TB;
      __shared__ double tabA[2][TN], tabZ[2][TN];
      if (anyfree) {   // (row-uniform)
        for (int i = tid; i < 4 * TN; i += PF_THREADS) {
          const int li = i / (2 * TN), z = (i / TN) & 1, m = i & (TN - 1);
          double sum = 0.0;
          for (int bb = 0; bb < TB; ++bb) {
            const int j = bb + z;   // tabA: ages 0..TB-1, tabZ: ages 1..TB
            if ((m >> bb) & 1) sum += j <= Kmax ? inv[li][j] : 0.0;
          }
          (z ? tabZ : tabA)[li][m] = sum;
        }
        __syncthreads();
      }
#endif
      for (int64_t a4 = a0 + cw * tid; a4 < a1 && amask; a4 += cw * PF_THREADS) {
        uint32_t mt4[4] = {0, 0, 0, 0}, mb4[4] = {0, 0, 0, 0};
        if (cw == 4) {
          // the 4 cells' labels of 8 ages per trip as label words, all loads in flight
          for (int j0 = 0; j0 <= jmax; j0 += 8) {
            if (!((amask >> j0) & 0xFFu)) continue;
            uint32_t wv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
              wv[u] = (j0 + u <= jmax && ((amask >> (j0 + u)) & 1u))
                          ? *(const uint32_t*)(L + rt - (int64_t)(j0 + u) * rowstep + a4)
                          : 0xFFFFFFFFu;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const uint32_t et = beq(wv[u] ^ topw) >> 7, eb = beq(wv[u]) >> 7;   // bits 0,8,16,24
              const int j = j0 + u;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                mt4[e] |= ((et >> (8 * e)) & 1u) << (j & 31);
                mb4[e] |= ((eb >> (8 * e)) & 1u) << (j & 31);
              }
            }
          }
        } else {
          for (int j = 0; j <= jmax; ++j) {
            const int lab = (int)L[rt - (int64_t)j * rowstep + a4];
            mt4[0] |= (lab == dtop ? 1u : 0u) << j;
            mb4[0] |= (lab == 0 ? 1u : 0u) << j;
          }
        }
        const int ne = (int)(a1 - a4 < cw ? a1 - a4 : cw);   // cells of this lane's group
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (e >= ne) break;
          const uint32_t mt = mt4[e], mb = mb4[e];
          const uint32_t e1 = (mt & 1u) | ((mb & 1u) << 16);
          s1 += e1;
#pragma unroll
          for (int q = 0; q < TO_MAXQ; ++q) {
            if (q >= nq) break;
            const int K = ks.K[q];
            const uint32_t e0 = ((mt >> K) & 1u) | (((mb >> K) & 1u) << 16);
            s0[q] += e0;
            sb[q] += e1 & e0;
          }
        }
#if TO_GEN_TAB
        if (anyfree) {
          // x1 of the ages 0..TB-1 and x0 of the ages 1..TB from the tables; pairs with K_q <= TB
          // charged from them, cells and legs in order (each pair's terms in the walk's order)
          double sa[4][2], sz[4][2];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            sa[e][0] = tabA[0][mt4[e] & (TN - 1u)]; sz[e][0] = tabZ[0][(mt4[e] >> 1) & (TN - 1u)];
            sa[e][1] = tabA[1][mb4[e] & (TN - 1u)]; sz[e][1] = tabZ[1][(mb4[e] >> 1) & (TN - 1u)];
          }
          uint32_t clo = 0;   // pairs (q, leg) with K_q <= TB that are not full
#pragma unroll
          for (int q = 0; q < TO_MAXQ; ++q)
            clo |= (q < nq && ks.K[q] <= TB) ? (3u << (2 * q)) & ~fullm : 0u;
          if (clo) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              if (e >= ne) break;
#pragma unroll
              for (int li = 0; li < 2; ++li) {
                const uint32_t mm = li == 0 ? mt4[e] : mb4[e];
#pragma unroll
                for (int q = 0; q < TO_MAXQ; ++q) {
                  if (!((clo >> (2 * q + li)) & 1u)) continue;
                  const uint32_t km = (1u << ks.K[q]) - 1u;
                  charge(q, fabs(tabA[li][mm & km] * sk[q][li][0] -
                                 tabZ[li][(mm >> 1) & km] * sk[q][li][1]), -1.0, 0.02);
                }
              }
            }
          }
#pragma unroll 1
          for (int j = TB; j <= kq; ++j) {
            asm volatile("" ::: "memory");   // the factors are re-read (broadcasts), not held
            const double iv0 = inv[0][j], iv1 = inv[1][j];
            uint32_t cq = 0;   // pairs with K_q == j (> TB) charged now
#pragma unroll
            for (int q = 0; q < TO_MAXQ; ++q)
              cq |= (q < nq && ks.K[q] == j && j > TB) ? (3u << (2 * q)) & ~fullm : 0u;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
#pragma unroll
              for (int li = 0; li < 2; ++li) {
                const uint32_t mm = li == 0 ? mt4[e] : mb4[e];
                const double v = ((mm >> j) & 1u) ? (li == 0 ? iv0 : iv1) : 0.0;
                if (cq && e < ne) {
#pragma unroll
                  for (int q = 0; q < TO_MAXQ; ++q)
                    if ((cq >> (2 * q + li)) & 1u)
                      charge(q, fabs(sa[e][li] * sk[q][li][0] - (sz[e][li] + v) * sk[q][li][1]),
                             -1.0, 0.02);
                }
                sa[e][li] += v;
                if (j > TB) sz[e][li] += v;   // (the table holds age TB already)
              }
            }
          }
        }
#else
        if (anyfree) {
          // legs that are not full: x1 = sum of inv over the member ages 0..K-1 (month t's
          // window), x0 over 1..K (month t-1's), both ascending.  One walk over the ages for
          // every (cell, leg) with inv read once per age (a broadcast): an age the cell is not
          // in adds 0.0, exact for these non-negative sums, so x1 / x0 are the sums over the set
          // bits in ascending order.  Pair q is charged at age K_q, cells and legs in order.
          double sa[4][2], sz[4][2];
#pragma unroll
          for (int e = 0; e < 4; ++e) { sa[e][0] = sa[e][1] = 0.0; sz[e][0] = sz[e][1] = 0.0; }
#pragma unroll 1
          for (int j = 0; j <= kq; ++j) {
            asm volatile("" ::: "memory");   // the factors are re-read (broadcasts), not held
            const double iv0 = inv[0][j], iv1 = inv[1][j];
            // pairs q with K_q == j are charged now: x1 = sa (ages < j), x0 = sz + v (ages 1..j)
            uint32_t cq = 0;
#pragma unroll
            for (int q = 0; q < TO_MAXQ; ++q)
              cq |= (q < nq && ks.K[q] == j) ? (3u << (2 * q)) & ~fullm : 0u;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
#pragma unroll
              for (int li = 0; li < 2; ++li) {
                const uint32_t mm = li == 0 ? mt4[e] : mb4[e];
                const double v = ((mm >> j) & 1u) ? (li == 0 ? iv0 : iv1) : 0.0;
                if (cq && e < ne) {
#pragma unroll
                  for (int q = 0; q < TO_MAXQ; ++q)
                    if ((cq >> (2 * q + li)) & 1u)
                      charge(q, fabs(sa[e][li] * sk[q][li][0] - (sz[e][li] + v) * sk[q][li][1]),
                             -1.0, 0.02);
                }
                sa[e][li] += v;
                if (j >= 1) sz[e][li] += v;
              }
            }
          }
        }
#endif
      }
    } else if constexpr (!BM) {
    // ages whose cohort is empty on both legs add 0.0 to every sum (inv 0.0) and make neither
    // leg full, so their loads are skipped; a row with no cohort formed yet (a panel's first
    // months) has all sums zero and skips its cells (exact: every skipped term is +0.0)
    uint64_t amask = ~0ull;
    if (jmax < 64) {
      amask = 0;
      for (int j = 0; j <= jmax; ++j)
        amask |= (inv[0][j] != 0.0 || inv[1][j] != 0.0) ? 1ull << j : 0ull;
    }
    auto live = [&](int j) { return j >= 64 || ((amask >> j) & 1ull); };
    // cell k of this lane, in the steady paths' order
    auto cell = [&](int k) -> int64_t {
      return cw == 1 ? a0 + tid + (int64_t)k * PF_THREADS
                     : a0 + 4 * tid + (int64_t)(k >> 2) * 4 * PF_THREADS + (k & 3);
    };
    // CC cells of the lane at a time, all their age loads in flight together.  Each age's
    // member weights go into running sums over ages >= 0 (sa) and >= 1 (sz): x1 of pair q is sa
    // before age K_q and x0 is sz after it -- the same ascending-age additions as one
    // accumulator per q -- so q is charged at age K_q (after the last age when K_q > jmax),
    // cell by cell: every turn[q] / cost[q] receives its terms in the same order as before.
    constexpr int CC = 2;
    for (int k = 0; amask && cell(k) < a1; k += CC) {
      int64_t ac[CC];
      bool on[CC];
      double sra[CC], usig[CC], sa[CC][2], sz[CC][2], m0[CC][2];
      int lab0[CC], labK[CC][TO_MAXQ];
#pragma unroll
      for (int c = 0; c < CC; ++c) {
        ac[c] = cell(k + c);
        on[c] = ac[c] < a1;
        sra[c] = -1.0;
        usig[c] = 0.02;
        if (IMP && on[c]) {
          sra[c] = cell_sra(ADV[rtw + ac[c]]);
          if (SIG) { const double sg = SIG[rtw + ac[c]]; usig[c] = (sg == sg) ? sg : 0.02; }
        }
        lab0[c] = -1;
#pragma unroll
        for (int li = 0; li < 2; ++li) { sa[c][li] = 0.0; sz[c][li] = 0.0; m0[c][li] = 0.0; }
#pragma unroll
        for (int q = 0; q < TO_MAXQ; ++q) labK[c][q] = -1;
      }
      for (int j0 = 0; j0 <= jmax; j0 += 8) {
        int labv[CC][8];
        double wv[CC][8];
#pragma unroll
        for (int c = 0; c < CC; ++c)
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const bool ok = on[c] && j0 + u <= jmax && live(j0 + u);
            const int64_t j = ok ? j0 + u : 0;
            labv[c][u] = ok ? (int)L[rt - j * rowstep + ac[c]] : -1;
            wv[c][u] = (VW && ok) ? W[rtw - j * rowstepw + ac[c]] : 1.0;
          }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int j = j0 + u;
          if (j > jmax) break;
          const double i0 = inv[0][j], i1 = inv[1][j];
          uint32_t cq = 0;   // pairs charged at this age
#pragma unroll
          for (int q = 0; q < TO_MAXQ; ++q) cq |= (q < nq && ks.K[q] == j) ? 1u << q : 0u;
#pragma unroll
          for (int c = 0; c < CC; ++c) {
            const int lab = labv[c][u];   // -1 for a dead age: m = 0, as if skipped
            const double w = VW ? valid_w(wv[c][u]) : 1.0;
            const double m[2] = {lab == dtop ? w * i0 : 0.0, lab == 0 ? w * i1 : 0.0};
            if (j == 0) { m0[c][0] = m[0]; m0[c][1] = m[1]; lab0[c] = lab; }
            if (cq) {
#pragma unroll
              for (int q = 0; q < TO_MAXQ; ++q) {
                if (!((cq >> q) & 1u)) continue;
                if (CNT) labK[c][q] = lab;
                if (!on[c]) continue;
#pragma unroll
                for (int li = 0; li < 2; ++li) {
                  if (full[q][li]) {
                    if (!CNT) charge(q, fabs(m0[c][li] - m[li]) * sk[q][li][0], sra[c], usig[c]);
                  } else {
                    charge(q, fabs(sa[c][li] * sk[q][li][0] - (sz[c][li] + m[li]) * sk[q][li][1]),
                           sra[c], usig[c]);
                  }
                }
              }
            }
#pragma unroll
            for (int li = 0; li < 2; ++li) {
              sa[c][li] += m[li];
              if (j >= 1) sz[c][li] += m[li];
            }
          }
        }
      }
#pragma unroll
      for (int c = 0; c < CC; ++c) {
        if (!on[c]) continue;
#pragma unroll
        for (int q = 0; q < TO_MAXQ; ++q) {   // windows reaching past the first month
          if (q >= nq) break;
          if (ks.K[q] <= jmax) continue;
#pragma unroll
          for (int li = 0; li < 2; ++li) {
            if (full[q][li]) {
              if (!CNT) charge(q, fabs(m0[c][li] - 0.0) * sk[q][li][0], sra[c], usig[c]);
            } else {
              charge(q, fabs(sa[c][li] * sk[q][li][0] - sz[c][li] * sk[q][li][1]), sra[c],
                     usig[c]);
            }
          }
        }
        if (CNT) {
          const uint32_t e1 = (lab0[c] == dtop ? 1u : 0u) | (lab0[c] == 0 ? 0x10000u : 0u);
          s1 += e1;
#pragma unroll
          for (int q = 0; q < TO_MAXQ; ++q) {
            if (q >= nq) break;
            const uint32_t e0 = (labK[c][q] == dtop ? 1u : 0u) | (labK[c][q] == 0 ? 0x10000u : 0u);
            s0[q] += e0;
            sb[q] += e1 & e0;
          }
        }
      }
    }
    }
  }
  __shared__ double red[PF_WAVES][2 * TO_MAXQ];
  __shared__ uint32_t cred[PF_WAVES][1 + 2 * TO_MAXQ];
  if (CNT) {
    const uint32_t x = (uint32_t)wave_sumi((int)s1);
    if (lane == 0) cred[wid][0] = x;
  }
#pragma unroll
  for (int q = 0; q < TO_MAXQ; ++q) {
    if (q >= nq) break;
    const double x1 = wave_sum(turn[q]);
    const double y1 = IMP ? wave_sum(cost[q]) : 0.0;
    if (lane == 0) { red[wid][2 * q] = x1; red[wid][2 * q + 1] = y1; }
    if (CNT) {
      const uint32_t x = (uint32_t)wave_sumi((int)s0[q]), y = (uint32_t)wave_sumi((int)sb[q]);
      if (lane == 0) { cred[wid][1 + 2 * q] = x; cred[wid][2 + 2 * q] = y; }
    }
  }
  __syncthreads();
  if (tid < nq) {
    const int q = tid, K = ks.K[q];
    double x = 0.0, y = 0.0;
    for (int w2 = 0; w2 < PF_WAVES; ++w2) { x += red[w2][2 * q]; y += red[w2][2 * q + 1]; }
    if (CNT) {
      uint32_t S1 = 0, S0 = 0, SB = 0;
      for (int w2 = 0; w2 < PF_WAVES; ++w2) {
        S1 += cred[w2][0];
        S0 += cred[w2][1 + 2 * q];
        SB += cred[w2][2 + 2 * q];
      }
#pragma unroll
      for (int li = 0; li < 2; ++li) {
        if (!pre && !full[q][li]) continue;   // (pre: only all-full rows get here)
        const uint32_t n1 = (S1 >> (16 * li)) & 0xFFFFu, n0 = (S0 >> (16 * li)) & 0xFFFFu,
                       nb = (SB >> (16 * li)) & 0xFFFFu;
        const double* tp = pre ? TPv + tb * TP_STRIDE : nullptr;
        const double i1 = pre ? tp[li * (TO_MAXQ + 1)] : inv[li][0];
        const double i0 = pre ? tp[li * (TO_MAXQ + 1) + 1 + q] : inv[li][K];
        const double skq = pre ? tp[2 * (TO_MAXQ + 1) + 2 * q + li] : sk[q][li][0];
        x += ((double)(n1 - nb) * i1 + (double)(n0 - nb) * i0 + (double)nb * fabs(i1 - i0)) *
             skq;
      }
    }
    TURNp[((int64_t)q * rows + tb) * Ct + c] = 0.5 * x;
    COSTp[((int64_t)q * rows + tb) * Ct + c] = IMP ? y : x * half_spread;
  }
}

// Steady equal-weight rows from the leg bitplanes k_label_sort_legs_ew wrote: ONE WAVE per
// (chunk, row), 64 cells per plane word (chunks of whole 256-cell groups: Ct == 1 or CH % 256
// == 0).  A full leg's turnover is three exact member counts
// (k_turnover's count path: members at t, at t - K_q, at both), here popcounts of plane words
// -- 10 words per 64 cells instead of 5 label bytes per cell -- and the same final arithmetic on
// the same integers, so the TURN / COST partials are k_turnover's bits.  Rows that are not all
// full go onto the general launch's work list as k_turnover's steady launch puts them.
#define TM_WAVES 4
#ifndef TM_EARLY
#define TM_EARLY 1   // the row's loads issued together (and its counts reduced packed)
#endif
__global__ __launch_bounds__(64 * TM_WAVES) void k_turnover_ew_mask(
    const uint64_t* __restrict__ LM, int64_t nwm, int T_m, int B, int64_t N, KSet ks, int64_t CH,
    int Ct, double half_spread, double* __restrict__ TURNp, double* __restrict__ COSTp,
    int32_t* __restrict__ gen_list, int32_t* __restrict__ gen_count,
    const double* __restrict__ TPv, const uint32_t* __restrict__ TPm) {
  const int lane = threadIdx.x & 63;
  const int rows = T_m * B;
  const int bid = (int)(blockIdx.x * TM_WAVES + (threadIdx.x >> 6));
  if (bid >= rows * Ct) return;   // no barriers below
  const int c = bid % Ct, tb = bid / Ct;
  const int t = tb / B, b = tb - t * B;
  const int nq = ks.n;
#if TM_EARLY
  // every load of the row at once -- its mask, its factors (lane q < nq), the plane words of
  // months t and t - K_q (addresses clamped to month 0 for the rows the mask sends elsewhere:
  // those loads are discarded) -- instead of mask -> words -> factors, three round trips
  const uint32_t m = TPm[tb];
  const int64_t w0 = (int64_t)c * CH / 64;
  const int64_t a1 = (int64_t)(c + 1) * CH < N ? (int64_t)(c + 1) * CH : N;
  const int64_t w1 = (a1 + 255) / 256 * 4;
  const uint64_t* r1 = LM + (int64_t)tb * 2 * nwm;
  const double* tp = TPv + (int64_t)tb * TP_STRIDE;
  double f1[2] = {0.0, 0.0}, f0[2] = {0.0, 0.0}, fs[2] = {0.0, 0.0};
  if (lane < nq) {
#pragma unroll
    for (int li = 0; li < 2; ++li) {
      f1[li] = tp[li * (TO_MAXQ + 1)];
      f0[li] = tp[li * (TO_MAXQ + 1) + 1 + lane];
      fs[li] = tp[2 * (TO_MAXQ + 1) + 2 * lane + li];
    }
  }
  constexpr int TMU = 2;   // word trips per lane in flight (N <= SEG_MAXN: at most 2)
  uint64_t x1[TMU][2], x0[TMU][TO_MAXQ][2];
#pragma unroll
  for (int u = 0; u < TMU; ++u) {
    const int64_t w = w0 + lane + 64 * u;
    const bool in = w < w1;
    const int64_t wi = in ? w : w0;
#pragma unroll
    for (int li = 0; li < 2; ++li) x1[u][li] = in ? r1[li * nwm + wi] : 0ull;
#pragma unroll
    for (int q = 0; q < TO_MAXQ; ++q) {
      const int tq = q < nq ? (t - ks.K[q] >= 0 ? t - ks.K[q] : 0) : 0;
      const uint64_t* r0 = LM + ((int64_t)tq * B + b) * 2 * nwm;
#pragma unroll
      for (int li = 0; li < 2; ++li) x0[u][q][li] = (in && q < nq) ? r0[li * nwm + wi] : 0ull;
    }
  }
  if (m & TP_EMPTY) return;   // k_turn_prep wrote its partials
  const uint32_t need = (1u << (2 * nq)) - 1u;
  if ((m & need) != need) {   // the general launch's row
    if (gen_list && lane == 0) {
      const int slot = atomicAdd(gen_count, 1);
      if (slot < rows * Ct) gen_list[slot] = bid;
    }
    return;
  }
  // member counts, both legs packed in one word (leg 0 low half; a chunk holds < 65536 cells)
  uint32_t n1 = 0, n0[TO_MAXQ], nb[TO_MAXQ];
#pragma unroll
  for (int q = 0; q < TO_MAXQ; ++q) { n0[q] = 0; nb[q] = 0; }
  auto count = [&](const uint64_t (&y1)[2], const uint64_t (&y0)[TO_MAXQ][2]) {
#pragma unroll
    for (int li = 0; li < 2; ++li) {
      n1 += (uint32_t)__popcll(y1[li]) << (16 * li);
#pragma unroll
      for (int q = 0; q < TO_MAXQ; ++q) {
        n0[q] += (uint32_t)__popcll(y0[q][li]) << (16 * li);
        nb[q] += (uint32_t)__popcll(y1[li] & y0[q][li]) << (16 * li);
      }
    }
  };
#pragma unroll
  for (int u = 0; u < TMU; ++u) count(x1[u], x0[u]);
  for (int64_t w = w0 + lane + 64 * TMU; w < w1; w += 64) {   // (wider chunks than SEG_MAXN)
    uint64_t y1[2], y0[TO_MAXQ][2];
#pragma unroll
    for (int li = 0; li < 2; ++li) y1[li] = r1[li * nwm + w];
#pragma unroll
    for (int q = 0; q < TO_MAXQ; ++q) {
      const uint64_t* r0 = LM + ((int64_t)(t - (q < nq ? ks.K[q] : 0)) * B + b) * 2 * nwm;
#pragma unroll
      for (int li = 0; li < 2; ++li) y0[q][li] = q < nq ? r0[li * nwm + w] : 0ull;
    }
    count(y1, y0);
  }
  auto wsum = [](uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
  };
  n1 = wsum(n1);
#pragma unroll
  for (int q = 0; q < TO_MAXQ; ++q) {
    if (q >= nq) break;
    n0[q] = wsum(n0[q]);
    nb[q] = wsum(nb[q]);
  }
  if (lane < nq) {
    const int q = lane;
    double x = 0.0;   // (k_turnover: the waves' f64 charge sums, +0.0 on an all-full row)
#pragma unroll
    for (int li = 0; li < 2; ++li) {
      uint32_t c0 = 0, cb = 0;
#pragma unroll
      for (int qq = 0; qq < TO_MAXQ; ++qq)
        if (qq == q) { c0 = (n0[qq] >> (16 * li)) & 0xFFFFu; cb = (nb[qq] >> (16 * li)) & 0xFFFFu; }
      const uint32_t c1 = (n1 >> (16 * li)) & 0xFFFFu;
      const double i1 = f1[li], i0 = f0[li], skq = fs[li];
      x += ((double)(c1 - cb) * i1 + (double)(c0 - cb) * i0 + (double)cb * fabs(i1 - i0)) * skq;
    }
    TURNp[((int64_t)q * rows + tb) * Ct + c] = 0.5 * x;
    COSTp[((int64_t)q * rows + tb) * Ct + c] = x * half_spread;
  }
#else
  const uint32_t m = TPm[tb];
  if (m & TP_EMPTY) return;   // k_turn_prep wrote its partials
  const uint32_t need = (1u << (2 * nq)) - 1u;
  if ((m & need) != need) {   // the general launch's row
    if (gen_list && lane == 0) {
      const int slot = atomicAdd(gen_count, 1);
      if (slot < rows * Ct) gen_list[slot] = bid;
    }
    return;
  }
  // chunk c's cells [c CH, min(N, (c + 1) CH)): whole 256-cell groups, 4 words each (cells past
  // N hold no member)
  const int64_t w0 = (int64_t)c * CH / 64;
  const int64_t a1 = (int64_t)(c + 1) * CH < N ? (int64_t)(c + 1) * CH : N;
  const int64_t w1 = (a1 + 255) / 256 * 4;
  const uint64_t* r1 = LM + (int64_t)tb * 2 * nwm;
  uint32_t n1[2] = {0, 0}, n0[TO_MAXQ][2], nb[TO_MAXQ][2];
#pragma unroll
  for (int q = 0; q < TO_MAXQ; ++q) n0[q][0] = n0[q][1] = nb[q][0] = nb[q][1] = 0;
  for (int64_t w = w0 + lane; w < w1; w += 64) {
    uint64_t x1[2], x0[TO_MAXQ][2];
#pragma unroll
    for (int li = 0; li < 2; ++li) x1[li] = r1[li * nwm + w];
#pragma unroll
    for (int q = 0; q < TO_MAXQ; ++q) {
      const uint64_t* r0 = LM + ((int64_t)(t - (q < nq ? ks.K[q] : 0)) * B + b) * 2 * nwm;
#pragma unroll
      for (int li = 0; li < 2; ++li) x0[q][li] = q < nq ? r0[li * nwm + w] : 0ull;
    }
#pragma unroll
    for (int li = 0; li < 2; ++li) {
      n1[li] += __popcll(x1[li]);
#pragma unroll
      for (int q = 0; q < TO_MAXQ; ++q) {
        n0[q][li] += __popcll(x0[q][li]);
        nb[q][li] += __popcll(x1[li] & x0[q][li]);
      }
    }
  }
  auto wsum = [](uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
  };
#pragma unroll
  for (int li = 0; li < 2; ++li) {
    n1[li] = wsum(n1[li]);
#pragma unroll
    for (int q = 0; q < TO_MAXQ; ++q) { n0[q][li] = wsum(n0[q][li]); nb[q][li] = wsum(nb[q][li]); }
  }
  if (lane < nq) {
    const int q = lane;
    const double* tp = TPv + (int64_t)tb * TP_STRIDE;
    double x = 0.0;   // (k_turnover: the waves' f64 charge sums, +0.0 on an all-full row)
#pragma unroll
    for (int li = 0; li < 2; ++li) {
      uint32_t c0 = 0, cb = 0;
#pragma unroll
      for (int qq = 0; qq < TO_MAXQ; ++qq)
        if (qq == q) { c0 = n0[qq][li]; cb = nb[qq][li]; }
      const double i1 = tp[li * (TO_MAXQ + 1)];
      const double i0 = tp[li * (TO_MAXQ + 1) + 1 + q];
      const double skq = tp[2 * (TO_MAXQ + 1) + 2 * q + li];
      x += ((double)(n1[li] - cb) * i1 + (double)(c0 - cb) * i0 + (double)cb * fabs(i1 - i0)) * skq;
    }
    TURNp[((int64_t)q * rows + tb) * Ct + c] = 0.5 * x;
    COSTp[((int64_t)q * rows + tb) * Ct + c] = x * half_spread;
  }
#endif
}

// Steady value-weight rows of the G = B / Bg panels that share one weight row (the grouped
// layout: G look-backs of one panel, TO_MAXG at most): one workgroup per (month t, weight panel
// p, chunk c) serves the G rows (t, g * Bg + p).  A cell's weights of months t and t - K_q and
// its ADV / vol are loaded once for all G rows, its labels per row; each row's charges go to
// its own accumulators in exactly the per-row launch's order (a lane's cells in order, then q,
// then leg), and each row is reduced by the per-row launch's tree -- its TURN / COST partials
// are the same bits.  Rows that are not all-full go onto the general launch's work list as the
// per-row launch's ids (tb * Ct + c).
#define TO_MAXG 4
#ifndef VWG_U
#define VWG_U 1   // cells per lane in flight in k_turnover_vwg (2 / 4 measured slower: C3 portfolio 0.241 -> 0.266 / 0.342 ms)
#endif
#ifndef VWG_WPE
#define VWG_WPE 1   // waves per EU the VGPR budget must allow (A/B knob)
#endif
template <bool IMP>
__global__ __launch_bounds__(PF_THREADS) __attribute__((amdgpu_waves_per_eu(VWG_WPE))) void k_turnover_vwg(
    const int8_t* __restrict__ L, const double* __restrict__ W, int T_m, int B, int64_t N,
    KSet ks, int n_bins, int64_t CH, int Ct, double half_spread, double k_impact, double aum,
    const double* __restrict__ ADV, const double* __restrict__ SIG, double* __restrict__ TURNp,
    double* __restrict__ COSTp, int32_t* __restrict__ gen_list, int32_t* __restrict__ gen_count,
    const double* __restrict__ TPv, const uint32_t* __restrict__ TPm, PanAddr pa) {
  const int Bg = pa.Bg, G = B / Bg;
  const int c = (int)(blockIdx.x % (unsigned)Ct);
  const int tp = (int)(blockIdx.x / (unsigned)Ct);
  const int t = tp / Bg, p = tp - t * Bg;
  const int rows = T_m * B;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nq = ks.n;
  const uint32_t need = (1u << (2 * nq)) - 1u;   // bit 2q + leg
  uint32_t act = 0;                              // this workgroup's steady rows (bit g)
#pragma unroll
  for (int g = 0; g < TO_MAXG; ++g) {
    if (g >= G) break;
    const int tb = t * B + g * Bg + p;
    const uint32_t m = TPm[tb];
    if (m & TP_EMPTY) continue;   // k_turn_prep wrote its partials
    if ((m & need) == need) act |= 1u << g;
    else if (gen_list && tid == 0) {   // the general launch's row (bounded like the per-row launch)
      const int slot = atomicAdd(gen_count, 1);
      if (slot < rows * Ct) gen_list[slot] = tb * Ct + c;
    }
  }
  if (!act) return;
  const int64_t a0 = (int64_t)c * CH;
  const int64_t a1 = a0 + CH < N ? a0 + CH : N;
  const int64_t rtw = (int64_t)t * pa.mw + (int64_t)p * N;   // pa.wrow(t, g * Bg + p), every g
  const int dtop = n_bins - 1;
  double turn[TO_MAXG][TO_MAXQ], cost[TO_MAXG][TO_MAXQ];
#pragma unroll
  for (int g = 0; g < TO_MAXG; ++g)
#pragma unroll
    for (int q = 0; q < TO_MAXQ; ++q) { turn[g][q] = 0.0; cost[g][q] = 0.0; }
  // VWG_U cells of a lane in flight (every load of them first), then charged in the lane's cell
  // order: the same per-lane sums as one cell at a time (the row is one latency chain per trip,
  // and a C3 launch is ~1 workgroup per CU)
  for (int64_t ab = a0 + tid; ab < a1; ab += VWG_U * PF_THREADS) {
    double x1u[VWG_U], x0u[VWG_U][TO_MAXQ], advu[VWG_U], sgu[VWG_U];
    int l1u[VWG_U][TO_MAXG], l0u[VWG_U][TO_MAXG][TO_MAXQ];
#pragma unroll
    for (int u = 0; u < VWG_U; ++u) {
      const int64_t a = ab + (int64_t)u * PF_THREADS;
      const bool in = a < a1;
      const int64_t ai = in ? a : a0;
      // every load of the cell first: weights / ADV / vol once, then each row's labels
      x1u[u] = W[rtw + ai];
#pragma unroll
      for (int q = 0; q < TO_MAXQ; ++q)
        x0u[u][q] = q < nq ? W[rtw - (int64_t)ks.K[q] * pa.mw + ai] : 1.0;
      advu[u] = 0.0;
      sgu[u] = 0.02;
      if (IMP) {
        advu[u] = ADV[rtw + ai];
        if (SIG) sgu[u] = SIG[rtw + ai];
      }
#pragma unroll
      for (int g = 0; g < TO_MAXG; ++g) {
        const bool on = g < G && ((act >> g) & 1u);
        const int64_t rt = pa.lrow(t, g * Bg + p);
        l1u[u][g] = on ? (int)L[rt + ai] : -1;
#pragma unroll
        for (int q = 0; q < TO_MAXQ; ++q)
          l0u[u][g][q] = (on && q < nq) ? (int)L[rt - (int64_t)ks.K[q] * pa.ml + ai] : -1;
      }
    }
#pragma unroll
    for (int u = 0; u < VWG_U; ++u) {
    if (ab + (int64_t)u * PF_THREADS >= a1) break;
    const double x1 = x1u[u];
    const double* x0 = x0u[u];
    const double adv = advu[u], sg = sgu[u];
    const int* l1 = l1u[u];
    const int (*l0)[TO_MAXQ] = l0u[u];
    const double vw1 = valid_w(x1);
    const double unit_sig = sg == sg ? sg : 0.02;
    const double sra = (IMP && adv > 0.0) ? sqrt(aum / adv) : -1.0;
#pragma unroll
    for (int g = 0; g < TO_MAXG; ++g) {
      if (g >= G || !((act >> g) & 1u)) continue;
      const double* tpv = TPv + (int64_t)(t * B + g * Bg + p) * TP_STRIDE;
#pragma unroll
      for (int q = 0; q < TO_MAXQ; ++q) {
        if (q >= nq) break;
        const double vw0 = valid_w(x0[q]);
#pragma unroll
        for (int li = 0; li < 2; ++li) {
          const int d = li == 0 ? dtop : 0;
          const double f1 = tpv[li * (TO_MAXQ + 1)];
          const double f0 = tpv[li * (TO_MAXQ + 1) + 1 + q];
          const double fs = tpv[2 * (TO_MAXQ + 1) + 2 * q + li];
          const double w1 = (l1[g] == d ? vw1 : 0.0) * f1;
          const double w0 = (l0[g][q] == d ? vw0 : 0.0) * f0;
          const double dw = fabs(w1 - w0) * fs;
          turn[g][q] += dw;
          if (IMP) {   // turnover_body's charge, term for term
            double unit = half_spread;
            if (sra >= 0.0) {
#ifdef VWG_NOSQRT   // A/B timing only (wrong costs): the charge without its square root
              const double im = k_impact * unit_sig * (dw * sra);
#else
              const double im = k_impact * unit_sig * (sqrt(dw) * sra);
#endif
              unit = unit + ((im == im) ? im : 0.0);
            }
            cost[g][q] += dw * unit;
          }
        }
      }
    }
    }
  }
  __shared__ double red[TO_MAXG][PF_WAVES][2 * TO_MAXQ];
#pragma unroll
  for (int g = 0; g < TO_MAXG; ++g) {
    if (g >= G || !((act >> g) & 1u)) continue;
#pragma unroll
    for (int q = 0; q < TO_MAXQ; ++q) {
      if (q >= nq) break;
      const double x1 = wave_sum(turn[g][q]);
      const double y1 = IMP ? wave_sum(cost[g][q]) : 0.0;
      if (lane == 0) { red[g][wid][2 * q] = x1; red[g][wid][2 * q + 1] = y1; }
    }
  }
  __syncthreads();
  if (tid < TO_MAXG * TO_MAXQ) {
    const int g = tid / TO_MAXQ, q = tid - g * TO_MAXQ;
    if (g < G && ((act >> g) & 1u) && q < nq) {
      const int tb = t * B + g * Bg + p;
      double x = 0.0, y = 0.0;
      for (int w2 = 0; w2 < PF_WAVES; ++w2) { x += red[g][w2][2 * q]; y += red[g][w2][2 * q + 1]; }
      TURNp[((int64_t)q * rows + tb) * Ct + c] = 0.5 * x;
      COSTp[((int64_t)q * rows + tb) * Ct + c] = IMP ? y : x * half_spread;
    }
  }
}

// BM (general launch, equal weight, every K <= 31): only the bit-mask path is compiled, so the
// kernel keeps the registers of that path (the dense path's arrays would double them).
template <bool VW, bool IMP, bool GEN, bool BM = false>
#ifndef TO_MINB_BM
#define TO_MINB_BM 4   // general equal-weight rows: workgroups per CU the VGPR budget must allow
                       // (4: the table walk's 129 VGPRs held to 128, no spills)
#endif
__global__ __launch_bounds__(PF_THREADS, BM ? TO_MINB_BM : 1) void k_turnover(
    const int8_t* __restrict__ L, const double* __restrict__ W, const double* __restrict__ FWp,
    int T_m, int B, int64_t N, KSet ks, int Kmax, int n_bins, int Cf, int64_t CH,
    int Ct, double half_spread, double k_impact, double aum, const double* __restrict__ ADV,
    const double* __restrict__ SIG, double* __restrict__ TURNp, double* __restrict__ COSTp,
    int32_t* __restrict__ gen_list, int32_t* __restrict__ gen_count,
    const double* __restrict__ TPv, const uint32_t* __restrict__ TPm, PanAddr pa) {
  if (!GEN) {
    turnover_body<VW, IMP, false>((int)blockIdx.x, L, W, FWp, T_m, B, N, ks, Kmax, n_bins, Cf, CH, Ct,
                                  half_spread, k_impact, aum, ADV, SIG, TURNp, COSTp, gen_list,
                                  gen_count, pa, TPv, TPm);
  } else {   // the general rows the steady launch put on the work list
    const int cap = T_m * B * Ct;                   // the list's capacity
    const int n0 = *(volatile int32_t*)gen_count;   // written by the previous launch
    const int n = n0 < cap ? n0 : cap;
    for (int i = (int)blockIdx.x; i < n; i += (int)gridDim.x) {
      turnover_body<VW, IMP, true, BM>(gen_list[i], L, W, FWp, T_m, B, N, ks, Kmax, n_bins, Cf, CH,
                                   Ct, half_spread, k_impact, aum, ADV, SIG, TURNp, COSTp,
                                   gen_list, gen_count, pa);
      __syncthreads();   // the shared tables are rebuilt for the next row
    }
  }
}


// ------------------------------------------------------------------------------ E2, E3
// one thread per (holding period q of the K set, t, b, decile d): combines decile d over the
// chunks and the cohorts; the d = 0 thread also totals the turnover / cost partials.  Output
// q lands at offset q * rows of the [nK][T_m][B] stacks (PR: [nK][T_m][B][nb]).
__global__ __launch_bounds__(256) void k_overlap(
    const double* __restrict__ SWRp, const double* __restrict__ SWp, KSet ks, int Kmax, int C,
    int nb, const double* __restrict__ TURNp, const double* __restrict__ COSTp, int Ct,
    int64_t rows, double* __restrict__ PR, double* __restrict__ TURN, double* __restrict__ COST,
    int legs, const int32_t* __restrict__ lwp) {
  // one thread per output (q, t, b, d), in PR's layout (flat grid: the one-workgroup-per-row
  // version was 64-lane workgroups with nb lanes busy, dispatch-bound at sweep sizes)
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (int64_t)ks.n * rows * nb) return;
  const int d = (int)(g % nb);
  const int64_t qtb = g / nb;
  const int q = (int)(qtb / rows);
  const int64_t tb = qtb - (int64_t)q * rows;
  const int K = ks.K[q];
  if (legs && d != 0 && d != nb - 1) {   // legs-only cohort sums: not computed
    PR[(q * rows + tb) * nb + d] = qnan();
  } else {
    // the partials' layout: n_bins per (row, age, chunk), or the legs-only two-leg layout (any
    // other word reads as n_bins: never an index past the n_bins layout)
    const int lw = *lwp == 2 ? 2 : nb;
    const int ds = lw == 2 ? (d == 0 ? 0 : 1) : d;
    double acc = 0.0;
    int n = 0;
    for (int k = 0; k < K; ++k) {
      double x = 0.0, y = 0.0;
      // chunk partials in trips of 8, loads first, then summed in chunk order
      for (int c0 = 0; c0 < C; c0 += 8) {
        double xr[8], yr[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int64_t o = ((tb * Kmax + k) * C + (c0 + u < C ? c0 + u : 0)) * lw + ds;
          xr[u] = c0 + u < C ? SWRp[o] : 0.0;
          yr[u] = c0 + u < C ? SWp[o] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (c0 + u >= C) break;
          x += xr[u];
          y += yr[u];
        }
      }
      if (y > 0.0) { acc += x / y; ++n; }
    }
    PR[(q * rows + tb) * nb + d] = n > 0 ? acc / (double)n : qnan();
  }
  if (d == 0 && TURNp) {
    const int64_t to = (q * rows + tb) * Ct;
    double x = 0.0, y = 0.0;
    for (int c = 0; c < Ct; ++c) { x += TURNp[to + c]; y += COSTp[to + c]; }
    if (TURN) TURN[q * rows + tb] = x;
    if (COST) COST[q * rows + tb] = y;
  }
}

// k_overlap with one thread per (t, b, decile d) serving every K of the set: the cohort terms
// of ages 0..Kmax-1 are read once (trips of OV_TRIP ages in flight, instead of one dependent
// load pair per age and K) and K's result is taken when the running sum reaches age K - 1 --
// the same terms summed in the same order as k_overlap, so PR / TURN / COST are bit-identical.
// Single-chunk cohort plans only (C == 1: C5's 30000-row batches); chunked plans (C3) keep
// k_overlap, whose K-parallel grid hides the chunk loop better (0.71 vs 0.89 ms portfolio).
#define OV_TRIP 8
__global__ __launch_bounds__(256) void k_overlap_rows(
    const double* __restrict__ SWRp, const double* __restrict__ SWp, KSet ks, int Kmax,
    int nb, const double* __restrict__ TURNp, const double* __restrict__ COSTp, int Ct,
    int64_t rows, double* __restrict__ PR, double* __restrict__ TURN, double* __restrict__ COST,
    int legs, const int32_t* __restrict__ lwp) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= rows * nb) return;
  const int d = (int)(g % nb);
  const int64_t tb = g / nb;
  if (legs && d != 0 && d != nb - 1) {   // legs-only cohort sums: not computed
    for (int q = 0; q < ks.n; ++q) PR[((int64_t)q * rows + tb) * nb + d] = qnan();
  } else {
    const int lw = *lwp == 2 ? 2 : nb;   // the partials' layout (k_overlap)
    const int ds = lw == 2 ? (d == 0 ? 0 : 1) : d;
    double acc = 0.0;
    int n = 0;
    for (int k0 = 0; k0 < Kmax; k0 += OV_TRIP) {
      double xs[OV_TRIP], ys[OV_TRIP];
#pragma unroll
      for (int u = 0; u < OV_TRIP; ++u) {   // one partial per (age, decile): loads first
        const int64_t o = (tb * Kmax + (k0 + u < Kmax ? k0 + u : 0)) * lw + ds;
        xs[u] = k0 + u < Kmax ? 0.0 + SWRp[o] : 0.0;   // 0.0 + x: k_overlap's chunk sum of one
        ys[u] = k0 + u < Kmax ? 0.0 + SWp[o] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < OV_TRIP; ++u) {
        const int k = k0 + u;
        if (k >= Kmax) break;
        if (ys[u] > 0.0) { acc += xs[u] / ys[u]; ++n; }
        for (int q = 0; q < ks.n; ++q)
          if (ks.K[q] == k + 1) PR[((int64_t)q * rows + tb) * nb + d] = n > 0 ? acc / (double)n : qnan();
      }
    }
  }
  if (d == 0 && TURNp) {
    for (int q = 0; q < ks.n; ++q) {
      const int64_t to = ((int64_t)q * rows + tb) * Ct;
      double x = 0.0, y = 0.0;
      for (int c = 0; c < Ct; ++c) { x += TURNp[to + c]; y += COSTp[to + c]; }
      if (TURN) TURN[(int64_t)q * rows + tb] = x;
      if (COST) COST[(int64_t)q * rows + tb] = y;
    }
  }
}

// one workgroup per (panel b, holding period q): the reference's long-short rule on PR[q].
// need_full (legs-only accounting): set when a panel lacks one leg's column, where the rule
// falls back to max - min over every decile (the caller reruns with every decile).
// one workgroup per (panel b, holding period q): batches of fewer than LS_PB panels (C3)
__global__ __launch_bounds__(256) void k_ls(const double* __restrict__ PR, int T_m, int B, int nb,
                                            double* __restrict__ LS,
                                            const double* __restrict__ COST,
                                            double* __restrict__ NET, int32_t* __restrict__ need_full) {
  const int b = blockIdx.x;
  const int64_t qo = (int64_t)blockIdx.y * T_m * B;
  PR += qo * nb;
  LS += qo;
  if (NET) { NET += qo; COST += qo; }
  __shared__ int has_lo, has_hi;
  if (threadIdx.x == 0) { has_lo = 0; has_hi = 0; }
  __syncthreads();
  int lo = 0, hi = 0;
  for (int t = threadIdx.x; t < T_m; t += blockDim.x) {
    const double* e = PR + ((int64_t)t * B + b) * nb;
    lo |= e[0] == e[0];
    hi |= e[nb - 1] == e[nb - 1];
  }
  if (lo) atomicOr(&has_lo, 1);
  if (hi) atomicOr(&has_hi, 1);
  __syncthreads();
  const bool both = has_lo && has_hi;
  if (need_full && !both && threadIdx.x == 0) atomicOr(need_full, 1);
  for (int t = threadIdx.x; t < T_m; t += blockDim.x) {
    const int64_t tb = (int64_t)t * B + b;
    const double* e = PR + tb * nb;
    bool any = false;
    double mx = -INFINITY, mn = INFINITY;
    for (int d = 0; d < nb; ++d)
      if (e[d] == e[d]) { any = true; mx = fmax(mx, e[d]); mn = fmin(mn, e[d]); }
    double v = qnan();
    if (any) v = both ? (e[nb - 1] - e[0]) : (mx - mn);
    LS[tb] = v;
    if (NET) NET[tb] = v - COST[tb];
  }
}

// Wide batches (C5: B = 800 panels of a grouped launch) in two launches instead of one
// workgroup per 64 panels walking every month twice (52 workgroups, 140 us per launch):
// k_ls_flags -- per (panel b, holding period q) whether some month has a decile-0 value
// (bit 0) and some month a decile-(nb-1) value (bit 1), from blocks of LS_FM months in
// parallel (64 panels x 4 month phases per workgroup, an atomicOr per panel into a zeroed
// [nK][B] word array) -- then k_ls_rows, one thread per (q, t, b) output with k_ls's rule.
// The same flags and the same per-output arithmetic as k_ls, so the same bits.
#define LS_PB 64   // batches of at least this many panels take the two-launch form
#define LS_FM 32   // months per k_ls_flags workgroup (8 per thread, loads in flight)
__global__ __launch_bounds__(256) void k_ls_flags(const double* __restrict__ PR, int T_m, int B,
                                                  int nb, int32_t* __restrict__ flags) {
  const int p = (int)threadIdx.x & 63, j = (int)threadIdx.x >> 6;
  const int b = (int)blockIdx.x * 64 + p;
  const int q = (int)blockIdx.y;
  const int t0 = (int)blockIdx.z * LS_FM;
  const bool on = b < B;
  const double* P0 = PR + (int64_t)q * T_m * B * nb;
  constexpr int TK = LS_FM / 4;
  double lo[TK], hi[TK];
#pragma unroll
  for (int k = 0; k < TK; ++k) {
    const int t = t0 + j + 4 * k;
    const bool ok = on && t < T_m;
    const double* e = P0 + ((int64_t)(ok ? t : 0) * B + (on ? b : 0)) * nb;
    lo[k] = ok ? e[0] : qnan();
    hi[k] = ok ? e[nb - 1] : qnan();
  }
  int f = 0;
#pragma unroll
  for (int k = 0; k < TK; ++k) f |= (lo[k] == lo[k] ? 1 : 0) | (hi[k] == hi[k] ? 2 : 0);
  __shared__ int fl[4][64];
  fl[j][p] = f;
  __syncthreads();
  if (j == 0 && on) {
    const int g = fl[0][p] | fl[1][p] | fl[2][p] | fl[3][p];
    if (g) atomicOr(flags + (int64_t)q * B + b, g);
  }
}

__global__ __launch_bounds__(256) void k_ls_rows(const double* __restrict__ PR, int T_m, int B,
                                                 int nb, int nq, const int32_t* __restrict__ flags,
                                                 double* __restrict__ LS,
                                                 const double* __restrict__ COST,
                                                 double* __restrict__ NET,
                                                 int32_t* __restrict__ need_full) {
  const int64_t rows = (int64_t)T_m * B;
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (int64_t)nq * rows) return;
  const int q = (int)(g / rows);
  const int64_t tb = g - (int64_t)q * rows;
  const int b = (int)(tb % B);
  const bool both = flags[(int64_t)q * B + b] == 3;
  if (need_full && !both && tb < B) atomicOr(need_full, 1);   // (month 0's thread of the panel)
  const double* e = PR + g * nb;
  const double lo = e[0], hi = e[nb - 1];
  double v = qnan();
  if (both && lo == lo && hi == hi) {   // (some decile holds a value: k_ls's D(n-1) - D0)
    v = hi - lo;
  } else {   // the interior deciles decide (any value at all; max - min without both legs)
    bool any = false;
    double mx = -INFINITY, mn = INFINITY;
    for (int d = 0; d < nb; ++d)
      if (e[d] == e[d]) { any = true; mx = fmax(mx, e[d]); mn = fmin(mn, e[d]); }
    if (any) v = both ? (hi - lo) : (mx - mn);
  }
  LS[g] = v;
  if (NET) NET[g] = v - COST[g];
}

// ---------------------------------------------------------------------------------- E6
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
__device__ __forceinline__ double uniform01(uint64_t seed, int64_t b, int t, int stream) {
  const uint64_t key = seed * 0xD1B54A32D192ED03ULL + (uint64_t)b * 0x9E3779B97F4A7C15ULL +
                       (uint64_t)(t * 4 + stream);
  return (double)(splitmix64(key) >> 11) * 0x1.0p-53;
}

// one thread per panel: the stationary-bootstrap source-month sequence
__global__ __launch_bounds__(256) void k_bootstrap_index(int T_m, int B, int64_t b0,
                                                         uint64_t seed, double p_new,
                                                         int32_t* __restrict__ src) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  int prev = 0;
  for (int t = 0; t < T_m; ++t) {
    const double u = uniform01(seed, b0 + b, t, 0);
    int jump = (int)(u * (double)T_m);
    jump = jump < T_m - 1 ? jump : T_m - 1;
    int cur = jump;
    if (t > 0) {
      const bool nw = uniform01(seed, b0 + b, t, 1) < p_new;
      cur = nw ? jump : (prev + 1 == T_m ? 0 : prev + 1);
    }
    src[(int64_t)b * T_m + t] = cur;
    prev = cur;
  }
}

// one thread per (panel, asset): sequential price product over the resampled months
__global__ __launch_bounds__(256) void k_bootstrap_panel(const double* __restrict__ R, int T_m,
                                                         int B, int64_t N,
                                                         const int32_t* __restrict__ src,
                                                         double p0, double* __restrict__ PMb) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (int64_t)B * N) return;
  const int b = (int)(g / N);
  const int64_t a = g - (int64_t)b * N;
  double prev = p0;
  for (int t = 0; t < T_m; ++t) {
    const double r = R[(int64_t)src[(int64_t)b * T_m + t] * N + a];
    const int64_t o = ((int64_t)t * B + b) * N + a;
    if (r == r) {
      const double f = 1.0 + r;
      prev = prev * f;
      PMb[o] = prev;
    } else {
      PMb[o] = absent_val();
    }
  }
}

void launch_bootstrap_index(hipStream_t st, int T_m, int B, int64_t b0, uint64_t seed,
                            double p_new, int32_t* src) {
  hipLaunchKernelGGL(k_bootstrap_index, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, T_m,
                     B, b0, seed, p_new, src);
}

// ------------------------------------------------------------------------------- C ABI
// 1: cohort sums through per-wave LDS atomics (k_cohort_lds) where they fit; 0: registers
static int g_tune_cohort_lds = 1;
// 1: label-sorted segment gathers (k_label_sort + k_cohort_seg) where N <= SEG_MAXN
static int g_tune_cohort_seg = 1;
// workgroups of the persistent general-row turnover launch (walking the work list)
static int64_t g_tune_turn_gen_grid = 8192;   // C5 portfolio: 512 49.1, 2048 40.1, 8192 39.5 ms
// 1: k_overlap_rows (one thread per (t, b, decile) serving every K of the set) for single-chunk
// cohort plans, 0: k_overlap always
static int g_tune_overlap_rows = 1;
// Diagnosis of the round-3 graph-replay fault (tests/test_gpu_capture.py): how the turnover
// work-list counter is reset before the steady launch (1: k_zero_i32, the default; 0:
// hipMemsetAsync, round 3's form), and an optional device int32 that receives the counter the
// general launch read (csm_tune_ptr("gen_probe")).  Neither changes a result.
static int g_tune_gen_reset = 1;
// 1: grouped batches' steady value-weight rows by k_turnover_vwg (a weight panel's groups in one
// workgroup) | 0 by the per-row launch (A/B; the same bits)
static int g_tune_turn_vwg = 1;
// steady equal-weight legs turnover from the leg bitplanes (k_turnover_ew_mask) | 0 from labels
static int g_tune_turn_mask = 1;
// the one-wave legs label sort's prefix ranks by v_mbcnt (1) | masked popcounts (0)
static int g_tune_ls_opt = 1;
static int32_t* g_gen_probe = nullptr;

__global__ void k_copy_i32(const int32_t* __restrict__ src, int32_t* __restrict__ dst) {
  if (threadIdx.x == 0) dst[0] = *(volatile const int32_t*)src;
}
// n int32 words set to v (a kernel node under capture, as the work-list counter's reset)
__global__ __launch_bounds__(256) void k_fill_i32(int32_t* __restrict__ p, int64_t n, int32_t v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}
static void fill_i32(hipStream_t st, int32_t* p, int64_t n, int32_t v) {
  const int64_t g = std::min<int64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(k_fill_i32, dim3((unsigned)(g > 0 ? g : 1)), dim3(256), 0, st, p, n, v);
}

struct PfPlan {
  int C, kpar, Ct;
  int64_t CH, CHt;
};

// Enough workgroups to fill 256 CUs several times over, chunks of >= PF_CHUNK_MIN assets.
// turnover workgroups wanted per launch (the row split into chunks to reach it); A/B knob
// "turn_want" -- set it before the portfolio workspace is sized
static int64_t g_tune_turn_want = 4096;
static PfPlan pf_plan(int32_t T_m, int32_t B, int64_t N, int32_t K, int32_t n_bins) {
  PfPlan p;
  // Batches of up to PF_PLAN_MIN_B panels are planned as PF_PLAN_MIN_B panels: the sweeps join
  // the four look-backs of a single-panel grid into one launch (B = 4) and a strategy-sharded
  // rank runs fewer of them (B = 1, 2), so a panel's turnover chunks -- and with them the bits
  // of its TURN / COST sums -- do not depend on how many look-backs share its launch.
  const int64_t rows = (int64_t)T_m * (B < PF_PLAN_MIN_B ? PF_PLAN_MIN_B : B);
  const int64_t want = 4096;
  const int64_t cmax = (N + PF_CHUNK_MIN - 1) / PF_CHUNK_MIN;
  // the turnover chunking depends on (rows, N) only; the cohort chunk count also on whether the
  // segment path takes this (N, Kmax, n_bins) -- the same for every K of a portfolio_multi call,
  // so a cohort pass gives the same partial sums as the per-K calls (bit for bit).  The plan
  // reads the "cohort_seg" and "turn_want" tune knobs: set them BEFORE sizing a workspace
  // (csm_portfolio_workspace), never between sizing and the call
  // (cohort-parallel grids, kpar = 1, made tens of thousands of tiny workgroups at C3 and
  // ran slower than one workgroup walking its K cohorts over a chunk.)
  (void)K;
  p.kpar = 0;
  int64_t C = (want + rows - 1) / rows;
  C = C < 1 ? 1 : (C > cmax ? cmax : C);
  // the label-sorted segment path (launch_cohort) owns every segment whole in one of its first
  // ceil(1024 / rows) chunks and writes zeros in the others: plan only those (C3: 4 -> 1 chunk,
  // a quarter of the cohort workgroups and overlap partials; the sums are the same bits)
  if (g_tune_cohort_seg && N <= SEG_MAXN && (int64_t)K * (n_bins + 1) <= SEG_MAXKD) {
    const int64_t cs = (1024 + rows - 1) / rows;
    C = C < cs ? C : (cs < 1 ? 1 : cs);
  }
  p.C = (int)C;
  p.CH = (N + C - 1) / C;
  int64_t Ct = (g_tune_turn_want + rows - 1) / rows;   // turnover chunks
  Ct = Ct < 1 ? 1 : (Ct > cmax ? cmax : Ct);
  const int64_t cmin = (N + 65471) / 65472;       // < 65536 cells per chunk (packed counts)
  Ct = Ct < cmin ? cmin : Ct;
  p.CHt = ((N + Ct - 1) / Ct + 63) / 64 * 64;   // chunk bounds on 64-cell (4-byte) boundaries
  p.Ct = (int)((N + p.CHt - 1) / p.CHt);
  return p;
}

// formation leg totals of each row: the chunk partials summed in chunk order, once per row
// (k_turnover reads them for K + 1 formation months per block)
__global__ __launch_bounds__(256) void k_fw_fold(const double* __restrict__ FWp, int64_t rows,
                                                 int C, double* __restrict__ FWt) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= 2 * rows) return;
  const int64_t row = i >> 1;
  const int leg = (int)(i & 1);
  double tot = 0.0;
  for (int c = 0; c < C; ++c) tot += FWp[(row * C + c) * 2 + leg];
  FWt[i] = tot;
}

// Returns whether the legs-only segment pass ran (its partials in the two-leg layout).
template <int NB>
static bool launch_cohort(hipStream_t st, const PfPlan& pl, const int8_t* L, const double* NR,
                          const double* W, int T_m, int B, int64_t N, int K, double* SWRp,
                          double* SWp, double* FWp, char* segws, int64_t perm_b, int64_t off_b,
                          int64_t wsrt_b, bool legs, const PanAddr& pa, int64_t lm_b = 0) {
  const dim3 g((unsigned)(pl.C * T_m * B), 1u, pl.kpar ? (unsigned)K : 1u);
  if (g_tune_cohort_seg && segws && !pl.kpar && K * (NB + 1) <= SEG_MAXKD) {
    uint16_t* PERM = (uint16_t*)(segws + perm_b);
    int32_t* OFF = (int32_t*)(segws + off_b);
    double* WSRT = (double*)(segws + wsrt_b);
    SegJ sj;
    sj.n = 1;
    sj.PERM[0] = PERM; sj.OFF[0] = OFF; sj.SWR[0] = SWRp; sj.SW[0] = SWp;
    const int xcd = pl.C == 1 && B >= 8;
    const int64_t rows = (int64_t)T_m * B;
    const int Cs = (int)std::min<int64_t>(pl.C, std::max<int64_t>(1, (1024 + rows - 1) / rows));
    const dim3 g1((unsigned)(T_m * B)),
        g2(xcd ? (unsigned)(8 * ((B + 7) / 8) * T_m) : (unsigned)(pl.C * T_m * B));
    const size_t lds = (size_t)(N + 1) * sizeof(double) +
                       (legs ? (size_t)K * 4 * sizeof(uint16_t) : (size_t)K * (NB + 1) * sizeof(int32_t));
    if (legs) {
      if (W) {
        hipLaunchKernelGGL((k_label_sort<NB, true, true>), g1, dim3(PF_THREADS), (size_t)N * 9, st, L, W, N,
                           pl.C, PERM, OFF, WSRT, FWp, pa);
        hipLaunchKernelGGL((k_cohort_seg<NB, true, true>), g2, dim3(PF_THREADS), lds, st, NR, sj,
                           (const double*)WSRT, T_m, B, N, K, pl.C, Cs, xcd, 1, pa, B);
      } else {
        if ((N & 3) == 0)   // one wave per row (C5's equal-weight legs)
          hipLaunchKernelGGL((g_tune_ls_opt ? k_label_sort_legs_ew<NB, true> : k_label_sort_legs_ew<NB, false>), dim3((unsigned)((T_m * (int64_t)B + PF_WAVES - 1) / PF_WAVES)),
                             dim3(PF_THREADS), 0, st, L, N, pl.C, (int64_t)T_m * B, PERM, OFF, FWp, pa,
                             g_tune_turn_mask ? (uint64_t*)(segws + lm_b) : nullptr, (N + 255) / 256 * 4);
        else
          hipLaunchKernelGGL((k_label_sort<NB, false, true>), g1, dim3(PF_THREADS), (size_t)N, st, L, W, N,
                             pl.C, PERM, OFF, WSRT, FWp, pa);
        hipLaunchKernelGGL((k_cohort_seg<NB, false, true>), g2, dim3(PF_THREADS), lds, st, NR, sj,
                           (const double*)WSRT, T_m, B, N, K, pl.C, Cs, xcd, 1, pa, B);
      }
    } else if (W) {
      hipLaunchKernelGGL((k_label_sort<NB, true>), g1, dim3(PF_THREADS), (size_t)N * 9, st, L, W, N, pl.C,
                         PERM, OFF, WSRT, FWp, pa);
      hipLaunchKernelGGL((k_cohort_seg<NB, true>), g2, dim3(PF_THREADS), lds, st, NR, sj,
                         (const double*)WSRT, T_m, B, N, K, pl.C, Cs, xcd, 1, pa, B);
    } else {
      hipLaunchKernelGGL((k_label_sort<NB, false>), g1, dim3(PF_THREADS), (size_t)N, st, L, W, N, pl.C,
                         PERM, OFF, WSRT, FWp, pa);
      hipLaunchKernelGGL((k_cohort_seg<NB, false>), g2, dim3(PF_THREADS), lds, st, NR, sj,
                         (const double*)WSRT, T_m, B, N, K, pl.C, Cs, xcd, 1, pa, B);
    }
    return legs;
  }
  if (g_tune_cohort_lds && !pl.kpar && K * NB <= AC_MAXKD) {
    const dim3 g2((unsigned)(pl.C * T_m * B));
    if (W)
      hipLaunchKernelGGL((k_cohort_lds<NB, true>), g2, dim3(PF_THREADS), 0, st, L, NR, W, T_m, B,
                         N, K, pl.C, pl.CH, SWRp, SWp, FWp, pa);
    else
      hipLaunchKernelGGL((k_cohort_lds<NB, false>), g2, dim3(PF_THREADS), 0, st, L, NR, W, T_m, B,
                         N, K, pl.C, pl.CH, SWRp, SWp, FWp, pa);
    return false;
  }
  if (W)
    hipLaunchKernelGGL((k_cohort<NB, true>), g, dim3(PF_THREADS), 0, st, L, NR, W, T_m, B, N, K,
                       pl.C, pl.CH, pl.kpar, SWRp, SWp, FWp, pa);
  else
    hipLaunchKernelGGL((k_cohort<NB, false>), g, dim3(PF_THREADS), 0, st, L, NR, W, T_m, B, N, K,
                       pl.C, pl.CH, pl.kpar, SWRp, SWp, FWp, pa);
  return false;
}

// Equal-weight cohort sums of nJ look-backs sharing one next_ret panel (segment path, one chunk
// per row): each J's label sort, then ONE k_cohort_seg launch staging each month's return row
// once for every J.  ws[q]: J q's workspace base; the partials land where launch_cohort puts
// them, bit for bit the same values.
// grouped: L[0] holds the Js' label panels group-major ([nJ][T_m][B * N]) and ws[0] is ONE
// workspace laid out for nJ * B panels (J q's panel b = panel q * B + b, as csm_cohort_sums_grouped
// lays them out): one label-sort launch for every J, and the same partials at those rows.
template <int NB>
static void launch_cohort_js(hipStream_t st, const PfPlan& pl, int nJ, const int8_t* const* L,
                             const double* NR, int T_m, int B, int64_t N, int K, char* const* ws,
                             int64_t swr_b, int64_t sw_b, int64_t fw_b, int64_t perm_b,
                             int64_t off_b, bool legs, bool grouped, int64_t lm_b) {
  const int xcd = B >= 8;
  const dim3 g2(xcd ? (unsigned)(8 * ((B + 7) / 8) * T_m) : (unsigned)(T_m * B));
  const PanAddr pa = pan_plain(B, N);
  const int Bo = grouped ? nJ * B : B;   // panels per month of the workspace rows
  auto label_sort = [&](const int8_t* Lq, char* w, int nrow_b, const PanAddr& pl_a) {
    uint16_t* PERM = (uint16_t*)(w + perm_b);
    int32_t* OFF = (int32_t*)(w + off_b);
    double* FWp = (double*)(w + fw_b);
    const int64_t rows = (int64_t)T_m * nrow_b;
    if (legs && (N & 3) == 0)
      hipLaunchKernelGGL((g_tune_ls_opt ? k_label_sort_legs_ew<NB, true> : k_label_sort_legs_ew<NB, false>),
                         dim3((unsigned)((rows + PF_WAVES - 1) / PF_WAVES)),
                         dim3(PF_THREADS), 0, st, Lq, N, 1, rows, PERM, OFF, FWp, pl_a,
                         g_tune_turn_mask ? (uint64_t*)(w + lm_b) : nullptr, (N + 255) / 256 * 4);
    else if (legs)
      hipLaunchKernelGGL((k_label_sort<NB, false, true>), dim3((unsigned)rows), dim3(PF_THREADS), (size_t)N,
                         st, Lq, (const double*)nullptr, N, 1, PERM, OFF, (double*)nullptr, FWp, pl_a);
    else
      hipLaunchKernelGGL((k_label_sort<NB, false>), dim3((unsigned)rows), dim3(PF_THREADS), (size_t)N, st,
                         Lq, (const double*)nullptr, N, 1, PERM, OFF, (double*)nullptr, FWp, pl_a);
  };
  if (grouped) label_sort(L[0], ws[0], nJ * B, pan_grouped(nJ, B, T_m, N));
  const int64_t PS = seg_stride(N);
  SegJ sj;
  sj.n = nJ;
  for (int q = 0; q < nJ; ++q) {
    char* w = grouped ? ws[0] : ws[q];
    if (!grouped) label_sort(L[q], w, B, pa);
    const int64_t r0 = grouped ? (int64_t)q * B : 0;   // J q's first workspace row of a month
    sj.PERM[q] = (uint16_t*)(w + perm_b) + r0 * PS;
    sj.OFF[q] = (int32_t*)(w + off_b) + r0 * (NB + 1);
    const int swv = legs ? 2 : NB;   // partials per (row, age): k_cohort_seg's layout
    sj.SWR[q] = (double*)(w + swr_b) + r0 * K * swv;   // (one cohort chunk)
    sj.SW[q] = (double*)(w + sw_b) + r0 * K * swv;
  }
  const size_t lds = (size_t)(N + 1) * sizeof(double) +
                     (legs ? (size_t)nJ * K * 4 * sizeof(uint16_t) : (size_t)nJ * K * (NB + 1) * sizeof(int32_t));
  if (legs)
    hipLaunchKernelGGL((k_cohort_seg<NB, false, true>), g2, dim3(PF_THREADS), lds, st, NR, sj,
                       (const double*)nullptr, T_m, B, N, K, 1, 1, xcd, 1, pa, Bo);
  else
    hipLaunchKernelGGL((k_cohort_seg<NB, false>), g2, dim3(PF_THREADS), lds, st, NR, sj,
                       (const double*)nullptr, T_m, B, N, K, 1, 1, xcd, 1, pa, Bo);
}

// Workspace layout of the cohort partials for (T_m, B, N, n_bins, Kmax): SWRp, SWp
// [rows][Kmax][C][n_bins], FWp [rows][C][2], then the turnover partials [rows][Ct] x 2.
struct PfLayout {
  PfPlan p;
  int64_t rows, swr, sw, fw, fwt, turn, cost, bytes;
  int64_t gen_b;                     // byte offset: int32 count + [rows * Ct] general-row work list
  int64_t tp_b, tpm_b;               // byte offsets: k_turn_prep's per-row factors and masks
  bool seg;                          // label-sort buffers present (N <= SEG_MAXN)
  int64_t perm_b, off_b, wsrt_b;     // byte offsets: uint16 [rows][N], int32 [rows][nb+1], f64 [rows][N]
  int64_t lm_b, nwm;                 // leg bitplanes uint64 [rows][2][nwm] (k_label_sort_legs_ew)
  int64_t lsf_b;                     // byte offset: int32 [TO_MAXQ][B] long-short leg flags (k_ls_flags)
  int64_t lw_b;                      // byte offset: int32, the cohort partials' width per (row,
                                     // age, chunk) the last cohort pass wrote: 2 = the legs-only
                                     // two-leg layout, else n_bins (read on the device by k_overlap*)
};
static PfLayout pf_layout(int32_t T_m, int32_t B, int64_t N, int32_t n_bins, int32_t Kmax) {
  PfLayout l;
  l.p = pf_plan(T_m, B, N, Kmax, n_bins);
  l.rows = (int64_t)T_m * B;
  const int64_t cs = l.rows * Kmax * l.p.C * n_bins;
  l.swr = 0;
  l.sw = cs;
  l.fw = 2 * cs;
  // [rows][2] folded totals; with one cohort chunk the partials ARE the totals (no fold launch)
  l.fwt = l.p.C == 1 ? l.fw : l.fw + l.rows * l.p.C * 2;
  l.turn = l.fwt + l.rows * 2;                              // [TO_MAXQ][rows][Ct]
  l.cost = l.turn + (int64_t)TO_MAXQ * l.rows * l.p.Ct;
  l.bytes = (l.cost + (int64_t)TO_MAXQ * l.rows * l.p.Ct) * 8 + 256;
  l.gen_b = (l.bytes + 255) / 256 * 256;
  l.bytes = l.gen_b + (1 + l.rows * l.p.Ct) * 4 + 256;
  l.tp_b = (l.bytes + 255) / 256 * 256;                    // k_turn_prep: f64 [rows][TP_STRIDE]
  l.tpm_b = l.tp_b + l.rows * TP_STRIDE * 8;               // then u32 [rows] full-leg masks
  l.bytes = l.tpm_b + l.rows * 4 + 256;
  l.seg = N <= SEG_MAXN;
  l.perm_b = l.off_b = l.wsrt_b = l.lm_b = 0;
  l.nwm = (N + 255) / 256 * 4;
  if (l.seg) {
    auto al = [](int64_t x) { return (x + 255) / 256 * 256; };
    l.perm_b = al(l.bytes);
    l.off_b = al(l.perm_b + l.rows * seg_stride(N) * 2);
    l.wsrt_b = al(l.off_b + l.rows * (n_bins + 1) * 4);
    l.lm_b = al(l.wsrt_b + l.rows * seg_stride(N) * 8);
    l.bytes = al(l.lm_b + l.rows * 2 * l.nwm * 8);
  }
  l.lsf_b = (l.bytes + 255) / 256 * 256;
  l.lw_b = l.lsf_b + (int64_t)TO_MAXQ * B * 4;
  l.bytes = l.lw_b + 4 + 256;
  return l;
}

extern "C" {

int csm_tune_portfolio(const char* key, int value) {
  if (key && !strcmp(key, "cohort_lds") && (value == 0 || value == 1)) {
    g_tune_cohort_lds = value;
    return CSM_OK;
  }
  if (key && !strcmp(key, "cohort_seg") && (value == 0 || value == 1)) {
    g_tune_cohort_seg = value;
    return CSM_OK;
  }
  if (key && !strcmp(key, "turn_want") && value >= 1) {
    g_tune_turn_want = value;
    return CSM_OK;
  }
  if (key && !strcmp(key, "turn_gen_grid") && value >= 1) {
    g_tune_turn_gen_grid = value;
    return CSM_OK;
  }
  if (key && !strcmp(key, "overlap_rows") && (value == 0 || value == 1)) {
    g_tune_overlap_rows = value;
    return CSM_OK;
  }
  if (key && !strcmp(key, "gen_reset") && (value == 0 || value == 1)) {
    g_tune_gen_reset = value;
    return CSM_OK;
  }
  if (key && !strcmp(key, "turn_vwg") && (value == 0 || value == 1)) {
    g_tune_turn_vwg = value;
    return CSM_OK;
  }
  if (key && !strcmp(key, "turn_mask") && (value == 0 || value == 1)) {
    g_tune_turn_mask = value;
    return CSM_OK;
  }
  if (key && !strcmp(key, "ls_opt") && (value == 0 || value == 1)) {
    g_tune_ls_opt = value;
    return CSM_OK;
  }
  return CSM_E_INVAL;
}

int csm_tune_ptr_portfolio(const char* key, void* p) {
  if (key && !strcmp(key, "gen_probe")) {
    g_gen_probe = (int32_t*)p;
    return CSM_OK;
  }
  return CSM_E_INVAL;
}

int64_t csm_portfolio_workspace(int32_t T_m, int32_t B, int64_t N, int32_t n_bins, int32_t K) {
  if (T_m < 0 || B < 1 || N <= 0 || n_bins < 1 || K < 1) return 0;
  return pf_layout(T_m, B, N, n_bins, K).bytes;
}

static bool legs_masks(const PfLayout& lay, bool legs, int64_t N, int Kmax, int n_bins);
static void planes_note(csm_ctx* ctx, void* ws, unsigned bits);

static int cohort_sums(csm_ctx* ctx, const int8_t* L, const double* NR, const double* W,
                       int32_t T_m, int32_t B, int64_t N, int32_t n_bins, int32_t Kmax,
                       void* workspace, bool legs, const PanAddr& pa) {
  int r = prep(ctx);
  if (r) return r;
  if (!L || !NR || !workspace || T_m < 0 || B < 1 || N <= 0 || Kmax < 1 || Kmax > TO_MAXK ||
      (int64_t)T_m * B > 0x7FFFFFFF)
    return set_err(ctx, CSM_E_INVAL, "csm_cohort_sums: bad arguments (T_m=%d B=%d N=%lld Kmax=%d)",
                   T_m, B, (long long)N, Kmax);
  if (T_m == 0) return CSM_OK;
  const PfLayout lay = pf_layout(T_m, B, N, n_bins, Kmax);
  double* ws = (double*)workspace;
  hipStream_t st = ctx->stream;
  bool dense = false;   // legs-only partials in the two-leg layout
  switch (n_bins) {
#define PF_CASE(NBV) case NBV: dense = launch_cohort<NBV>(st, lay.p, L, NR, W, T_m, B, N, Kmax, ws + lay.swr, ws + lay.sw, ws + lay.fw, lay.seg ? (char*)workspace : nullptr, lay.perm_b, lay.off_b, lay.wsrt_b, legs, pa, lay.lm_b); break;
    PF_CASE(2) PF_CASE(3) PF_CASE(4) PF_CASE(5) PF_CASE(10) PF_CASE(20) PF_CASE(30)
#undef PF_CASE
    default:
      return set_err(ctx, CSM_E_INVAL, "csm_cohort_sums: n_bins=%d unsupported (2,3,4,5,10,20,30)", n_bins);
  }
  LAUNCH_CHECK(ctx, "k_cohort");
  fill_i32(st, (int32_t*)((char*)workspace + lay.lw_b), 1, dense ? 2 : n_bins);
  planes_note(ctx, workspace, !W && legs_masks(lay, legs, N, Kmax, n_bins) ? 1u : 0u);
  if (lay.p.C > 1) {
    hipLaunchKernelGGL(k_fw_fold, dim3((unsigned)((2 * lay.rows + 255) / 256)), dim3(256), 0, st,
                       (const double*)(ws + lay.fw), lay.rows, lay.p.C, ws + lay.fwt);
    LAUNCH_CHECK(ctx, "k_fw_fold");
  }
  return CSM_OK;
}

int csm_cohort_sums(csm_ctx* ctx, const int8_t* L, const double* NR, const double* W, int32_t T_m,
                    int32_t B, int64_t N, int32_t n_bins, int32_t Kmax, void* workspace) {
  return cohort_sums(ctx, L, NR, W, T_m, B, N, n_bins, Kmax, workspace, false, pan_plain(B, N));
}

int csm_cohort_sums_js(csm_ctx* ctx, int32_t nJ, const int8_t* const* L, const double* NR,
                       int32_t T_m, int32_t B, int64_t N, int32_t n_bins, int32_t Kmax,
                       int32_t legs, void* const* workspaces) {
  int r = prep(ctx);
  if (r) return r;
  if (!L || !NR || !workspaces || nJ < 1 || nJ > SEG_MAXJ || T_m < 0 || B < 1 || N <= 0 ||
      Kmax < 1 || Kmax > TO_MAXK || (int64_t)T_m * B > 0x7FFFFFFF)
    return set_err(ctx, CSM_E_INVAL, "csm_cohort_sums_js: bad arguments (nJ=%d T_m=%d B=%d N=%lld "
                   "Kmax=%d; 1 <= nJ <= %d)", nJ, T_m, B, (long long)N, Kmax, SEG_MAXJ);
  if (legs && N > SEG_MAXN)
    return set_err(ctx, CSM_E_INVAL, "csm_cohort_sums_js: legs on rows of <= %d assets (N=%lld)",
                   SEG_MAXN, (long long)N);
  for (int q = 0; q < nJ; ++q)
    if (!L[q] || !workspaces[q])
      return set_err(ctx, CSM_E_INVAL, "csm_cohort_sums_js: L[%d] or workspace[%d] is NULL", q, q);
  if (T_m == 0) return CSM_OK;
  const PfLayout lay = pf_layout(T_m, B, N, n_bins, Kmax);
  // one staged return row for every J: the segment path with one chunk per row; otherwise the
  // per-J passes (the same partials)
  const bool shared = g_tune_cohort_seg && lay.seg && lay.p.C == 1 && !lay.p.kpar &&
                      (legs ? nJ * Kmax * 4 : nJ * Kmax * (n_bins + 1)) <= SEG_MAXKD &&
                      (n_bins == 2 || n_bins == 3 || n_bins == 4 || n_bins == 5 || n_bins == 10 ||
                       n_bins == 20 || n_bins == 30);
  if (!shared) {
    for (int q = 0; q < nJ; ++q) {
      r = cohort_sums(ctx, L[q], NR, nullptr, T_m, B, N, n_bins, Kmax, workspaces[q], legs != 0,
                      pan_plain(B, N));
      if (r) return r;
    }
    return CSM_OK;
  }
  hipStream_t st = ctx->stream;
  char* ws[SEG_MAXJ];
  for (int q = 0; q < nJ; ++q) ws[q] = (char*)workspaces[q];
  switch (n_bins) {
#define PJ_CASE(NBV) case NBV: launch_cohort_js<NBV>(st, lay.p, nJ, L, NR, T_m, B, N, Kmax, ws, lay.swr * 8, lay.sw * 8, lay.fw * 8, lay.perm_b, lay.off_b, legs != 0, false, lay.lm_b); break;
    PJ_CASE(2) PJ_CASE(3) PJ_CASE(4) PJ_CASE(5) PJ_CASE(10) PJ_CASE(20) PJ_CASE(30)
#undef PJ_CASE
  }
  LAUNCH_CHECK(ctx, "k_cohort_seg (shared next_ret)");
  for (int q = 0; q < nJ; ++q)
    fill_i32(st, (int32_t*)(ws[q] + lay.lw_b), 1, legs ? 2 : n_bins);
  for (int q = 0; q < nJ; ++q) planes_note(ctx, ws[q], legs_masks(lay, legs != 0, N, Kmax, n_bins) ? 1u : 0u);
  // (the shared path has one cohort chunk: each J's partials are its folded totals)
  return CSM_OK;
}

int csm_cohort_sums_js_grouped(csm_ctx* ctx, int32_t nJ, const int8_t* L, const double* NR,
                               int32_t T_m, int32_t B, int64_t N, int32_t n_bins, int32_t Kmax,
                               int32_t legs, void* workspace) {
  int r = prep(ctx);
  if (r) return r;
  if (!L || !NR || !workspace || nJ < 1 || nJ > SEG_MAXJ || T_m < 0 || B < 1 || N <= 0 ||
      Kmax < 1 || Kmax > TO_MAXK || (int64_t)T_m * nJ * B > 0x7FFFFFFF)
    return set_err(ctx, CSM_E_INVAL, "csm_cohort_sums_js_grouped: bad arguments (nJ=%d T_m=%d B=%d "
                   "N=%lld Kmax=%d; 1 <= nJ <= %d)", nJ, T_m, B, (long long)N, Kmax, SEG_MAXJ);
  if (legs && N > SEG_MAXN)
    return set_err(ctx, CSM_E_INVAL, "csm_cohort_sums_js_grouped: legs on rows of <= %d assets "
                   "(N=%lld)", SEG_MAXN, (long long)N);
  if (T_m == 0) return CSM_OK;
  const PfLayout lay = pf_layout(T_m, nJ * B, N, n_bins, Kmax);
  const bool shared = g_tune_cohort_seg && lay.seg && lay.p.C == 1 && !lay.p.kpar &&
                      (legs ? nJ * Kmax * 4 : nJ * Kmax * (n_bins + 1)) <= SEG_MAXKD &&
                      (n_bins == 2 || n_bins == 3 || n_bins == 4 || n_bins == 5 || n_bins == 10 ||
                       n_bins == 20 || n_bins == 30);
  if (!shared)   // the grouped pass with every group reading the one next_ret block
    return cohort_sums(ctx, L, NR, nullptr, T_m, nJ * B, N, n_bins, Kmax, workspace, legs != 0,
                       pan_grouped(nJ, B, T_m, N, true));
  hipStream_t st = ctx->stream;
  char* ws = (char*)workspace;
  switch (n_bins) {
#define PJ_CASE(NBV) case NBV: launch_cohort_js<NBV>(st, lay.p, nJ, &L, NR, T_m, B, N, Kmax, &ws, lay.swr * 8, lay.sw * 8, lay.fw * 8, lay.perm_b, lay.off_b, legs != 0, true, lay.lm_b); break;
    PJ_CASE(2) PJ_CASE(3) PJ_CASE(4) PJ_CASE(5) PJ_CASE(10) PJ_CASE(20) PJ_CASE(30)
#undef PJ_CASE
  }
  LAUNCH_CHECK(ctx, "k_cohort_seg (shared next_ret, grouped)");
  fill_i32(st, (int32_t*)(ws + lay.lw_b), 1, legs ? 2 : n_bins);
  planes_note(ctx, workspace, legs_masks(lay, legs != 0, N, Kmax, n_bins) ? 1u : 0u);
  return CSM_OK;
}

int64_t csm_portfolio_plan(int32_t T_m, int32_t B, int64_t N, int32_t n_bins, int32_t K) {
  if (T_m < 0 || B < 1 || N <= 0 || n_bins < 1 || K < 1) return -1;
  const PfPlan p = pf_plan(T_m, B, N, K, n_bins);
  return (int64_t)p.C | ((int64_t)p.Ct << 32);
}

int csm_cohort_sums_legs(csm_ctx* ctx, const int8_t* L, const double* NR, const double* W,
                         int32_t T_m, int32_t B, int64_t N, int32_t n_bins, int32_t Kmax,
                         void* workspace) {
  if (N > SEG_MAXN)
    return set_err(ctx, CSM_E_INVAL, "csm_cohort_sums_legs: rows of <= %d assets (N=%lld)", SEG_MAXN,
                   (long long)N);
  return cohort_sums(ctx, L, NR, W, T_m, B, N, n_bins, Kmax, workspace, true, pan_plain(B, N));
}

// Whether the cohort pass of this layout ran k_label_sort_legs_ew (legs, equal weights, N % 4 ==
// 0, the segment path -- launch_cohort's and launch_cohort_js's choice), so the workspace holds
// the leg bitplanes.  (Tune knobs are set before a workspace is sized, csmom.h.)
static bool legs_masks(const PfLayout& lay, bool legs, int64_t N, int Kmax, int n_bins) {
  return g_tune_turn_mask && legs && (N & 3) == 0 && lay.seg && g_tune_cohort_seg &&
         !lay.p.kpar && (int64_t)Kmax * (n_bins + 1) <= SEG_MAXKD &&
         (lay.p.Ct == 1 || lay.p.CHt % 256 == 0);
}

// The cohort pass records, per workspace, whether it wrote the leg bitplanes (the
// turnover pass must not infer it from knobs that may have changed in between; bit 0).  (The
// partials' layout is a word in the workspace itself, PfLayout::lw_b.)
static void planes_note(csm_ctx* ctx, void* ws, unsigned bits) {
  int hit = -1;
  for (int i = 0; i < 32; ++i)
    if (ctx->planes_ws[i] == ws) { hit = i; break; }
  if (bits && hit < 0) {
    hit = ctx->planes_next;
    ctx->planes_ws[hit] = ws;
    ctx->planes_next = (ctx->planes_next + 1) % 32;
  } else if (!bits && hit >= 0) {
    ctx->planes_ws[hit] = nullptr;
  }
  if (hit >= 0) ctx->planes_bits[hit] = (unsigned char)bits;
}
static unsigned ws_bits(const csm_ctx* ctx, const void* ws) {
  for (int i = 0; i < 32; ++i)
    if (ws && ctx->planes_ws[i] == ws) return ctx->planes_bits[i];
  return 0u;
}
static bool planes_have(const csm_ctx* ctx, const void* ws) { return (ws_bits(ctx, ws) & 1u) != 0; }

static int portfolio_from_cohorts(csm_ctx* ctx, const int8_t* L, const double* W,
                                  int32_t T_m, int32_t B, int64_t N, int32_t n_bins,
                                  int32_t Kmax, int32_t nK, const int32_t* Ks,
                                  double half_spread, double k_impact, double aum,
                                  const double* ADV, const double* SIG, double* PR, double* LS,
                                  double* TURN, double* COST, double* NET, void* workspace,
                                  bool legs, int32_t* need_full, const PanAddr& pa) {
  int r = prep(ctx);
  if (r) return r;
  bool ks_ok = Ks && nK >= 1;
  for (int q = 0; ks_ok && q < nK; ++q) ks_ok = Ks[q] >= 1 && Ks[q] <= Kmax;
  if (!L || !PR || !LS || !workspace || T_m < 0 || B < 1 || N <= 0 || !ks_ok ||
      Kmax > TO_MAXK || n_bins < 2 || n_bins > 30 || !(half_spread >= 0.0) ||
      !(k_impact >= 0.0) || !(aum >= 0.0) || (int64_t)T_m * B > 0x7FFFFFFF)
    return set_err(ctx, CSM_E_INVAL, "csm_portfolio_from_cohorts: bad arguments (T_m=%d B=%d N=%lld nK=%d Kmax=%d)",
                   T_m, B, (long long)N, nK, Kmax);
  if (NET && !COST)
    return set_err(ctx, CSM_E_INVAL, "csm_portfolio: NET needs COST");
  if (T_m == 0) return CSM_OK;
  const PfLayout lay = pf_layout(T_m, B, N, n_bins, Kmax);
  double* ws = (double*)workspace;
  hipStream_t st = ctx->stream;
  const bool costs = TURN || COST;
  const int64_t rb = (int64_t)T_m * B;   // cells of one [T_m][B] output
  for (int q0 = 0; q0 < nK; q0 += TO_MAXQ) {
    KSet ks;
    ks.n = nK - q0 < TO_MAXQ ? nK - q0 : TO_MAXQ;
    for (int q = 0; q < TO_MAXQ; ++q) ks.K[q] = q < ks.n ? Ks[q0 + q] : 1;
    if (costs) {
      const bool imp = ADV && aum > 0.0;
      const int64_t nblk = lay.p.Ct * lay.rows;
      // general rows: the steady launch appends them to a work list that a persistent launch
      // walks (C5 112.0 -> 108.9, C3 1.438 -> 1.405 ms/step against a second full grid)
      int32_t* gen_count = (int32_t*)((char*)workspace + lay.gen_b);
      int32_t* gen_list = gen_count + 1;
      // the counter is reset by k_turn_prep's first thread (a kernel node, replay-safe), or --
      // gen_reset 0, the diagnosis of tests/test_gpu_capture.py -- by hipMemsetAsync
      if (!g_tune_gen_reset)
        HIP_CHECK(ctx, hipMemsetAsync(gen_count, 0, sizeof(int32_t), st));
      const unsigned gen_grid = (unsigned)std::min<int64_t>(nblk, g_tune_turn_gen_grid);
      // steady rows take their factors from k_turn_prep (no per-workgroup prologue: equal
      // weights since round 2, value weights / impact costs since round 4)
      const bool prep = true;
      double* TPv = prep ? (double*)((char*)workspace + lay.tp_b) : nullptr;
      uint32_t* TPm = prep ? (uint32_t*)((char*)workspace + lay.tpm_b) : nullptr;
      if (prep)
        hipLaunchKernelGGL(k_turn_prep, dim3((unsigned)((lay.rows + TP_THREADS - 1) / TP_THREADS)),
                           dim3(TP_THREADS), 0, st, (const double*)(ws + lay.fwt), T_m, B, ks, TPv,
                           TPm, g_tune_gen_reset ? gen_count : (int32_t*)nullptr, lay.p.Ct,
                           ws + lay.turn, ws + lay.cost);
      for (int gen = 0; gen < 2; ++gen) {
        int kq = 0;
        for (int q = 0; q < ks.n; ++q) kq = ks.K[q] > kq ? ks.K[q] : kq;
        auto kern = gen ? (W ? (imp ? k_turnover<true, true, true> : k_turnover<true, false, true>)
                             : (imp ? k_turnover<false, true, true>
                                    : (kq <= 31 && (N & 3) == 0 ? k_turnover<false, false, true, true>
                                                                : k_turnover<false, false, true>)))
                        : (W ? (imp ? k_turnover<true, true, false> : k_turnover<true, false, false>)
                             : (imp ? k_turnover<false, true, false> : k_turnover<false, false, false>));
        // value weights shared by the groups of a grouped batch: the steady rows of a weight
        // panel's G groups in one workgroup (weights / ADV loaded once for them)
        if (!gen && W && g_tune_turn_vwg && pa.Bg < pa.B && pa.B / pa.Bg <= TO_MAXG) {
          hipLaunchKernelGGL(imp ? k_turnover_vwg<true> : k_turnover_vwg<false>,
                             dim3((unsigned)((int64_t)T_m * pa.Bg * lay.p.Ct)), dim3(PF_THREADS), 0,
                             st, L, W, T_m, B, N, ks, n_bins, lay.p.CHt, lay.p.Ct, half_spread,
                             k_impact, aum, ADV, SIG, ws + lay.turn, ws + lay.cost, gen_list,
                             gen_count, (const double*)TPv, (const uint32_t*)TPm, pa);
          continue;
        }
        // equal-weight legs after the legs label sort: the steady rows' member counts from the
        // leg bitplanes it wrote (k_turnover_ew_mask), not from label bytes
        if (!gen && !W && !imp && legs_masks(lay, legs, N, Kmax, n_bins) &&
            planes_have(ctx, workspace)) {
          hipLaunchKernelGGL(k_turnover_ew_mask, dim3((unsigned)((nblk + TM_WAVES - 1) / TM_WAVES)),
                             dim3(64 * TM_WAVES), 0, st,
                             (const uint64_t*)((char*)workspace + lay.lm_b), lay.nwm, T_m, B, N, ks,
                             lay.p.CHt, lay.p.Ct, half_spread, ws + lay.turn, ws + lay.cost,
                             gen_list, gen_count, (const double*)TPv, (const uint32_t*)TPm);
          continue;
        }
        hipLaunchKernelGGL(kern, dim3(gen ? gen_grid : (unsigned)nblk), dim3(PF_THREADS), 0, st,
                           L, W, (const double*)(ws + lay.fwt), T_m, B, N, ks, Kmax, n_bins, 1,
                           lay.p.CHt, lay.p.Ct, half_spread, k_impact, aum, ADV, SIG,
                           ws + lay.turn, ws + lay.cost, gen_list, gen_count,
                           (const double*)TPv, (const uint32_t*)TPm, pa);
      }
      LAUNCH_CHECK(ctx, "k_turnover");
      if (g_gen_probe) {
        hipLaunchKernelGGL(k_copy_i32, dim3(1), dim3(64), 0, st, (const int32_t*)gen_count, g_gen_probe);
        LAUNCH_CHECK(ctx, "k_copy_i32");
      }
    }
    double* TURNq = TURN ? TURN + q0 * rb : nullptr;
    double* COSTq = COST ? COST + q0 * rb : nullptr;
    double* NETq = NET ? NET + q0 * rb : nullptr;
    double* PRq = PR + q0 * rb * n_bins;
    if (g_tune_overlap_rows && lay.p.C == 1)   // chunked plans (C3): k_overlap 0.71 vs 0.89 ms
      hipLaunchKernelGGL(k_overlap_rows, dim3((unsigned)(((int64_t)lay.rows * n_bins + 255) / 256)),
                         dim3(256), 0, st,
                         (const double*)(ws + lay.swr), (const double*)(ws + lay.sw), ks, Kmax,
                         n_bins, costs ? (const double*)(ws + lay.turn) : nullptr,
                         (const double*)(ws + lay.cost), lay.p.Ct, (int64_t)lay.rows, PRq, TURNq,
                         COSTq, legs ? 1 : 0, (const int32_t*)((char*)workspace + lay.lw_b));
    else
    hipLaunchKernelGGL(k_overlap, dim3((unsigned)(((int64_t)ks.n * lay.rows * n_bins + 255) / 256)),
                       dim3(256), 0, st,
                       (const double*)(ws + lay.swr), (const double*)(ws + lay.sw), ks, Kmax,
                       lay.p.C, n_bins, costs ? (const double*)(ws + lay.turn) : nullptr,
                       (const double*)(ws + lay.cost), lay.p.Ct, (int64_t)lay.rows, PRq, TURNq,
                       COSTq, legs ? 1 : 0, (const int32_t*)((char*)workspace + lay.lw_b));
    LAUNCH_CHECK(ctx, "k_overlap");
    if (B >= LS_PB && T_m > 0) {   // wide batches (C5): flags over month blocks, then one
      // thread per output (one workgroup per 64 panels: 227 -> 140 us per 800-panel launch)
      int32_t* lsf = (int32_t*)((char*)workspace + lay.lsf_b);
      fill_i32(st, lsf, (int64_t)ks.n * B, 0);
      hipLaunchKernelGGL(k_ls_flags, dim3((unsigned)((B + 63) / 64), (unsigned)ks.n,
                                          (unsigned)((T_m + LS_FM - 1) / LS_FM)),
                         dim3(256), 0, st, (const double*)PRq, T_m, B, n_bins, lsf);
      hipLaunchKernelGGL(k_ls_rows, dim3((unsigned)(((int64_t)ks.n * T_m * B + 255) / 256)),
                         dim3(256), 0, st, (const double*)PRq, T_m, B, n_bins, ks.n,
                         (const int32_t*)lsf, LS + q0 * rb, (const double*)COSTq, NETq,
                         legs ? need_full : nullptr);
    } else
      hipLaunchKernelGGL(k_ls, dim3((unsigned)B, (unsigned)ks.n), dim3(256), 0, st,
                         (const double*)PRq, T_m, B, n_bins, LS + q0 * rb, (const double*)COSTq,
                         NETq, legs ? need_full : nullptr);
    LAUNCH_CHECK(ctx, "k_ls");
  }
  return CSM_OK;
}

int csm_portfolio_from_cohorts_multi(csm_ctx* ctx, const int8_t* L, const double* W,
                                     int32_t T_m, int32_t B, int64_t N, int32_t n_bins,
                                     int32_t Kmax, int32_t nK, const int32_t* Ks,
                                     double half_spread, double k_impact, double aum,
                                     const double* ADV, const double* SIG, double* PR, double* LS,
                                     double* TURN, double* COST, double* NET, void* workspace) {
  return portfolio_from_cohorts(ctx, L, W, T_m, B, N, n_bins, Kmax, nK, Ks, half_spread, k_impact,
                                aum, ADV, SIG, PR, LS, TURN, COST, NET, workspace, false, nullptr,
                                pan_plain(B, N));
}

int csm_portfolio_from_cohorts_legs(csm_ctx* ctx, const int8_t* L, const double* W,
                                    int32_t T_m, int32_t B, int64_t N, int32_t n_bins,
                                    int32_t Kmax, int32_t nK, const int32_t* Ks,
                                    double half_spread, double k_impact, double aum,
                                    const double* ADV, const double* SIG, double* PR, double* LS,
                                    double* TURN, double* COST, double* NET, void* workspace,
                                    int32_t* need_full) {
  if (!need_full)
    return set_err(ctx, CSM_E_INVAL, "csm_portfolio_from_cohorts_legs: need_full is required");
  return portfolio_from_cohorts(ctx, L, W, T_m, B, N, n_bins, Kmax, nK, Ks, half_spread, k_impact,
                                aum, ADV, SIG, PR, LS, TURN, COST, NET, workspace, true, need_full,
                                pan_plain(B, N));
}

int csm_cohort_sums_grouped(csm_ctx* ctx, int32_t G, const int8_t* L, const double* NR,
                            const double* W, int32_t T_m, int32_t Bg, int64_t N, int32_t n_bins,
                            int32_t Kmax, int32_t legs, void* workspace) {
  if (G < 1 || Bg < 1 || (int64_t)G * Bg > 0x7FFFFFFF || (legs && N > SEG_MAXN))
    return set_err(ctx, CSM_E_INVAL, "csm_cohort_sums_grouped: bad arguments (G=%d Bg=%d N=%lld legs=%d;"
                   " legs on rows of <= %d assets)", G, Bg, (long long)N, legs, SEG_MAXN);
  return cohort_sums(ctx, L, NR, W, T_m, G * Bg, N, n_bins, Kmax, workspace, legs != 0,
                     pan_grouped(G, Bg, T_m, N));
}

int csm_portfolio_from_cohorts_grouped(csm_ctx* ctx, int32_t G, const int8_t* L, const double* W,
                                       int32_t T_m, int32_t Bg, int64_t N, int32_t n_bins,
                                       int32_t Kmax, int32_t nK, const int32_t* Ks,
                                       double half_spread, double k_impact, double aum,
                                       const double* ADV, const double* SIG, double* PR,
                                       double* LS, double* TURN, double* COST, double* NET,
                                       void* workspace, int32_t legs, int32_t* need_full) {
  if (G < 1 || Bg < 1 || (int64_t)G * Bg > 0x7FFFFFFF || (legs && !need_full))
    return set_err(ctx, CSM_E_INVAL, "csm_portfolio_from_cohorts_grouped: bad arguments (G=%d Bg=%d "
                   "legs=%d; legs needs need_full)", G, Bg, legs);
  return portfolio_from_cohorts(ctx, L, W, T_m, G * Bg, N, n_bins, Kmax, nK, Ks, half_spread,
                                k_impact, aum, ADV, SIG, PR, LS, TURN, COST, NET, workspace,
                                legs != 0, legs ? need_full : nullptr, pan_grouped(G, Bg, T_m, N));
}

int csm_portfolio_from_cohorts(csm_ctx* ctx, const int8_t* L, const double* W, int32_t T_m,
                               int32_t B, int64_t N, int32_t n_bins, int32_t Kmax, int32_t K,
                               double half_spread, double k_impact, double aum, const double* ADV,
                               const double* SIG, double* PR, double* LS, double* TURN,
                               double* COST, double* NET, void* workspace) {
  const int32_t ks[1] = {K};
  return csm_portfolio_from_cohorts_multi(ctx, L, W, T_m, B, N, n_bins, Kmax, 1, ks, half_spread,
                                          k_impact, aum, ADV, SIG, PR, LS, TURN, COST, NET,
                                          workspace);
}

int csm_portfolio(csm_ctx* ctx, const int8_t* L, const double* NR, const double* W, int32_t T_m,
                  int32_t B, int64_t N, int32_t n_bins, int32_t K, double half_spread,
                  double k_impact, double aum, const double* ADV, const double* SIG, double* PR,
                  double* LS, double* TURN, double* COST, double* NET, void* workspace) {
  int r = csm_cohort_sums(ctx, L, NR, W, T_m, B, N, n_bins, K, workspace);
  if (r) return r;
  if (!PR || !LS)
    return set_err(ctx, CSM_E_INVAL, "csm_portfolio: PR and LS are required");
  return csm_portfolio_from_cohorts(ctx, L, W, T_m, B, N, n_bins, K, K, half_spread, k_impact,
                                    aum, ADV, SIG, PR, LS, TURN, COST, NET, workspace);
}

int csm_bootstrap(csm_ctx* ctx, const double* R, int32_t T_m, int64_t N, int32_t B, int64_t b0,
                  uint64_t seed, double mean_block, double p0, int32_t* src, double* PMb) {
  int r = prep(ctx);
  if (r) return r;
  if (!R || !src || !PMb || T_m < 1 || N <= 0 || B < 1 || b0 < 0 || !(mean_block >= 1.0))
    return set_err(ctx, CSM_E_INVAL, "csm_bootstrap: bad arguments (T_m=%d N=%lld B=%d)", T_m,
                   (long long)N, B);
  hipLaunchKernelGGL(k_bootstrap_index, dim3((unsigned)((B + 255) / 256)), dim3(256), 0,
                     ctx->stream, T_m, B, b0, seed, 1.0 / mean_block, src);
  LAUNCH_CHECK(ctx, "k_bootstrap_index");
  const int64_t cells = (int64_t)B * N;
  hipLaunchKernelGGL(k_bootstrap_panel, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0,
                     ctx->stream, R, T_m, B, N, (const int32_t*)src, p0, PMb);
  LAUNCH_CHECK(ctx, "k_bootstrap_panel");
  return CSM_OK;
}

}  // extern "C"

// =====================================================================================
// Share-turnover features (src/features.py:60-107) and the momentum x volume double sort
// (LeSw00 section II; rules T1, T2 in oracle/features_oracle.py).
// =====================================================================================
#define TF_THREADS 128
#define TF_MAXLB 48

// One thread per asset walks its present rows in order.  turn_avg is pandas 2.3.3's
// roll_mean (fixed window, min_periods = 1) restated: Kahan-compensated add / remove with
// separate compensations, the consecutive-same-value and all-positive / all-negative
// fix-ups -- bit for bit (-ffp-contract=off keeps every product / sum rounded on its own).
__global__ __launch_bounds__(TF_THREADS) void k_turn_features(
    const double* __restrict__ PM, const double* __restrict__ VOL, const double* __restrict__ so,
    const double* __restrict__ mcap, int T_m, int64_t N, int lb, double* __restrict__ ADV,
    double* __restrict__ SH, double* __restrict__ TURN, double* __restrict__ TAVG) {
  __shared__ double ring[TF_MAXLB * TF_THREADS];
  const int tid = threadIdx.x;
  const int64_t a = (int64_t)blockIdx.x * TF_THREADS + tid;
  if (a >= N) return;
  double* rg = ring + tid;
  const double s_out = so[a], m_cap = mcap[a];
  int n = 0;                                  // present rows so far
  int64_t nobs = 0, neg = 0, same = 0;
  double sx = 0.0, cadd = 0.0, crem = 0.0, prev = 0.0;
  for (int t = 0; t < T_m; ++t) {
    const int64_t o = (int64_t)t * N + a;
    const double p = PM[o];
    if (is_absent(p)) {
      ADV[o] = qnan(); SH[o] = qnan(); TURN[o] = qnan(); TAVG[o] = qnan();
      continue;
    }
    double vol = VOL[o];
    vol = vol == vol ? vol : 0.0;
    const double adv = vol / 21.0;
    double sh = qnan();
    if (s_out == s_out) {
      sh = s_out;
    } else if (m_cap != 0.0 && p == p && p > 0.0) {   // NaN market cap is truthy in Python
      const double q = m_cap / p;
      sh = (q == q && fabs(q) < INFINITY) ? trunc(q) : qnan();
    }
    const double tv = sh > 0.0 ? adv / sh : qnan();
    ADV[o] = adv; SH[o] = sh; TURN[o] = tv;
    // rolling mean over the last lb present rows
    if (n == 0) {
      nobs = neg = same = 0;
      sx = cadd = crem = 0.0;
      prev = tv;
    } else if (n >= lb) {
      const double v = rg[((n - lb) % lb) * TF_THREADS];   // leaves the window
      if (v == v) {
        --nobs;
        const double y = -v - crem;
        const double u = sx + y;
        crem = (u - sx) - y;
        sx = u;
        if (signbit(v)) --neg;
      }
    }
    if (tv == tv) {
      ++nobs;
      const double y = tv - cadd;
      const double u = sx + y;
      cadd = (u - sx) - y;
      sx = u;
      if (signbit(tv)) ++neg;
      same = (tv == prev) ? same + 1 : 1;
      prev = tv;
    }
    rg[(n % lb) * TF_THREADS] = tv;
    ++n;
    double r = qnan();
    if (nobs >= 1) {
      r = sx / (double)nobs;
      if (same >= nobs) r = prev;
      else if (neg == 0 && r < 0.0) r = 0.0;
      else if (neg == nobs && r > 0.0) r = 0.0;
    }
    TAVG[o] = r;
  }
}

// X masked to the rows where M is valid (the double sort's tercile universe)
__global__ __launch_bounds__(256) void k_mask_nan(const double* __restrict__ M,
                                                  const double* __restrict__ X, int64_t n,
                                                  double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = M[i] == M[i] ? X[i] : qnan();
}

__global__ __launch_bounds__(256) void k_combine_labels(const int8_t* __restrict__ Lm,
                                                        const int8_t* __restrict__ Lv,
                                                        int64_t n, int nv,
                                                        int8_t* __restrict__ Lc) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    const int a = Lm[i], b = Lv[i];
    Lc[i] = (a >= 0 && b >= 0) ? (int8_t)(a * nv + b) : (int8_t)-1;
  }
}

extern "C" {

int csm_turnover_features(csm_ctx* ctx, const double* PM, const double* VOL, const double* so,
                          const double* mcap, int32_t T_m, int64_t N, int32_t lookback,
                          double* ADV, double* SH, double* TURN, double* TAVG) {
  int r = prep(ctx);
  if (r) return r;
  if (!PM || !VOL || !so || !mcap || !ADV || !SH || !TURN || !TAVG || T_m < 0 || N <= 0 ||
      lookback < 1 || lookback > TF_MAXLB)
    return set_err(ctx, CSM_E_INVAL, "csm_turnover_features: bad arguments (T_m=%d N=%lld lookback=%d, max %d)",
                   T_m, (long long)N, lookback, TF_MAXLB);
  if (T_m == 0) return CSM_OK;
  hipLaunchKernelGGL(k_turn_features, dim3((unsigned)((N + TF_THREADS - 1) / TF_THREADS)),
                     dim3(TF_THREADS), 0, ctx->stream, PM, VOL, so, mcap, T_m, N, lookback, ADV,
                     SH, TURN, TAVG);
  LAUNCH_CHECK(ctx, "k_turn_features");
  return CSM_OK;
}

int csm_double_sort_labels(csm_ctx* ctx, const double* M, const double* X, const int8_t* Lm,
                           const int8_t* Lv, int32_t T_m, int64_t N, int32_t n_vol, double* Xm,
                           int8_t* Lc) {
  int r = prep(ctx);
  if (r) return r;
  if (!M || T_m < 0 || N <= 0 || n_vol < 1 || (!Xm && !Lc) || (Xm && !X) || (Lc && (!Lm || !Lv)))
    return set_err(ctx, CSM_E_INVAL, "csm_double_sort_labels: bad arguments");
  const int64_t n = (int64_t)T_m * N;
  if (n == 0) return CSM_OK;
  const unsigned g = (unsigned)((n + 255) / 256);
  if (Xm) {
    hipLaunchKernelGGL(k_mask_nan, dim3(g), dim3(256), 0, ctx->stream, M, X, n, Xm);
    LAUNCH_CHECK(ctx, "k_mask_nan");
  }
  if (Lc) {
    hipLaunchKernelGGL(k_combine_labels, dim3(g), dim3(256), 0, ctx->stream, Lm, Lv, n, n_vol, Lc);
    LAUNCH_CHECK(ctx, "k_combine_labels");
  }
  return CSM_OK;
}

}  // extern "C"

// =====================================================================================
// Per-(strategy, panel) performance summary of the long-short series, the sweep's last step
// (src/utils.py:8-16 Sharpe at `freq` periods a year; NaN months dropped, run_demo.py:67):
// months, mean, Sharpe (ddof = 1), mean turnover, mean cost, mean and Sharpe of net.  One
// workgroup per (panel, strategy); fixed-order reductions (mean first, then squared
// deviations, as NumPy's std does).
// =====================================================================================
#define SUM_FIELDS 7
__device__ __forceinline__ double block_sum256(double v, double* scr) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) scr[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < PF_WAVES; ++w) s += scr[w];
  __syncthreads();
  return s;
}

__global__ __launch_bounds__(PF_THREADS) void k_summary(const double* __restrict__ LS,
                                                        const double* __restrict__ TURN,
                                                        const double* __restrict__ COST,
                                                        const double* __restrict__ NET, int T_m,
                                                        int B, double freq,
                                                        double* __restrict__ out) {
  __shared__ double scr[PF_WAVES];
  const int b = blockIdx.x, q = blockIdx.y;
  const int64_t base = (int64_t)q * T_m * B;
  double n = 0.0, s = 0.0, st = 0.0, sc = 0.0, sn = 0.0;
  for (int t = threadIdx.x; t < T_m; t += PF_THREADS) {
    const int64_t o = base + (int64_t)t * B + b;
    const double x = LS[o];
    if (x == x) {
      n += 1.0;
      s += x;
      if (TURN) { st += TURN[o]; sc += COST[o]; sn += NET[o]; }
    }
  }
  n = block_sum256(n, scr);
  s = block_sum256(s, scr);
  st = block_sum256(st, scr);
  sc = block_sum256(sc, scr);
  sn = block_sum256(sn, scr);
  const double mean = s / n, nmean = sn / n;
  double v = 0.0, vn = 0.0;
  for (int t = threadIdx.x; t < T_m; t += PF_THREADS) {
    const int64_t o = base + (int64_t)t * B + b;
    const double x = LS[o];
    if (x == x) {
      v += (x - mean) * (x - mean);
      if (NET) vn += (NET[o] - nmean) * (NET[o] - nmean);
    }
  }
  v = block_sum256(v, scr);
  vn = block_sum256(vn, scr);
  if (threadIdx.x == 0) {
    const double sd = sqrt(v / (n - 1.0)), sdn = sqrt(vn / (n - 1.0));
    const double rf = sqrt(freq);
    double* o = out + ((int64_t)q * B + b) * SUM_FIELDS;
    o[0] = n;
    o[1] = mean;
    o[2] = sd > 0.0 ? mean * freq / (sd * rf) : qnan();
    o[3] = TURN ? st / n : qnan();
    o[4] = TURN ? sc / n : qnan();
    o[5] = TURN ? nmean : qnan();
    o[6] = (TURN && sdn > 0.0) ? nmean * freq / (sdn * rf) : qnan();
  }
}

extern "C" {

int csm_summary(csm_ctx* ctx, const double* LS, const double* TURN, const double* COST,
                const double* NET, int32_t nS, int32_t T_m, int32_t B, double freq,
                double* out) {
  int r = prep(ctx);
  if (r) return r;
  if (!LS || !out || nS < 1 || T_m < 0 || B < 1 || !(freq > 0.0) ||
      ((TURN != nullptr) != (COST != nullptr)) || ((TURN != nullptr) != (NET != nullptr)))
    return set_err(ctx, CSM_E_INVAL, "csm_summary: bad arguments (nS=%d T_m=%d B=%d)", nS, T_m, B);
  hipLaunchKernelGGL(k_summary, dim3((unsigned)B, (unsigned)nS), dim3(PF_THREADS), 0, ctx->stream,
                     LS, TURN, COST, NET, T_m, B, freq, out);
  LAUNCH_CHECK(ctx, "k_summary");
  return CSM_OK;
}

}  // extern "C"
