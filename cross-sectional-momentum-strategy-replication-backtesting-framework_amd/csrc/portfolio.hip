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
//   k_overlap      one workgroup per (t, b): chunk partials summed in chunk order, cohort
//                  means -> overlapped decile returns (E2), turnover / cost totals
//   k_ls           one workgroup per panel: the reference's long-short rule
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

#define PF_THREADS 256
#define PF_WAVES (PF_THREADS / 64)
#define PF_CHUNK_MIN 256     // assets per chunk, at least one per thread
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

// -------------------------------------------------------------------------------- E1
// Cohort sums do not depend on the holding period: a pass with Kmax cohorts serves every
// K <= Kmax (the sweep runs one pass per J for all its K).  Per-lane decile accumulators
// live in registers (predicated adds; SW > 0 doubles as "the cohort has a valid member",
// weights being > 0, so no count is kept).
template <int NB, bool VW>
__global__ __launch_bounds__(PF_THREADS) void k_cohort(
    const int8_t* __restrict__ L, const double* __restrict__ NR, const double* __restrict__ W,
    int T_m, int B, int64_t N, int K, int C, int64_t CH, int kpar, double* __restrict__ SWRp,
    double* __restrict__ SWp, double* __restrict__ FWp) {
  __shared__ double red[PF_WAVES][2 * NB + 2];
  const int c = blockIdx.x;
  const int tb = blockIdx.y;
  const int t = tb / B, b = tb - t * B;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t a0 = (int64_t)c * CH;
  const int64_t a1 = a0 + CH < N ? a0 + CH : N;
  const int64_t rt = ((int64_t)t * B + b) * N;
  const int k_lo = kpar ? (int)blockIdx.z : 0, k_hi = kpar ? k_lo + 1 : K;
  for (int k = k_lo; k < k_hi; ++k) {
    const int s = t - k;
    const int64_t ob = (((int64_t)tb * K + k) * C + c) * NB;
    if (s < 0) {
      if (tid < NB) { SWRp[ob + tid] = 0.0; SWp[ob + tid] = 0.0; }
      continue;
    }
    const int64_t rs = ((int64_t)s * B + b) * N;
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
        if (VW) wx[u] = in ? W[rs + i] : 0.0;
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
    double* __restrict__ SWp, double* __restrict__ FWp) {
  __shared__ double acc_r[PF_WAVES][AC_MAXKD];   // sum of w * r per (age, decile)
  __shared__ double acc_w[PF_WAVES][AC_MAXKD];   // sum of w (equal weight: the count)
  __shared__ double red[PF_WAVES][2];
  const int c = blockIdx.x;
  const int tb = blockIdx.y;
  const int t = tb / B, b = tb - t * B;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int KD = K * NB;
  for (int i = lane; i < KD; i += 64) { acc_r[wid][i] = 0.0; acc_w[wid][i] = 0.0; }
  const int64_t a0 = (int64_t)c * CH;
  const int64_t a1 = a0 + CH < N ? a0 + CH : N;
  const int64_t rt = ((int64_t)t * B + b) * N;
  const int kmax = t + 1 < K ? t + 1 : K;   // ages with a formation month s = t - k >= 0
  double ft = 0.0, fb = 0.0;
  double* ar = acc_r[wid];
  double* aw = acc_w[wid];
  __syncthreads();
  const int64_t rowstep = (int64_t)B * N;   // one month back
  for (int64_t a = a0 + tid; a < a1; a += PF_THREADS) {
    const double r = NR[rt + a];
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
        if (VW) wx[u] = k < kmax ? W[o] : 0.0;
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

__global__ __launch_bounds__(PF_THREADS) void k_turnover(
    const int8_t* __restrict__ L, const double* __restrict__ W, const double* __restrict__ FWp,
    int T_m, int B, int64_t N, KSet ks, int Kmax, int n_bins, int Cf, int64_t CH,
    double half_spread, double k_impact, double aum, const double* __restrict__ ADV,
    const double* __restrict__ SIG, double* __restrict__ TURNp, double* __restrict__ COSTp) {
  const int c = blockIdx.x, Ct = gridDim.x;
  const int tb = blockIdx.y;
  const int rows = gridDim.y;
  const int t = tb / B, b = tb - t * B;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  __shared__ double inv[2][TO_MAXK + 1];      // [leg][j]: 1/total of cohort s = t - j (0 = empty)
  __shared__ double sk[TO_MAXQ][2][2];        // [q][leg][month t, t-1]: 1/K_u (0 if none)
  __shared__ int full[TO_MAXQ][2];
  for (int j = tid; j <= Kmax; j += PF_THREADS) {
    const int s = t - j;
#pragma unroll
    for (int li = 0; li < 2; ++li) {
      double tot = 0.0;
      if (s >= 0)
        for (int cc = 0; cc < Cf; ++cc) tot += FWp[(((int64_t)s * B + b) * Cf + cc) * 2 + li];
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
    full[q][li] = (k1 == K && k0 == K) ? 1 : 0;
  }
  __syncthreads();
  const int64_t a0 = (int64_t)c * CH;
  const int64_t a1 = a0 + CH < N ? a0 + CH : N;
  const int64_t rt = ((int64_t)t * B + b) * N;
  const bool impact = ADV && aum > 0.0;
  const int nq = ks.n;
  double turn[TO_MAXQ], cost[TO_MAXQ];
#pragma unroll
  for (int q = 0; q < TO_MAXQ; ++q) { turn[q] = 0.0; cost[q] = 0.0; }
  auto charge = [&](int q, double dw, double adv, double unit_sig) {
    turn[q] += dw;
    double unit = half_spread;
    if (impact && adv > 0.0) {
      const double im = k_impact * unit_sig * sqrt(dw * aum / adv);
      unit = unit + ((im == im) ? im : 0.0);
    }
    cost[q] += dw * unit;
  };
  bool all_full = true;
  for (int q = 0; q < nq; ++q) all_full = all_full && full[q][0] && full[q][1];
  if (all_full) {
    // steady state: 2 cells per lane per trip, every load issued before use
    constexpr int TU = 2;
    for (int64_t i0 = a0 + tid; i0 < a1; i0 += TU * PF_THREADS) {
      int l1[TU], l0[TU][TO_MAXQ];
      double x1[TU], x0[TU][TO_MAXQ], adv[TU], sg[TU];
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        const int64_t a = i0 + (int64_t)u * PF_THREADS;
        const bool in = a < a1;
        l1[u] = in ? (int)L[rt + a] : -1;
        x1[u] = (W && in) ? W[rt + a] : 1.0;
#pragma unroll
        for (int q = 0; q < TO_MAXQ; ++q) {
          const bool use = in && q < nq;
          const int64_t rk = ((int64_t)(t - (use ? ks.K[q] : 0)) * B + b) * N;
          l0[u][q] = use ? (int)L[rk + a] : -1;
          x0[u][q] = (W && use) ? W[rk + a] : 1.0;
        }
        adv[u] = (impact && in) ? ADV[rt + a] : 0.0;
        sg[u] = (impact && SIG && in) ? SIG[rt + a] : 0.02;
      }
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        const double vw1 = (x1[u] > 0.0 && x1[u] < INFINITY) ? x1[u] : 0.0;
        const double unit_sig = sg[u] == sg[u] ? sg[u] : 0.02;
#pragma unroll
        for (int q = 0; q < TO_MAXQ; ++q) {
          if (q >= nq) break;
          const double vw0 = (x0[u][q] > 0.0 && x0[u][q] < INFINITY) ? x0[u][q] : 0.0;
          const int K = ks.K[q];
#pragma unroll
          for (int li = 0; li < 2; ++li) {
            const int d = li == 0 ? n_bins - 1 : 0;
            const double w1 = (l1[u] == d ? vw1 : 0.0) * inv[li][0];
            const double w0 = (l0[u][q] == d ? vw0 : 0.0) * inv[li][K];
            charge(q, fabs(w1 - w0) * sk[q][li][0], adv[u], unit_sig);
          }
        }
      }
    }
  } else {
    for (int64_t a = a0 + tid; a < a1; a += PF_THREADS) {
      double unit_sig = 0.02, adv = 0.0;
      if (impact) {
        adv = ADV[rt + a];
        if (SIG) { const double sg = SIG[rt + a]; unit_sig = (sg == sg) ? sg : 0.02; }
      }
      for (int q = 0; q < nq; ++q) {
        const int K = ks.K[q];
#pragma unroll
        for (int li = 0; li < 2; ++li) {
          const int d = li == 0 ? n_bins - 1 : 0;
          double dw;
          if (full[q][li]) {
            const int64_t o1 = rt + a, o0 = ((int64_t)(t - K) * B + b) * N + a;
            const double w1 = member_w(L[o1], d, W, o1) * inv[li][0];
            const double w0 = member_w(L[o0], d, W, o0) * inv[li][K];
            dw = fabs(w1 - w0) * sk[q][li][0];
          } else {
            double x1 = 0.0, x0 = 0.0;
            for (int j = 0; j <= K; ++j) {
              const double iv = inv[li][j];
              if (iv == 0.0) continue;
              const int64_t o = ((int64_t)(t - j) * B + b) * N + a;
              const double w = member_w(L[o], d, W, o) * iv;
              if (j < K) x1 += w;
              if (j >= 1) x0 += w;
            }
            dw = fabs(x1 * sk[q][li][0] - x0 * sk[q][li][1]);
          }
          charge(q, dw, adv, unit_sig);
        }
      }
    }
  }
  __shared__ double red[PF_WAVES][2 * TO_MAXQ];
#pragma unroll
  for (int q = 0; q < TO_MAXQ; ++q) {
    if (q >= nq) break;
    const double x1 = wave_sum(turn[q]), y1 = wave_sum(cost[q]);
    if (lane == 0) { red[wid][2 * q] = x1; red[wid][2 * q + 1] = y1; }
  }
  __syncthreads();
  if (tid < nq) {
    const int q = tid;
    double x = 0.0, y = 0.0;
    for (int w2 = 0; w2 < PF_WAVES; ++w2) { x += red[w2][2 * q]; y += red[w2][2 * q + 1]; }
    TURNp[((int64_t)q * rows + tb) * Ct + c] = 0.5 * x;
    COSTp[((int64_t)q * rows + tb) * Ct + c] = y;
  }
}

// ------------------------------------------------------------------------------ E2, E3
// one 64-lane workgroup per (t, b, holding period q of the K set): lane d < nb combines decile
// d over the chunks and the cohorts; lane 0 also totals the turnover / cost partials.  Output
// q lands at offset q * rows of the [nK][T_m][B] stacks (PR: [nK][T_m][B][nb]).
__global__ __launch_bounds__(64) void k_overlap(
    const double* __restrict__ SWRp, const double* __restrict__ SWp, KSet ks, int Kmax, int C,
    int nb, const double* __restrict__ TURNp, const double* __restrict__ COSTp, int Ct,
    int64_t rows, double* __restrict__ PR, double* __restrict__ TURN, double* __restrict__ COST) {
  const int64_t tb = blockIdx.x;
  const int q = blockIdx.y;
  const int K = ks.K[q];
  const int d = threadIdx.x;
  if (d < nb) {
    double acc = 0.0;
    int n = 0;
    for (int k = 0; k < K; ++k) {
      double x = 0.0, y = 0.0;
      for (int c = 0; c < C; ++c) {
        const int64_t o = ((tb * Kmax + k) * C + c) * nb + d;
        x += SWRp[o];
        y += SWp[o];
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

// one workgroup per (panel b, holding period q): the reference's long-short rule on PR[q].
__global__ __launch_bounds__(256) void k_ls(const double* __restrict__ PR, int T_m, int B, int nb,
                                            double* __restrict__ LS,
                                            const double* __restrict__ COST,
                                            double* __restrict__ NET) {
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

// ------------------------------------------------------------------------------- C ABI
// 1: cohort sums through per-wave LDS atomics (k_cohort_lds) where they fit; 0: registers
static int g_tune_cohort_lds = 1;

struct PfPlan {
  int C, kpar, Ct;
  int64_t CH, CHt;
};

// Enough workgroups to fill 256 CUs several times over, chunks of >= PF_CHUNK_MIN assets.
static PfPlan pf_plan(int32_t T_m, int32_t B, int64_t N, int32_t K) {
  PfPlan p;
  const int64_t rows = (int64_t)T_m * B;
  const int64_t want = 4096;
  const int64_t cmax = (N + PF_CHUNK_MIN - 1) / PF_CHUNK_MIN;
  // the chunking depends on (rows, N) only, so a cohort pass gives the same partial sums
  // whatever Kmax it was planned for (portfolio_multi == per-K portfolio, bit for bit)
  // (cohort-parallel grids, kpar = 1, made tens of thousands of tiny workgroups at C3 and
  // ran slower than one workgroup walking its K cohorts over a chunk.)
  (void)K;
  p.kpar = 0;
  int64_t C = (want + rows - 1) / rows;
  C = C < 1 ? 1 : (C > cmax ? cmax : C);
  p.C = (int)C;
  p.CH = (N + C - 1) / C;
  int64_t Ct = (want + rows - 1) / rows;
  Ct = Ct < 1 ? 1 : (Ct > cmax ? cmax : Ct);
  p.Ct = (int)Ct;
  p.CHt = (N + Ct - 1) / Ct;
  return p;
}

template <int NB>
static void launch_cohort(hipStream_t st, const PfPlan& pl, const int8_t* L, const double* NR,
                          const double* W, int T_m, int B, int64_t N, int K, double* SWRp,
                          double* SWp, double* FWp) {
  const dim3 g((unsigned)pl.C, (unsigned)(T_m * B), pl.kpar ? (unsigned)K : 1u);
  if (g_tune_cohort_lds && !pl.kpar && K * NB <= AC_MAXKD) {
    const dim3 g2((unsigned)pl.C, (unsigned)(T_m * B));
    if (W)
      hipLaunchKernelGGL((k_cohort_lds<NB, true>), g2, dim3(PF_THREADS), 0, st, L, NR, W, T_m, B,
                         N, K, pl.C, pl.CH, SWRp, SWp, FWp);
    else
      hipLaunchKernelGGL((k_cohort_lds<NB, false>), g2, dim3(PF_THREADS), 0, st, L, NR, W, T_m, B,
                         N, K, pl.C, pl.CH, SWRp, SWp, FWp);
    return;
  }
  if (W)
    hipLaunchKernelGGL((k_cohort<NB, true>), g, dim3(PF_THREADS), 0, st, L, NR, W, T_m, B, N, K,
                       pl.C, pl.CH, pl.kpar, SWRp, SWp, FWp);
  else
    hipLaunchKernelGGL((k_cohort<NB, false>), g, dim3(PF_THREADS), 0, st, L, NR, W, T_m, B, N, K,
                       pl.C, pl.CH, pl.kpar, SWRp, SWp, FWp);
}

// Workspace layout of the cohort partials for (T_m, B, N, n_bins, Kmax): SWRp, SWp
// [rows][Kmax][C][n_bins], FWp [rows][C][2], then the turnover partials [rows][Ct] x 2.
struct PfLayout {
  PfPlan p;
  int64_t rows, swr, sw, fw, turn, cost, bytes;
};
static PfLayout pf_layout(int32_t T_m, int32_t B, int64_t N, int32_t n_bins, int32_t Kmax) {
  PfLayout l;
  l.p = pf_plan(T_m, B, N, Kmax);
  l.rows = (int64_t)T_m * B;
  const int64_t cs = l.rows * Kmax * l.p.C * n_bins;
  l.swr = 0;
  l.sw = cs;
  l.fw = 2 * cs;
  l.turn = l.fw + l.rows * l.p.C * 2;                      // [TO_MAXQ][rows][Ct]
  l.cost = l.turn + (int64_t)TO_MAXQ * l.rows * l.p.Ct;
  l.bytes = (l.cost + (int64_t)TO_MAXQ * l.rows * l.p.Ct) * 8 + 256;
  return l;
}

extern "C" {

int csm_tune_portfolio(const char* key, int value) {
  if (key && !strcmp(key, "cohort_lds") && (value == 0 || value == 1)) {
    g_tune_cohort_lds = value;
    return CSM_OK;
  }
  return CSM_E_INVAL;
}

int64_t csm_portfolio_workspace(int32_t T_m, int32_t B, int64_t N, int32_t n_bins, int32_t K) {
  if (T_m < 0 || B < 1 || N <= 0 || n_bins < 1 || K < 1) return 0;
  return pf_layout(T_m, B, N, n_bins, K).bytes;
}

int csm_cohort_sums(csm_ctx* ctx, const int8_t* L, const double* NR, const double* W, int32_t T_m,
                    int32_t B, int64_t N, int32_t n_bins, int32_t Kmax, void* workspace) {
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
  switch (n_bins) {
#define PF_CASE(NBV) case NBV: launch_cohort<NBV>(st, lay.p, L, NR, W, T_m, B, N, Kmax, ws + lay.swr, ws + lay.sw, ws + lay.fw); break;
    PF_CASE(2) PF_CASE(3) PF_CASE(4) PF_CASE(5) PF_CASE(10) PF_CASE(20) PF_CASE(30)
#undef PF_CASE
    default:
      return set_err(ctx, CSM_E_INVAL, "csm_cohort_sums: n_bins=%d unsupported (2,3,4,5,10,20,30)", n_bins);
  }
  LAUNCH_CHECK(ctx, "k_cohort");
  return CSM_OK;
}

int csm_portfolio_from_cohorts_multi(csm_ctx* ctx, const int8_t* L, const double* W,
                                     int32_t T_m, int32_t B, int64_t N, int32_t n_bins,
                                     int32_t Kmax, int32_t nK, const int32_t* Ks,
                                     double half_spread, double k_impact, double aum,
                                     const double* ADV, const double* SIG, double* PR, double* LS,
                                     double* TURN, double* COST, double* NET, void* workspace) {
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
      hipLaunchKernelGGL(k_turnover, dim3((unsigned)lay.p.Ct, (unsigned)lay.rows),
                         dim3(PF_THREADS), 0, st, L, W, (const double*)(ws + lay.fw), T_m, B, N,
                         ks, Kmax, n_bins, lay.p.C, lay.p.CHt, half_spread, k_impact, aum, ADV,
                         SIG, ws + lay.turn, ws + lay.cost);
      LAUNCH_CHECK(ctx, "k_turnover");
    }
    double* TURNq = TURN ? TURN + q0 * rb : nullptr;
    double* COSTq = COST ? COST + q0 * rb : nullptr;
    double* NETq = NET ? NET + q0 * rb : nullptr;
    double* PRq = PR + q0 * rb * n_bins;
    hipLaunchKernelGGL(k_overlap, dim3((unsigned)lay.rows, (unsigned)ks.n), dim3(64), 0, st,
                       (const double*)(ws + lay.swr), (const double*)(ws + lay.sw), ks, Kmax,
                       lay.p.C, n_bins, costs ? (const double*)(ws + lay.turn) : nullptr,
                       (const double*)(ws + lay.cost), lay.p.Ct, (int64_t)lay.rows, PRq, TURNq,
                       COSTq);
    LAUNCH_CHECK(ctx, "k_overlap");
    hipLaunchKernelGGL(k_ls, dim3((unsigned)B, (unsigned)ks.n), dim3(256), 0, st,
                       (const double*)PRq, T_m, B, n_bins, LS + q0 * rb, (const double*)COSTq,
                       NETq);
    LAUNCH_CHECK(ctx, "k_ls");
  }
  return CSM_OK;
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
