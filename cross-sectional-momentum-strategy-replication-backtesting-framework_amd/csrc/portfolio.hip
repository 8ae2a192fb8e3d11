// portfolio.hip -- portfolio accounting beyond the reference's K = 1 equal-weight case
// (rules E1..E6 in oracle/portfolio_oracle.py and DESIGN.md 8).
//
//   k_cohort       one workgroup per (holding month t, panel b, cohort age k): decile sums of
//                  w * next_ret and w over the members of the cohort formed at t - k whose
//                  next_ret[t] is valid (E1), plus the formation totals of the two legs (k = 0)
//   k_turnover     one workgroup per (t, b): aggregate leg weights of the K overlapping
//                  cohorts at t and t - 1, |dw| summed into turnover and into the spread +
//                  square-root-impact cost of src/execution_models.py:4-12 (E4, E5)
//   k_overlap_ls   one workgroup per panel: cohort means -> overlapped decile returns (E2),
//                  the reference's long-short rule (run_demo.py:60-67) per panel (E3), net
//   k_bootstrap_*  stationary month bootstrap with a counter-based splitmix64 stream (E6)
//
// Panels are batched as [T_m][B][N] rows (B cross-sections per month), the sweep layout.
// Everything is HBM/latency-bound integer + fp64 work (no MFMA).  Reductions are per-lane
// fp64 partial sums combined by a fixed shuffle tree and then in wave order, so results are
// deterministic run to run.
#include "csm_common.h"

#define PF_THREADS 256
#define PF_WAVES (PF_THREADS / 64)
#define PF_MAXB 20

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
template <int NB>
__global__ __launch_bounds__(PF_THREADS) void k_cohort(
    const int8_t* __restrict__ L, const double* __restrict__ NR, const double* __restrict__ W,
    int T_m, int B, int64_t N, int K, double* __restrict__ SWR, double* __restrict__ SW,
    int32_t* __restrict__ CNT, double* __restrict__ FW) {
  const int k = blockIdx.x;
  const int tb = blockIdx.y;           // t * B + b
  const int t = tb / B, b = tb - t * B;
  const int s = t - k;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t obase = ((int64_t)tb * K + k) * NB;
  if (s < 0) {
    if (tid < NB) { SWR[obase + tid] = 0.0; SW[obase + tid] = 0.0; CNT[obase + tid] = 0; }
    return;
  }
  const int64_t rs = ((int64_t)s * B + b) * N;   // formation row
  const int64_t rt = ((int64_t)t * B + b) * N;   // holding row
  double swr[NB], sw[NB];
  int cn[NB];
#pragma unroll
  for (int d = 0; d < NB; ++d) { swr[d] = 0.0; sw[d] = 0.0; cn[d] = 0; }
  double ft = 0.0, fb = 0.0;  // formation totals of the top / bottom legs (k == 0 only)
  for (int64_t i = tid; i < N; i += PF_THREADS) {
    const int lab = L[rs + i];
    if (lab < 0) continue;
    const double r = NR[rt + i];
    double w = 1.0;
    if (W) {
      w = W[rs + i];
      if (!(w > 0.0 && w < INFINITY)) continue;
    }
    if (k == 0) {
      ft += lab == NB - 1 ? w : 0.0;
      fb += lab == 0 ? w : 0.0;
    }
    if (r != r) continue;
#pragma unroll
    for (int d = 0; d < NB; ++d) {
      const bool h = lab == d;
      swr[d] += h ? w * r : 0.0;
      sw[d] += h ? w : 0.0;
      cn[d] += h ? 1 : 0;
    }
  }
  __shared__ double red[PF_WAVES][2 * NB + 2];
  __shared__ int redc[PF_WAVES][NB];
#pragma unroll
  for (int d = 0; d < NB; ++d) {
    const double a = wave_sum(swr[d]), c = wave_sum(sw[d]);
    const int n = wave_sumi(cn[d]);
    if (lane == 0) { red[wid][d] = a; red[wid][NB + d] = c; redc[wid][d] = n; }
  }
  if (k == 0) {
    const double a = wave_sum(ft), c = wave_sum(fb);
    if (lane == 0) { red[wid][2 * NB] = a; red[wid][2 * NB + 1] = c; }
  }
  __syncthreads();
  if (tid < NB) {
    double a = 0.0, c = 0.0;
    int n = 0;
    for (int w2 = 0; w2 < PF_WAVES; ++w2) { a += red[w2][tid]; c += red[w2][NB + tid]; n += redc[w2][tid]; }
    SWR[obase + tid] = a;
    SW[obase + tid] = c;
    CNT[obase + tid] = n;
  }
  if (k == 0 && tid < 2) {
    double a = 0.0;
    for (int w2 = 0; w2 < PF_WAVES; ++w2) a += red[w2][2 * NB + tid];
    FW[(int64_t)tb * 2 + tid] = a;   // [t][b][leg]: leg 0 = top, 1 = bottom
  }
}

// ------------------------------------------------------------------------------ E4, E5
// Aggregate weight of asset a in leg (label d, totals index li) at month u (over the K
// cohorts u-K+1..u); returns 0 when no cohort is non-empty.
__device__ __forceinline__ double leg_weight(const int8_t* __restrict__ L,
                                             const double* __restrict__ W,
                                             const double* __restrict__ FW, int u, int B, int b,
                                             int64_t N, int64_t a, int K, int d, int li) {
  if (u < 0) return 0.0;
  double acc = 0.0;
  int kt = 0;
  for (int k = 0; k < K; ++k) {
    const int s = u - k;
    if (s < 0) break;
    const double tot = FW[((int64_t)s * B + b) * 2 + li];
    if (!(tot > 0.0)) continue;
    ++kt;
    const int64_t o = ((int64_t)s * B + b) * N + a;
    const double w = member_w(L[o], d, W, o);
    acc += w / tot;
  }
  return kt > 0 ? acc / (double)kt : 0.0;
}

__global__ __launch_bounds__(PF_THREADS) void k_turnover(
    const int8_t* __restrict__ L, const double* __restrict__ W, const double* __restrict__ FW,
    int T_m, int B, int64_t N, int K, int n_bins, double half_spread, double k_impact,
    double aum, const double* __restrict__ ADV, const double* __restrict__ SIG,
    double* __restrict__ TURN, double* __restrict__ COST) {
  const int tb = blockIdx.x;
  const int t = tb / B, b = tb - t * B;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t rt = ((int64_t)t * B + b) * N;
  const bool impact = ADV && aum > 0.0;
  double turn = 0.0, cost = 0.0;
  for (int64_t a = tid; a < N; a += PF_THREADS) {
    double unit_sig = 0.02, adv = 0.0;
    if (impact) {
      adv = ADV[rt + a];
      if (SIG) { const double sg = SIG[rt + a]; unit_sig = (sg == sg) ? sg : 0.02; }
    }
#pragma unroll
    for (int li = 0; li < 2; ++li) {
      const int d = li == 0 ? n_bins - 1 : 0;
      const double w1 = leg_weight(L, W, FW, t, B, b, N, a, K, d, li);
      const double w0 = leg_weight(L, W, FW, t - 1, B, b, N, a, K, d, li);
      const double dw = fabs(w1 - w0);
      turn += dw;
      double unit = half_spread;
      if (impact && adv > 0.0) {
        const double im = k_impact * unit_sig * sqrt(dw * aum / adv);
        unit = unit + ((im == im) ? im : 0.0);
      }
      cost += dw * unit;
    }
  }
  __shared__ double red[PF_WAVES][2];
  const double a = wave_sum(turn), c = wave_sum(cost);
  if (lane == 0) { red[wid][0] = a; red[wid][1] = c; }
  __syncthreads();
  if (tid == 0) {
    double x = 0.0, y = 0.0;
    for (int w2 = 0; w2 < PF_WAVES; ++w2) { x += red[w2][0]; y += red[w2][1]; }
    if (TURN) TURN[tb] = 0.5 * x;
    if (COST) COST[tb] = y;
  }
}

// ------------------------------------------------------------------------------ E2, E3
__global__ __launch_bounds__(PF_THREADS) void k_overlap_ls(
    const double* __restrict__ SWR, const double* __restrict__ SW,
    const int32_t* __restrict__ CNT, int T_m, int B, int K, int nb, double* __restrict__ PR,
    double* __restrict__ LS, const double* __restrict__ COST, double* __restrict__ NET) {
  const int b = blockIdx.x;
  __shared__ int has_lo, has_hi;
  if (threadIdx.x == 0) { has_lo = 0; has_hi = 0; }
  __syncthreads();
  for (int t = threadIdx.x; t < T_m; t += blockDim.x) {
    const int64_t tb = (int64_t)t * B + b;
    for (int d = 0; d < nb; ++d) {
      double s = 0.0;
      int n = 0;
      for (int k = 0; k < K; ++k) {
        const int64_t o = (tb * K + k) * nb + d;
        if (CNT[o] > 0) { s += SWR[o] / SW[o]; ++n; }
      }
      const double v = n > 0 ? s / (double)n : qnan();
      PR[tb * nb + d] = v;
      if (n > 0 && d == 0) atomicOr(&has_lo, 1);
      if (n > 0 && d == nb - 1) atomicOr(&has_hi, 1);
    }
  }
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
    if (NET) NET[tb] = v - (COST ? COST[tb] : 0.0);
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
template <int NB>
static void launch_cohort(hipStream_t st, const int8_t* L, const double* NR, const double* W,
                          int T_m, int B, int64_t N, int K, double* SWR, double* SW,
                          int32_t* CNT, double* FW) {
  hipLaunchKernelGGL(k_cohort<NB>, dim3(K, (unsigned)(T_m * B)), dim3(PF_THREADS), 0, st, L, NR,
                     W, T_m, B, N, K, SWR, SW, CNT, FW);
}

extern "C" {

int64_t csm_portfolio_workspace(int32_t T_m, int32_t B, int32_t n_bins, int32_t K) {
  if (T_m < 0 || B < 1 || n_bins < 1 || K < 1) return 0;
  const int64_t cells = (int64_t)T_m * B * K * n_bins;
  return cells * (8 + 8 + 4) + (int64_t)T_m * B * 2 * 8 + 64;
}

int csm_portfolio(csm_ctx* ctx, const int8_t* L, const double* NR, const double* W, int32_t T_m,
                  int32_t B, int64_t N, int32_t n_bins, int32_t K, double half_spread,
                  double k_impact, double aum, const double* ADV, const double* SIG, double* PR,
                  double* LS, double* TURN, double* COST, double* NET, void* workspace) {
  int r = prep(ctx);
  if (r) return r;
  if (!L || !NR || !PR || !LS || !workspace || T_m < 0 || B < 1 || N <= 0 || K < 1 ||
      K > 240 || !(half_spread >= 0.0) || !(k_impact >= 0.0) || !(aum >= 0.0) ||
      (int64_t)T_m * B > 0x7FFFFFFF)
    return set_err(ctx, CSM_E_INVAL, "csm_portfolio: bad arguments (T_m=%d B=%d N=%lld K=%d)",
                   T_m, B, (long long)N, K);
  if (NET && !COST)
    return set_err(ctx, CSM_E_INVAL, "csm_portfolio: NET needs COST");
  if (T_m == 0) return CSM_OK;
  const int64_t cells = (int64_t)T_m * B * K * n_bins;
  double* SWR = (double*)workspace;
  double* SW = SWR + cells;
  double* FW = SW + cells;
  int32_t* CNT = (int32_t*)(FW + (int64_t)T_m * B * 2);
  hipStream_t st = ctx->stream;
  switch (n_bins) {
    case 2: launch_cohort<2>(st, L, NR, W, T_m, B, N, K, SWR, SW, CNT, FW); break;
    case 3: launch_cohort<3>(st, L, NR, W, T_m, B, N, K, SWR, SW, CNT, FW); break;
    case 4: launch_cohort<4>(st, L, NR, W, T_m, B, N, K, SWR, SW, CNT, FW); break;
    case 5: launch_cohort<5>(st, L, NR, W, T_m, B, N, K, SWR, SW, CNT, FW); break;
    case 10: launch_cohort<10>(st, L, NR, W, T_m, B, N, K, SWR, SW, CNT, FW); break;
    case 20: launch_cohort<20>(st, L, NR, W, T_m, B, N, K, SWR, SW, CNT, FW); break;
    default:
      return set_err(ctx, CSM_E_INVAL, "csm_portfolio: n_bins=%d unsupported (2,3,4,5,10,20)", n_bins);
  }
  LAUNCH_CHECK(ctx, "k_cohort");
  if (TURN || COST) {
    hipLaunchKernelGGL(k_turnover, dim3((unsigned)(T_m * B)), dim3(PF_THREADS), 0, st, L, W,
                       (const double*)FW, T_m, B, N, K, n_bins, half_spread, k_impact, aum, ADV,
                       SIG, TURN, COST);
    LAUNCH_CHECK(ctx, "k_turnover");
  }
  hipLaunchKernelGGL(k_overlap_ls, dim3((unsigned)B), dim3(PF_THREADS), 0, st,
                     (const double*)SWR, (const double*)SW, (const int32_t*)CNT, T_m, B, K,
                     n_bins, PR, LS, (const double*)COST, NET);
  LAUNCH_CHECK(ctx, "k_overlap_ls");
  return CSM_OK;
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
