// sweep_boot.hip -- the bootstrap sweep's scan without a materialised price panel
// (csm_boot_scan; BASELINE configs[4], rule E6 in oracle/portfolio_oracle.py).  Round 2 ran C5 as
// csm_bootstrap (PMb [T_m][B][N] written: 1.2 GB per batch of 100 panels) -> the multi-J scan (PMb
// read; mom_J + next_ret + bucket ids written per J: 18 B per cell and J) -> the decile pass on
// ids.  k_boot_scan generates each resampled price in registers from the base return rows
// (R_base, 12 MB: cache-resident) with k_bootstrap_panel's arithmetic, runs
// k_momentum_multi_reg2's scan on it (the same factors in the same order: the same mom_J bits and
// bucket ids), and writes mom_J + ids per J and ONE next_ret panel for every J: 10 B per cell and
// J + 8 B per cell instead of 18 B per cell and J + 24 B per cell.  The decile pass
// (csm_deciles_ids) then runs on M / ids unchanged.
//
// Why one next_ret panel is exact.  NR_J of the scan is ps_new / psff_J - 1 on J's ranked rows
// (run_demo.py:48: pct_change over the ranked subset, then shift(-1)), NaN elsewhere.  A
// bootstrap panel has no present row with a NaN price (a month is either absent or a finite
// product), so while every present price is finite and non-zero no fl(1 + ret) factor after the
// first valid return is NaN: every present row from a J's first ranked row on is ranked, psff_J
// is that row's own price, and NR_J equals the shared x_next / x - 1 on every row that J ranks.
// The portfolio reads next_ret only for members ranked at formation month s, in holding months
// t >= s, where the asset is ranked again (present) or absent (NaN in both), so PR / LS / TURN /
// COST / NET are unchanged.  A generated price that is not finite and non-zero sets *bad, and
// the caller reruns the batch on the materialised path.
//
// Measured and not kept (profiles/r03/experiments/ab1_*): ranking from the ids WITHOUT writing
// mom_J -- a row histogram kernel (bucket ranges of the order statistics, labels of the certain
// cells, candidate lists), a second scan writing mom_J only for the candidates, a finish kernel
// selecting inside the ranges.  The second scan repeats the whole scan's arithmetic with a range
// test per cell: C5 rank stage 118 ms/step against 55 for bootstrap + scan + decile pass.
#include "csm_common.h"

#define BS_MAXJ 4
#define BS_RW 16        // generic register ring: max(J) + skip <= 16
#ifndef BS_CHUNK
#define BS_CHUNK 8      // months of R rows in flight per lane
#endif
#ifndef BS_MINB
#define BS_MINB 1
#endif
#define BS_THREADS 256

struct BSSet {
  int J[BS_MAXJ];
  uint16_t* IDS[BS_MAXJ];   // nullable together
  double* M[BS_MAXJ];
};

// Window product of look-back J (slots [RW - J - skip, RW - skip) of the shift register, oldest
// first).  FIX: the default grid J = 3, 6, 9, 12, skip 1 with compile-time windows (J - 1
// multiplies each); otherwise every slot predicated (acc starts at 1.0, and 1.0 * x == x, so the
// product is the same oldest-first sequence).
template <int RW, bool FIX>
__device__ __forceinline__ double win_prod(const double (&f)[RW], int q, int lo, int hi) {
  if (FIX) {
    constexpr int Jq[4] = {3, 6, 9, 12};
    double acc = 0.0;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      if (qq != q) continue;
      const int l = RW - Jq[qq] - 1;
      double a = f[l];
#pragma unroll
      for (int k = l + 1; k < RW - 1; ++k) a = a * f[k];
      acc = a;
    }
    return acc;
  }
  double acc = 1.0;
#pragma unroll
  for (int k = 0; k < RW; ++k) acc = (k >= lo && k < hi) ? acc * f[k] : acc;
  return acc;
}

// One lane per two adjacent assets of one panel (N even): column c0 = b * N + a0 of the
// [T_m][B * N] layout.  R rows are gathered by the panel's source months, BS_CHUNK months in
// flight.
template <int RW, bool FIX>
__global__ __launch_bounds__(BS_THREADS, BS_MINB) void k_boot_scan(
    const double* __restrict__ R, int T_m, int64_t N, int B, const int32_t* __restrict__ src,
    double p0, int nJ, int skip, BSSet js, double* __restrict__ NR, int32_t* __restrict__ bad) {
  const int64_t BN = (int64_t)B * N;
  const int64_t c0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 2;
  if (c0 >= BN) return;   // no barriers below
  const int b = (int)(c0 / N);
  const int64_t a0 = c0 - (int64_t)b * N;
  const int32_t* sb = src + (int64_t)b * T_m;
  const double NaN = qnan();
  double f[2][RW];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int k = 0; k < RW; ++k) f[c][k] = NaN;
  double pff[2] = {NaN, NaN};
  double prv[2] = {p0, p0};     // the bootstrap price product
  int pc[2] = {-1, -1};         // last present row (the shared next_ret)
  bool badp = false;
  int lo[BS_MAXJ];
#pragma unroll
  for (int q = 0; q < BS_MAXJ; ++q) lo[q] = RW - js.J[q] - skip;
  const int hi = RW - skip;
  const bool with_ids = js.IDS[0] != nullptr;
  for (int m0 = 0; m0 < T_m; m0 += BS_CHUNK) {
    int s[BS_CHUNK];
#pragma unroll
    for (int j = 0; j < BS_CHUNK; ++j) s[j] = (m0 + j < T_m) ? sb[m0 + j] : 0;
    double2 rr[BS_CHUNK];
#pragma unroll
    for (int j = 0; j < BS_CHUNK; ++j)
      rr[j] = (m0 + j < T_m) ? *reinterpret_cast<const double2*>(R + (int64_t)s[j] * N + a0)
                             : make_double2(NaN, NaN);
#pragma unroll
    for (int j = 0; j < BS_CHUNK; ++j) {
      const int m = m0 + j;
      if (m >= T_m) break;
      const double rs[2] = {rr[j].x, rr[j].y};
      double xs[2], rt[2];
      bool ab[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        // k_bootstrap_panel: a valid return extends the price product, a NaN one is an absent month
        const double r = rs[c];
        ab[c] = !(r == r);
        if (!ab[c]) {
          const double fct = 1.0 + r;
          prv[c] = prv[c] * fct;
        }
        const double x = prv[c];
        xs[c] = x;
        if (!ab[c] && !(fabs(x) < INFINITY && x != 0.0)) badp = true;
        // k_momentum_multi_reg2's step on a present x (never NaN here).  pff and px (the shared
        // next_ret's previous price) are both the last present price, so ret doubles as the
        // pending row's next_ret below: one f64 division per asset-month instead of two
        const double ret = x / pff[c] - 1.0;
        rt[c] = ret;
        // the shared next_ret also needs every factor fl(1 + ret) after the first present price
        // finite and non-zero (x / pff can overflow or round to a zero factor even when both
        // prices are): otherwise 0 * inf could leave a J's ranked row without a return
        {
          const double fr = 1.0 + ret;
          if (!ab[c] && pff[c] == pff[c] && !(fabs(fr) < INFINITY && fr != 0.0)) badp = true;
        }
        pff[c] = ab[c] ? pff[c] : x;
#pragma unroll
        for (int k = 0; k + 1 < RW; ++k) f[c][k] = ab[c] ? f[c][k] : f[c][k + 1];
        f[c][RW - 1] = ab[c] ? f[c][RW - 1] : 1.0 + ret;
      }
      const int64_t o = (int64_t)m * BN + c0;
      {   // shared next_ret: absent rows NaN now, present rows when the next present one comes
        int wp[2];
        double vp[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          wp[c] = (!ab[c] && pc[c] >= 0) ? pc[c] : -1;
          vp[c] = rt[c];   // == x / (last present price) - 1.0
          if (!ab[c]) pc[c] = m;
        }
        if (wp[0] >= 0 && wp[0] == wp[1]) {
          *reinterpret_cast<double2*>(NR + (int64_t)wp[0] * BN + c0) = make_double2(vp[0], vp[1]);
        } else {
          if (wp[0] >= 0) NR[(int64_t)wp[0] * BN + c0] = vp[0];
          if (wp[1] >= 0) NR[(int64_t)wp[1] * BN + c0 + 1] = vp[1];
        }
        if (ab[0] && ab[1]) {
          *reinterpret_cast<double2*>(NR + o) = make_double2(NaN, NaN);
        } else {
          if (ab[0]) NR[o] = NaN;
          if (ab[1]) NR[o + 1] = NaN;
        }
      }
#pragma unroll
      for (int q = 0; q < BS_MAXJ; ++q) {
        if (q >= nJ) break;
        double mom[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) mom[c] = ab[c] ? NaN : win_prod<RW, FIX>(f[c], q, lo[q], hi) - 1.0;
        *reinterpret_cast<double2*>(js.M[q] + o) = make_double2(mom[0], mom[1]);
        if (with_ids)
          *reinterpret_cast<uint32_t*>(js.IDS[q] + o) = csm_fid(mom[0]) | (csm_fid(mom[1]) << 16);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 2; ++c)
    if (pc[c] >= 0) NR[(int64_t)pc[c] * BN + c0 + c] = NaN;   // no later present month
  if (badp) *bad = 1;
}

// the bootstrap source-month sequences (portfolio.hip)
void launch_bootstrap_index(hipStream_t st, int T_m, int B, int64_t b0, uint64_t seed,
                            double p_new, int32_t* src);

extern "C" {

int csm_boot_scan(csm_ctx* ctx, const double* R, int32_t T_m, int64_t N, int32_t B, int64_t b0,
                  uint64_t seed, double mean_block, double p0, const int32_t* Js, int32_t nJ,
                  int32_t skip, int32_t* src, double* const* M, uint16_t* const* IDS, double* NR,
                  int32_t* bad) {
  int r = prep(ctx);
  if (r) return r;
  if (!R || !Js || !src || !M || !NR || !bad || T_m < 1 || N <= 0 || N % 2 != 0 || B < 1 ||
      b0 < 0 || nJ < 1 || nJ > BS_MAXJ || skip < 0 || !(mean_block >= 1.0))
    return set_err(ctx, CSM_E_INVAL, "csm_boot_scan: bad arguments (T_m=%d N=%lld B=%d nJ=%d; "
                   "N even, 1 <= nJ <= %d)", T_m, (long long)N, B, nJ, BS_MAXJ);
  BSSet js;
  bool fix = nJ == 4 && skip == 1;
  for (int qq = 0; qq < BS_MAXJ; ++qq) {
    const bool on = qq < nJ;
    js.J[qq] = on ? Js[qq] : 1;
    js.M[qq] = on ? M[qq] : nullptr;
    js.IDS[qq] = (on && IDS) ? IDS[qq] : nullptr;
    if (on && (Js[qq] < 1 || Js[qq] + skip > BS_RW || !M[qq] || !aligned16(M[qq]) ||
               (IDS && (!IDS[qq] || ((uintptr_t)IDS[qq] & 3u)))))
      return set_err(ctx, CSM_E_INVAL, "csm_boot_scan: J[%d]=%d (J + skip <= %d) or its buffers "
                     "invalid / misaligned", qq, on ? Js[qq] : 0, BS_RW);
    if (on && Js[qq] != 3 * (qq + 1)) fix = false;
  }
  if (!aligned16(R) || !aligned16(NR))
    return set_err(ctx, CSM_E_INVAL, "csm_boot_scan: R and NR must be 16-B aligned");
  HIP_CHECK(ctx, zero_i32_async(bad, 1, ctx->stream));
  launch_bootstrap_index(ctx->stream, T_m, B, b0, seed, 1.0 / mean_block, src);
  LAUNCH_CHECK(ctx, "k_bootstrap_index");
  const int64_t BN = (int64_t)B * N;
  const unsigned blocks = (unsigned)((BN / 2 + BS_THREADS - 1) / BS_THREADS);
  if (fix)   // J = 3, 6, 9, 12, skip 1: a 13-slot ring, compile-time windows
    hipLaunchKernelGGL((k_boot_scan<13, true>), dim3(blocks), dim3(BS_THREADS), 0, ctx->stream, R,
                       T_m, N, B, (const int32_t*)src, p0, nJ, skip, js, NR, bad);
  else
    hipLaunchKernelGGL((k_boot_scan<BS_RW, false>), dim3(blocks), dim3(BS_THREADS), 0, ctx->stream,
                       R, T_m, N, B, (const int32_t*)src, p0, nJ, skip, js, NR, bad);
  LAUNCH_CHECK(ctx, "k_boot_scan");
  return CSM_OK;
}

}  // extern "C"
