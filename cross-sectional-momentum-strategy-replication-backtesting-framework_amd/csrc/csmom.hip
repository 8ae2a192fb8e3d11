// csmom.hip -- hand-written gfx950 (CDNA4) kernels + C ABI for the momentum backtest hot path.
//
// Every kernel here is HBM- or latency-bound integer/fp64 work; nothing is a contraction, so
// no MFMA.  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (the fp64 products and
// lerps must not be contracted into FMAs -- bit-exactness with NumPy/pandas depends on it).
//
// Reference behaviour restated (file:line into the reference):
//   month-end         src/features.py:34-39   (groupby ticker x Grouper('ME'): last / sum)
//   ret/mom scan      src/features.py:44-52   (pct_change ffill; shift(skip).rolling(J) prod)
//   next_ret          run_demo.py:48          (pct_change within the ranked subset, shift(-1))
//   deciles           run_demo.py:18-29,46    (pd.qcut(q=n, labels=False, duplicates='drop'))
//   decile means      run_demo.py:49-55       (dropna; groupby(date, decile).mean())
//   long-short        run_demo.py:57-67
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>


#include "csm_common.h"

// =====================================================================================
// Kernel A: month-end aggregation.  One thread per (month, VEC assets); a wave streams
// 64*VEC*8 contiguous bytes per day row (1 KiB at VEC=2).  Days of a month are walked in
// order so the Kahan volume sum matches pandas' group_sum bit for bit.
// =====================================================================================
template <int VEC, bool WITH_VOL>
__global__ __launch_bounds__(256) void k_month_end(const double* __restrict__ P,
                                                   const double* __restrict__ V,
                                                   const int64_t* __restrict__ month_start,
                                                   int64_t N, double* __restrict__ PM,
                                                   double* __restrict__ VOL) {
  const int m = blockIdx.y;
  const int64_t a = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * VEC;
  if (a >= N) return;
  const int64_t d0 = month_start[m], d1 = month_start[m + 1];
  double last[VEC];
  bool anyp[VEC], anyv[VEC];
  double s[VEC], c[VEC];
#pragma unroll
  for (int k = 0; k < VEC; ++k) {
    last[k] = 0.0; anyp[k] = false; anyv[k] = false; s[k] = 0.0; c[k] = 0.0;
  }
  const double* p = P + d0 * N + a;
  const double* v = WITH_VOL ? V + d0 * N + a : nullptr;
  int64_t d = d0;
  // prices only, a business month (<= 24 rows): every row load in flight at once, one round
  // trip per thread (the 8-row batches and the serial tail below took three to eight); rows
  // past the month are ABSENT placeholders, which change nothing
  constexpr int MD = 24;
  if (!WITH_VOL && d1 - d0 <= MD) {
    const int nd = (int)(d1 - d0);
    double x[MD][VEC];
#pragma unroll
    for (int j = 0; j < MD; ++j) {
      if (j < nd) {
        if (VEC == 2) {
          const double2 t = *reinterpret_cast<const double2*>(p + (int64_t)j * N);
          x[j][0] = t.x; x[j][VEC - 1] = t.y;
        } else {
          x[j][0] = p[(int64_t)j * N];
        }
      } else {
#pragma unroll
        for (int k = 0; k < VEC; ++k) x[j][k] = absent_val();
      }
    }
#pragma unroll
    for (int j = 0; j < MD; ++j) {
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        const bool pr = !is_absent(x[j][k]);
        const bool ok = pr && !isnan_d(x[j][k]);
        anyp[k] |= pr;
        anyv[k] |= ok;
        last[k] = ok ? x[j][k] : last[k];
      }
    }
    d = d1;
  }
  // 8-day batches keep 8 row loads in flight per lane before the dependent selects.
  for (; d + 8 <= d1; d += 8) {
    double x[8][VEC];
    double y[WITH_VOL ? 8 : 1][VEC];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (VEC == 2) {
        double2 t = *reinterpret_cast<const double2*>(p + j * N);
        x[j][0] = t.x; x[j][VEC - 1] = t.y;
        if (WITH_VOL) { double2 u = *reinterpret_cast<const double2*>(v + j * N); y[j][0] = u.x; y[j][VEC - 1] = u.y; }
      } else {
        x[j][0] = p[j * N];
        if (WITH_VOL) y[j][0] = v[j * N];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        const bool pr = !is_absent(x[j][k]);
        const bool ok = pr && !isnan_d(x[j][k]);
        anyp[k] |= pr;
        anyv[k] |= ok;
        last[k] = ok ? x[j][k] : last[k];
        if (WITH_VOL && pr) {
          double val = y[j][k];
          val = isnan_d(val) ? 0.0 : val;
          const double yy = val - c[k];
          const double tt = s[k] + yy;
          double cc = (tt - s[k]) - yy;
          c[k] = isnan_d(cc) ? 0.0 : cc;
          s[k] = tt;
        }
      }
    }
    p += 8 * N;
    if (WITH_VOL) v += 8 * N;
  }
  for (; d < d1; ++d) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      const double xv = p[k];
      const bool pr = !is_absent(xv);
      const bool ok = pr && !isnan_d(xv);
      anyp[k] |= pr;
      anyv[k] |= ok;
      last[k] = ok ? xv : last[k];
      if (WITH_VOL && pr) {
        double val = v[k];
        val = isnan_d(val) ? 0.0 : val;
        const double yy = val - c[k];
        const double tt = s[k] + yy;
        double cc = (tt - s[k]) - yy;
        c[k] = isnan_d(cc) ? 0.0 : cc;
        s[k] = tt;
      }
    }
    p += N;
    if (WITH_VOL) v += N;
  }
  double out[VEC];
#pragma unroll
  for (int k = 0; k < VEC; ++k) out[k] = anyp[k] ? (anyv[k] ? last[k] : qnan()) : absent_val();
  double* o = PM + (int64_t)m * N + a;
  if (VEC == 2) {
    *reinterpret_cast<double2*>(o) = make_double2(out[0], out[VEC - 1]);
  } else {
    o[0] = out[0];
  }
  if (WITH_VOL) {
    double* w = VOL + (int64_t)m * N + a;
#pragma unroll
    for (int k = 0; k < VEC; ++k) w[k] = anyp[k] ? s[k] : 0.0;
  }
}

// =====================================================================================
// Per-asset scan state and one present-row step (shared by k_momentum and k_signal).
// The J+skip ring of factors fl(1+ret) lives in LDS, slot-major with a per-lane column
// (stride RS doubles), so a wave's ring accesses are conflict-free.
// mom = (prod over the J oldest ring entries of fl(1+ret), left to right) - 1.
// =====================================================================================
struct ScanLane {
  double pff;   // last valid month price (features.py:44 grouped ffill)
  double psff;  // last valid price among ranked rows (run_demo.py:48 subset ffill)
  int head;     // index of the oldest ring entry
  int prev;     // month of the pending ranked row (its next_ret waits for the next row)
};

__device__ __forceinline__ void scan_init(ScanLane& s, double* ring, int RS, int W,
                                          const double* __restrict__ carry, int64_t N,
                                          int64_t a, bool live) {
  if (live && carry) {
    for (int k = 0; k < W; ++k) ring[k * RS] = carry[(int64_t)k * N + a];
    s.pff = carry[(int64_t)W * N + a];
    s.psff = carry[(int64_t)(W + 1) * N + a];
  } else {
    for (int k = 0; k < W; ++k) ring[k * RS] = qnan();
    s.pff = qnan();
    s.psff = qnan();
  }
  s.head = 0;
  s.prev = -1;
}

// Consumes month m's price x of asset a; returns mom (NaN when absent / undefined).
__device__ __forceinline__ double scan_step(ScanLane& s, double x, int m, double* ring, int RS,
                                            int W, int J, int64_t N, int64_t a,
                                            double* __restrict__ R, double* __restrict__ M,
                                            double* __restrict__ NR) {
  const double NaN = qnan();
  const int64_t o = (int64_t)m * N + a;
  if (is_absent(x)) {
    if (R) R[o] = NaN;
    M[o] = NaN;
    NR[o] = NaN;
    return NaN;
  }
  const bool xv = !isnan_d(x);
  const double pnew = xv ? x : s.pff;
  const double ret = pnew / s.pff - 1.0;
  s.pff = pnew;
  ring[s.head * RS] = 1.0 + ret;          // push: overwrite the oldest, advance head
  s.head = (s.head + 1 == W) ? 0 : s.head + 1;
  double acc = ring[s.head * RS];
  int idx = s.head;
  for (int k = 1; k < J; ++k) {
    idx = (idx + 1 == W) ? 0 : idx + 1;
    acc = acc * ring[idx * RS];
  }
  const double mom = acc - 1.0;
  const bool ranked = !isnan_d(mom);
  const double ps_new = xv ? x : s.psff;
  if (s.prev >= 0) NR[(int64_t)s.prev * N + a] = ps_new / s.psff - 1.0;
  if (ranked) {
    s.psff = ps_new;
    s.prev = m;
  } else {
    NR[o] = NaN;
    s.prev = -1;
  }
  if (R) R[o] = ret;
  M[o] = mom;
  return mom;
}

// scan_step for two adjacent assets a0, a0 + 1 (a0 even) with their stores paired: mom_J
// (and ret_1m) as one 16-B store per row, next_ret as one 16-B store when both assets write
// the same row (the steady state), so a wave issues half the store instructions.  Same
// arithmetic in the same order as two scan_step calls: bit-identical outputs.
template <int JC = 0>   // JC > 0: J fixed at compile time (the product's ring reads unrolled)
__device__ __forceinline__ void scan_step_pair(ScanLane (&s)[2], const double (&x)[2], int m,
                                               double* ring0, int RS, int W, int J, int64_t N,
                                               int64_t a0, double* __restrict__ R,
                                               double* __restrict__ M, double* __restrict__ NR,
                                               double (&mom)[2]) {
  const double NaN = qnan();
  double ret[2];
  int wp[2];          // next_ret row of the pending ranked row (-1: none)
  double vp[2];
  bool wc[2];         // NaN next_ret at row m
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    double* ring = ring0 + c;
    wp[c] = -1;
    vp[c] = NaN;
    if (is_absent(x[c])) {
      ret[c] = NaN; mom[c] = NaN; wc[c] = true;
      continue;
    }
    const bool xv = !isnan_d(x[c]);
    const double pnew = xv ? x[c] : s[c].pff;
    ret[c] = pnew / s[c].pff - 1.0;
    s[c].pff = pnew;
    ring[s[c].head * RS] = 1.0 + ret[c];
    s[c].head = (s[c].head + 1 == W) ? 0 : s[c].head + 1;
    double acc = ring[s[c].head * RS];
    int idx = s[c].head;
    if constexpr (JC > 0) {
      double f[JC];   // the ring reads all issued before the product
#pragma unroll
      for (int k = 1; k < JC; ++k) {
        idx = (idx + 1 == W) ? 0 : idx + 1;
        f[k] = ring[idx * RS];
      }
#pragma unroll
      for (int k = 1; k < JC; ++k) acc = acc * f[k];
    } else {
      for (int k = 1; k < J; ++k) {
        idx = (idx + 1 == W) ? 0 : idx + 1;
        acc = acc * ring[idx * RS];
      }
    }
    mom[c] = acc - 1.0;
    const bool ranked = !isnan_d(mom[c]);
    const double ps_new = xv ? x[c] : s[c].psff;
    if (s[c].prev >= 0) { wp[c] = s[c].prev; vp[c] = ps_new / s[c].psff - 1.0; }
    if (ranked) {
      s[c].psff = ps_new;
      s[c].prev = m;
      wc[c] = false;
    } else {
      s[c].prev = -1;
      wc[c] = true;
    }
  }
  const int64_t o = (int64_t)m * N + a0;
  if (R) *reinterpret_cast<double2*>(R + o) = make_double2(ret[0], ret[1]);
  *reinterpret_cast<double2*>(M + o) = make_double2(mom[0], mom[1]);
  if (wp[0] >= 0 && wp[0] == wp[1]) {
    *reinterpret_cast<double2*>(NR + (int64_t)wp[0] * N + a0) = make_double2(vp[0], vp[1]);
  } else {
    if (wp[0] >= 0) NR[(int64_t)wp[0] * N + a0] = vp[0];
    if (wp[1] >= 0) NR[(int64_t)wp[1] * N + a0 + 1] = vp[1];
  }
  if (wc[0] && wc[1]) {
    *reinterpret_cast<double2*>(NR + o) = make_double2(NaN, NaN);
  } else {
    if (wc[0]) NR[o] = NaN;
    if (wc[1]) NR[o + 1] = NaN;
  }
}

__device__ __forceinline__ void scan_finish(ScanLane& s, double* ring, int RS, int W, int64_t N,
                                            int64_t a, double* __restrict__ NR,
                                            const double* __restrict__ next_pm,
                                            double* __restrict__ carry_out) {
  if (s.prev >= 0) {
    double nr = qnan();
    if (next_pm) {
      const double x = next_pm[a];
      if (!is_absent(x)) {
        const double ps_new = isnan_d(x) ? s.psff : x;
        nr = ps_new / s.psff - 1.0;
      }
    }
    NR[(int64_t)s.prev * N + a] = nr;
  }
  if (carry_out) {
    int idx = s.head;
    for (int k = 0; k < W; ++k) {  // carry rows hold the ring's factors, oldest first
      carry_out[(int64_t)k * N + a] = ring[idx * RS];
      idx = (idx + 1 == W) ? 0 : idx + 1;
    }
    carry_out[(int64_t)W * N + a] = s.pff;
    carry_out[(int64_t)(W + 1) * N + a] = s.psff;
  }
}

// Month range of chunk g when T_m months are split into G contiguous chunks (earlier
// chunks take the remainder) -- the same split as distributed.month_partition.
__device__ __forceinline__ void chunk_range(int T_m, int G, int g, int& m0, int& m1) {
  const int base = T_m / G, rem = T_m % G;
  m0 = g * base + (g < rem ? g : rem);
  m1 = m0 + base + (g < rem ? 1 : 0);
}

// =====================================================================================
// Kernel B: per-asset scan over month prices (present rows only).  One thread per asset;
// PM rows prefetched SCAN_CHUNK months ahead (SCAN_CHUNK * 512 B in flight per wave).
// =====================================================================================
#define SCAN_THREADS 128
#define SCAN_CHUNK 16

__device__ __forceinline__ void momentum_body(
    double* ring_lds, const double* __restrict__ PM, int T_m, int64_t N, int J, int skip,
    double* __restrict__ R, double* __restrict__ M, double* __restrict__ NR,
    const double* __restrict__ carry, const double* __restrict__ next_pm,
    double* __restrict__ carry_out, uint16_t* __restrict__ IDS = nullptr);

__global__ __launch_bounds__(256) void k_momentum(
    const double* __restrict__ PM, int T_m, int64_t N, int J, int skip, double* __restrict__ R,
    double* __restrict__ M, double* __restrict__ NR, const double* __restrict__ carry,
    const double* __restrict__ next_pm, double* __restrict__ carry_out) {
  extern __shared__ __attribute__((aligned(16))) double ring_lds[];
  momentum_body(ring_lds, PM, T_m, N, J, skip, R, M, NR, carry, next_pm, carry_out);
}

// Time-chunked scan (small N): chunk blockIdx.y scans its month range from the carry that
// k_fold_carry rebuilt for it -- C x more waves in flight, same results bit for bit.
__global__ __launch_bounds__(256) void k_momentum_chunked(
    const double* __restrict__ PM, int T_m, int G, int64_t N, int J, int skip,
    double* __restrict__ R, double* __restrict__ M, double* __restrict__ NR,
    const double* __restrict__ carry, const double* __restrict__ next_pm,
    uint16_t* __restrict__ IDS) {
  extern __shared__ __attribute__((aligned(16))) double ring_lds[];
  const int g = blockIdx.y;
  int m0, m1;
  chunk_range(T_m, G, g, m0, m1);
  const int W = J + skip;
  const int64_t off = (int64_t)m0 * N;
  momentum_body(ring_lds, PM + off, m1 - m0, N, J, skip, R ? R + off : nullptr, M + off,
                NR + off, g > 0 ? carry + (int64_t)g * (W + 2) * N : nullptr,
                next_pm + (int64_t)g * N, nullptr, IDS ? IDS + off : nullptr);
}

__device__ __forceinline__ void momentum_body(
    double* ring_lds, const double* __restrict__ PM, int T_m, int64_t N, int J, int skip,
    double* __restrict__ R, double* __restrict__ M, double* __restrict__ NR,
    const double* __restrict__ carry, const double* __restrict__ next_pm,
    double* __restrict__ carry_out, uint16_t* __restrict__ IDS) {
  const int W = J + skip;
  const int tid = threadIdx.x;
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + tid;
  const bool live = a < N;
  const int RS = blockDim.x;
  double* ring = ring_lds + tid;
  ScanLane s;
  scan_init(s, ring, RS, W, carry, N, a, live);
  if (!live) return;
  for (int m0 = 0; m0 < T_m; m0 += SCAN_CHUNK) {
    double buf[SCAN_CHUNK];
#pragma unroll
    for (int j = 0; j < SCAN_CHUNK; ++j)
      buf[j] = (m0 + j < T_m) ? PM[(int64_t)(m0 + j) * N + a] : absent_val();
#pragma unroll
    for (int j = 0; j < SCAN_CHUNK; ++j) {
      const int m = m0 + j;
      if (m >= T_m) break;
      const double mom = scan_step(s, buf[j], m, ring, RS, W, J, N, a, R, M, NR);
      if (IDS) IDS[(int64_t)m * N + a] = (uint16_t)csm_fid(mom);   // the decile pass's bucket id
    }
  }
  scan_finish(s, ring, RS, W, N, a, NR, next_pm, carry_out);
}

// Several look-backs in one scan (parameter sweeps, C3 / C5): one read of PM, one ring of
// Jmax + skip factors fl(1 + ret), and per J the sequential product over the oldest J of its
// last J + skip factors -- the same factors in the same order as k_momentum with a ring of
// exactly J + skip, so M and NR are bit-identical to per-J k_momentum calls.  NR is kept per
// J: the ranked subset (and so next_ret's subset-ffill, run_demo.py:48) starts J + skip
// present months after the first price.  No carry / next_pm (whole panels only).
#define MJ_MAX 4
struct MJSet {
  int J[MJ_MAX];
  double* M[MJ_MAX];
  double* NR[MJ_MAX];
  uint16_t* IDS[MJ_MAX];   // nullable: fixed-map bucket ids of M (csm_momentum_multi_ids)
};

__global__ __launch_bounds__(256) void k_momentum_multi(const double* __restrict__ PM, int T_m,
                                                        int64_t N, int nJ, int skip, int W,
                                                        MJSet mj) {
  extern __shared__ __attribute__((aligned(16))) double ring_lds[];
  const int tid = threadIdx.x;
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + tid;
  if (a >= N) return;   // no barriers below
  const int RS = blockDim.x;
  double* ring = ring_lds + tid;
  const double NaN = qnan();
  for (int k = 0; k < W; ++k) ring[k * RS] = NaN;
  int head = 0;
  double pff = NaN;
  double psff[MJ_MAX];
  int prev[MJ_MAX];
#pragma unroll
  for (int q = 0; q < MJ_MAX; ++q) { psff[q] = NaN; prev[q] = -1; }
  for (int m0 = 0; m0 < T_m; m0 += SCAN_CHUNK) {
    double buf[SCAN_CHUNK];
#pragma unroll
    for (int j = 0; j < SCAN_CHUNK; ++j)
      buf[j] = (m0 + j < T_m) ? PM[(int64_t)(m0 + j) * N + a] : absent_val();
#pragma unroll
    for (int j = 0; j < SCAN_CHUNK; ++j) {
      const int m = m0 + j;
      if (m >= T_m) break;
      const double x = buf[j];
      const int64_t o = (int64_t)m * N + a;
      if (is_absent(x)) {
#pragma unroll
        for (int q = 0; q < MJ_MAX; ++q)
          if (q < nJ) {
            mj.M[q][o] = NaN; mj.NR[q][o] = NaN;
            if (mj.IDS[q]) mj.IDS[q][o] = (uint16_t)CSM_FB_NAN;
          }
        continue;
      }
      const bool xv = !isnan_d(x);
      const double pnew = xv ? x : pff;
      const double ret = pnew / pff - 1.0;
      pff = pnew;
      ring[head * RS] = 1.0 + ret;          // push: overwrite the oldest, advance head
      head = (head + 1 == W) ? 0 : head + 1;
#pragma unroll
      for (int q = 0; q < MJ_MAX; ++q) {
        if (q >= nJ) break;
        const int J = mj.J[q];
        int idx = head + (W - J - skip);      // oldest of this J's window
        if (idx >= W) idx -= W;
        double acc = ring[idx * RS];
        for (int k = 1; k < J; ++k) {
          idx = (idx + 1 == W) ? 0 : idx + 1;
          acc = acc * ring[idx * RS];
        }
        const double mom = acc - 1.0;
        const double ps_new = xv ? x : psff[q];
        if (prev[q] >= 0) mj.NR[q][(int64_t)prev[q] * N + a] = ps_new / psff[q] - 1.0;
        if (!isnan_d(mom)) {
          psff[q] = ps_new;
          prev[q] = m;
        } else {
          mj.NR[q][o] = NaN;
          prev[q] = -1;
        }
        mj.M[q][o] = mom;
        if (mj.IDS[q]) mj.IDS[q][o] = (uint16_t)csm_fid(mom);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < MJ_MAX; ++q)
    if (q < nJ && prev[q] >= 0) mj.NR[q][(int64_t)prev[q] * N + a] = NaN;
}

// Register-ring variant for max(J) + skip <= RW: the last RW factors live in registers as a
// shift register (f[RW-1] newest), and J's product runs over all RW slots with the slots
// outside its window predicated off.  acc starts at 1.0 and 1.0 * x == x exactly, so the
// product is still oldest-first over the same factors: bit-identical, no LDS round trips.
template <int RW>
__global__ __launch_bounds__(256) void k_momentum_multi_reg(const double* __restrict__ PM,
                                                            int T_m, int64_t N, int nJ, int skip,
                                                            MJSet mj) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= N) return;
  const double NaN = qnan();
  double f[RW];
#pragma unroll
  for (int k = 0; k < RW; ++k) f[k] = NaN;
  double pff = NaN;
  double psff[MJ_MAX];
  int prev[MJ_MAX], lo[MJ_MAX];
#pragma unroll
  for (int q = 0; q < MJ_MAX; ++q) {
    psff[q] = NaN; prev[q] = -1;
    lo[q] = RW - mj.J[q] - skip;   // window = slots [lo, RW - skip)
  }
  const int hi = RW - skip;
  for (int m0 = 0; m0 < T_m; m0 += SCAN_CHUNK) {
    double buf[SCAN_CHUNK];
#pragma unroll
    for (int j = 0; j < SCAN_CHUNK; ++j)
      buf[j] = (m0 + j < T_m) ? PM[(int64_t)(m0 + j) * N + a] : absent_val();
#pragma unroll
    for (int j = 0; j < SCAN_CHUNK; ++j) {
      const int m = m0 + j;
      if (m >= T_m) break;
      const double x = buf[j];
      const int64_t o = (int64_t)m * N + a;
      if (is_absent(x)) {
#pragma unroll
        for (int q = 0; q < MJ_MAX; ++q)
          if (q < nJ) {
            mj.M[q][o] = NaN; mj.NR[q][o] = NaN;
            if (mj.IDS[q]) mj.IDS[q][o] = (uint16_t)CSM_FB_NAN;
          }
        continue;
      }
      const bool xv = !isnan_d(x);
      const double pnew = xv ? x : pff;
      const double ret = pnew / pff - 1.0;
      pff = pnew;
#pragma unroll
      for (int k = 0; k + 1 < RW; ++k) f[k] = f[k + 1];
      f[RW - 1] = 1.0 + ret;
#pragma unroll
      for (int q = 0; q < MJ_MAX; ++q) {
        if (q >= nJ) break;
        double acc = 1.0;
#pragma unroll
        for (int k = 0; k < RW; ++k) acc = (k >= lo[q] && k < hi) ? acc * f[k] : acc;
        const double mom = acc - 1.0;
        const double ps_new = xv ? x : psff[q];
        if (prev[q] >= 0) mj.NR[q][(int64_t)prev[q] * N + a] = ps_new / psff[q] - 1.0;
        if (!isnan_d(mom)) {
          psff[q] = ps_new;
          prev[q] = m;
        } else {
          mj.NR[q][o] = NaN;
          prev[q] = -1;
        }
        mj.M[q][o] = mom;
        if (mj.IDS[q]) mj.IDS[q][o] = (uint16_t)csm_fid(mom);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < MJ_MAX; ++q)
    if (q < nJ && prev[q] >= 0) mj.NR[q][(int64_t)prev[q] * N + a] = NaN;
}
// Two adjacent assets per lane (a0 even): 16-B PM loads, mom_J / next_ret as one 16-B store
// per row when both assets write the same row (as k_signal's scan_step_pair), ids as one 4-B
// store: a wave moves 1 KiB per load / store instruction.  Same arithmetic per asset in the
// same order as k_momentum_multi_reg: bit-identical outputs.  N even, 16-B aligned buffers.
#define MJ2_CHUNK 8
// CH (csm_momentum_multi_chunked): chunk blockIdx.y of G scans its month range [ms, me) from
// the carry k_fold_carry rebuilt for max(J) (the last max(J) + skip factors, the month price
// pff) plus each J's subset-ffilled price psf[g][q] -- a smaller J's ring is the newest J + skip
// of the same factors -- and finishes its pending rows with npm[g] (the next chunk's first
// present price), as k_momentum_chunked does per J: the same bits.
// FIX: the default grid J = 3, 6, 9, 12 (in that order), skip 1, in a 13-slot ring with
// compile-time windows (J - 1 multiplies each, no predicated slots): the same oldest-first
// product (1.0 * x == x), about half the code -- the predicated chunked kernel was 85 KB, past
// the instruction cache.
template <int RW, bool FIX>
__device__ __forceinline__ double mj_window(const double (&f)[RW], int q, int lo, int hi) {
  if constexpr (FIX) {
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

template <int RW, bool CH = false, bool FIX = false>
__global__ __launch_bounds__(256) void k_momentum_multi_reg2(const double* __restrict__ PM,
                                                             int T_m, int64_t N, int nJ, int skip,
                                                             MJSet mj, int G = 1,
                                                             const double* __restrict__ carry = nullptr,
                                                             const double* __restrict__ npm = nullptr,
                                                             const double* __restrict__ psf = nullptr) {
  const int64_t a0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 2;
  if (a0 >= N) return;
  const double NaN = qnan();
  double f[2][RW];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int k = 0; k < RW; ++k) f[c][k] = NaN;
  double pff[2] = {NaN, NaN};
  double psff[2][MJ_MAX];
  int prev[2][MJ_MAX], lo[MJ_MAX];
  int Wmax = 0;
#pragma unroll
  for (int q = 0; q < MJ_MAX; ++q) {
    psff[0][q] = psff[1][q] = NaN;
    prev[0][q] = prev[1][q] = -1;
    lo[q] = RW - mj.J[q] - skip;   // window = slots [lo, RW - skip)
    if (q < nJ && mj.J[q] + skip > Wmax) Wmax = mj.J[q] + skip;
  }
  const int hi = RW - skip;
  int ms = 0, me = T_m;
  const int g = CH ? (int)blockIdx.y : 0;
  if (CH) {
    chunk_range(T_m, G, g, ms, me);
    if (g > 0) {   // the carried state: ring slots [RW - Wmax, RW) oldest first, pff, psff per J
      const double* cg = carry + (int64_t)g * (Wmax + 2) * N + a0;
#pragma unroll
      for (int k = 0; k < RW; ++k)
        if (k >= RW - Wmax) {
          const double2 v = *reinterpret_cast<const double2*>(cg + (int64_t)(k - (RW - Wmax)) * N);
          f[0][k] = v.x;
          f[1][k] = v.y;
        }
      const double2 pv = *reinterpret_cast<const double2*>(cg + (int64_t)Wmax * N);
      pff[0] = pv.x;
      pff[1] = pv.y;
#pragma unroll
      for (int q = 0; q < MJ_MAX; ++q)
        if (q < nJ) {
          const double2 v = *reinterpret_cast<const double2*>(psf + ((int64_t)g * MJ_MAX + q) * N + a0);
          psff[0][q] = v.x;
          psff[1][q] = v.y;
        }
    }
  }
  for (int m0 = ms; m0 < me; m0 += MJ2_CHUNK) {
    double2 buf[MJ2_CHUNK];
#pragma unroll
    for (int j = 0; j < MJ2_CHUNK; ++j)
      buf[j] = (m0 + j < me) ? *reinterpret_cast<const double2*>(PM + (int64_t)(m0 + j) * N + a0)
                             : make_double2(absent_val(), absent_val());
#pragma unroll
    for (int j = 0; j < MJ2_CHUNK; ++j) {
      const int m = m0 + j;
      if (m >= me) break;
      const double xs[2] = {buf[j].x, buf[j].y};
      const int64_t o = (int64_t)m * N + a0;
      bool ab[2], xv[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const double x = xs[c];
        ab[c] = is_absent(x);
        xv[c] = x == x;
        const double pnew = xv[c] ? x : pff[c];
        const double ret = pnew / pff[c] - 1.0;
        pff[c] = ab[c] ? pff[c] : pnew;
#pragma unroll
        for (int k = 0; k + 1 < RW; ++k) f[c][k] = ab[c] ? f[c][k] : f[c][k + 1];
        f[c][RW - 1] = ab[c] ? f[c][RW - 1] : 1.0 + ret;
      }
#pragma unroll
      for (int q = 0; q < MJ_MAX; ++q) {
        if (q >= nJ) break;
        double mom[2], vp[2];
        int wp[2];
        bool wc[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const double acc = mj_window<RW, FIX>(f[c], q, lo[q], hi);
          mom[c] = ab[c] ? NaN : acc - 1.0;
          const double ps_new = xv[c] ? xs[c] : psff[c][q];
          wp[c] = (!ab[c] && prev[c][q] >= 0) ? prev[c][q] : -1;
          vp[c] = ps_new / psff[c][q] - 1.0;
          const bool ranked = mom[c] == mom[c];
          wc[c] = !ranked;
          psff[c][q] = ranked ? ps_new : psff[c][q];
          prev[c][q] = ranked ? m : (ab[c] ? prev[c][q] : -1);
        }
        double* Mq = mj.M[q];
        double* NRq = mj.NR[q];
        *reinterpret_cast<double2*>(Mq + o) = make_double2(mom[0], mom[1]);
        if (wp[0] >= 0 && wp[0] == wp[1]) {
          *reinterpret_cast<double2*>(NRq + (int64_t)wp[0] * N + a0) = make_double2(vp[0], vp[1]);
        } else {
          if (wp[0] >= 0) NRq[(int64_t)wp[0] * N + a0] = vp[0];
          if (wp[1] >= 0) NRq[(int64_t)wp[1] * N + a0 + 1] = vp[1];
        }
        if (wc[0] && wc[1]) {
          *reinterpret_cast<double2*>(NRq + o) = make_double2(NaN, NaN);
        } else {
          if (wc[0]) NRq[o] = NaN;
          if (wc[1]) NRq[o + 1] = NaN;
        }
        if (mj.IDS[q])
          *reinterpret_cast<uint32_t*>(mj.IDS[q] + o) = csm_fid(mom[0]) | (csm_fid(mom[1]) << 16);
      }
    }
  }
  // pending ranked rows: next_ret from the next chunk's first present price (CH), else NaN
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const double x = CH ? npm[(int64_t)g * N + a0 + c] : absent_val();
#pragma unroll
    for (int q = 0; q < MJ_MAX; ++q)
      if (q < nJ && prev[c][q] >= 0) {
        double nr = NaN;
        if (CH && !is_absent(x)) {
          const double ps_new = isnan_d(x) ? psff[c][q] : x;
          nr = ps_new / psff[c][q] - 1.0;
        }
        mj.NR[q][(int64_t)prev[c][q] * N + a0 + c] = nr;
      }
  }
}

#define MJ_REG_W 16

// F's step: scan_step without outputs (the state transition only).
__device__ __forceinline__ void scan_shadow(ScanLane& s, double x, int m, double* ring, int RS,
                                            int W, int J) {
  if (is_absent(x)) return;
  const bool xv = !isnan_d(x);
  const double pnew = xv ? x : s.pff;
  const double ret = pnew / s.pff - 1.0;
  s.pff = pnew;
  ring[s.head * RS] = 1.0 + ret;
  s.head = (s.head + 1 == W) ? 0 : s.head + 1;
  double acc = ring[s.head * RS];
  int idx = s.head;
  for (int k = 1; k < J; ++k) {
    idx = (idx + 1 == W) ? 0 : idx + 1;
    acc = acc * ring[idx * RS];
  }
  const bool ranked = !isnan_d(acc - 1.0);
  if (ranked) {
    s.psff = xv ? x : s.psff;
    s.prev = m;
  } else {
    s.prev = -1;
  }
}

#ifdef SIG_HIST
__device__ uint32_t* g_sig_hist;   // A/B build only: csm_signal_ids' per-month id histogram
#endif

#define HALO_WALK 24   // a business month's day rows in one batch of loads
#define HALO_MAXG 64

// Month-end of asset a over day rows [d0, d1) (k_signal's reduction: last valid price, NaN if
// the month has rows but no price, ABSENT if none), walked back from the last row: one load for
// the usual month whose last row holds a price, else rows HALO_WALK at a time in flight.
__device__ __forceinline__ double halo_month_price(const double* __restrict__ P, int64_t d0,
                                                   int64_t d1, int64_t N, int64_t a) {
  if (d1 <= d0) return absent_val();
  const double xl = P[(d1 - 1) * N + a];
  if (xl == xl) return xl;
  bool p = !is_absent(xl);
  for (int64_t d = d1 - 2; d >= d0; d -= HALO_WALK) {
    double xs[HALO_WALK];
#pragma unroll
    for (int u = 0; u < HALO_WALK; ++u) xs[u] = d - u >= d0 ? P[(d - u) * N + a] : absent_val();
#pragma unroll
    for (int u = 0; u < HALO_WALK; ++u) {
      if (xs[u] == xs[u]) return xs[u];
      p |= !is_absent(xs[u]);
    }
  }
  return p ? qnan() : absent_val();
}

// =====================================================================================
// Kernel AB (fused): month-end aggregation + scan in one stream over the daily panel, for
// large N.  One wave per block, two assets per lane (16-B row loads, 1 KiB per wave-
// instruction).  While month m is reduced and scanned, the MAXD day rows of months m+1..m+3
// are already in flight (four register buffers).  Months shorter than MAXD re-load their last
// row into the spare slots: those loads hit L1/L2 (no extra HBM bytes), keep the load count
// fixed so vmcnt waits stay counted, and do not change "last non-NaN" / "any present".
// The month prices never round-trip through HBM unless PM is requested.
// =====================================================================================
// VEC assets per lane (VEC = 2: 16-B row loads, 1 KiB per wave-instruction; VEC = 1: twice
// the waves, 8-B loads), NBUF month buffers (NBUF - 1 months in flight).
template <int VEC> struct RowT;
template <> struct RowT<1> { typedef double T; };
template <> struct RowT<2> { typedef double2 T; };
__device__ __forceinline__ double comp(double v, int) { return v; }
__device__ __forceinline__ double comp(double2 v, int k) { return k == 0 ? v.x : v.y; }

// P is row-major [T_d][N]: consecutive day rows of a wave are N * 8 B apart.
// BW > 1: BW waves cover 64 * VEC * BW adjacent assets and walk them independently (no
// barrier), so a CU's loads of a day row are one BW-KiB span.
// Speculative shards keep PM only for the first and last W + SHARD_PM_EDGE months (what the
// summary walks and the repair read for a dense asset); other months are re-derived from the
// daily panel for the rare asset that needs them (shard_pm_at).
#define SHARD_PM_EDGE 8
__device__ __forceinline__ bool shard_pm_kept(int m, int T_m, int W) {
  return m < W + SHARD_PM_EDGE || m >= T_m - (W + SHARD_PM_EDGE);
}

// SH (speculative date shard): carry_out is instead a [5][N] end-state record -- present
// months of the shard, the pending ranked row (month index, -1 none), its subset-ffilled
// price, and the first / last present month (-1 none) -- for k_shard_summary_state and
// k_shard_repair.
// BL (VEC 2): day rows by raw buffer loads (see load_month).
// HALO (with SH, the halo date-shard pass): month_start holds ha.H halo months, the shard's
// T_m months and ha.F forward months; a prologue does k_halo_pm + k_shard_halo's work for the
// lane's assets -- the halo months' and forward months' prices (the month's last day row, a walk
// back where it holds no price), the scan state the halo leaves from an empty state, its flags
// (ha.flags) -- and the shard's scan continues from that state in the same registers / LDS ring,
// the forward price finishing the pending ranked row: the same state, so the same outputs, as
// k_shard_halo -> k_signal<SH> (csm_signal_shard_halo), without two launches and their
// dependent walks between them.
struct HaloArgs {
  int H, F, before, after;
  uint8_t* flags;
};
#define HALO_BATCH 8   // halo / forward months per prologue batch (LDS: [8][RS] prices + lists)
template <int MAXD, int VEC, int NBUF, int BW, bool SH, bool BL, int JC = 0, bool HALO = false>
__global__ __launch_bounds__(64 * BW) void k_signal(
    const double* __restrict__ P, const int64_t* __restrict__ month_start, int T_m, int64_t N,
    int J, int skip, double* __restrict__ PMo, double* __restrict__ R, double* __restrict__ M,
    double* __restrict__ NR, const double* __restrict__ carry, const double* __restrict__ next_pm,
    double* __restrict__ carry_out, int64_t T_d, uint16_t* __restrict__ IDS, HaloArgs ha) {
  static_assert(!HALO || (SH && VEC == 2), "the halo prologue: shard passes, paired lanes");
  typedef typename RowT<VEC>::T VT;
  extern __shared__ __attribute__((aligned(16))) double ring_lds[];  // [W][64 * VEC * BW]
  const int W = J + skip;
  const int tid = threadIdx.x;
  const int64_t a0 = ((int64_t)blockIdx.x * 64 * BW + tid) * VEC;
  const bool live = a0 < N;
  const int RS = 64 * VEC * BW;
  ScanLane sl[VEC];
  // SH counters live in LDS after the ring ([3][RS] ints: present months, first, last present
  // month): the kernel already holds ~500 registers, and these are touched once per month
  int* shc = reinterpret_cast<int*>(ring_lds + W * RS);
#pragma unroll
  for (int k = 0; k < VEC; ++k) {
    scan_init(sl[k], ring_lds + VEC * tid + k, RS, W, HALO ? nullptr : carry, N, a0 + k, live);
    if (SH) {
      shc[VEC * tid + k] = 0;
      shc[RS + VEC * tid + k] = -1;
      shc[2 * RS + VEC * tid + k] = -1;
    }
  }
  double npmh[VEC];   // HALO: the forward price of each asset (csm_shard_halo's next_pm)
  if constexpr (HALO) {
    // Months in batches of HU: each lane loads its two assets' last day row of every month of
    // the batch (one 16-B load a month, all in flight); the cells whose last day holds no price
    // (a missing day, a listing, a delisting, an absent month) are listed per wave and walked
    // back by the wave's lanes in parallel, a cell per lane (halo_month_price); then each lane
    // scans its halo months from an empty state (k_shard_halo's scan_shadow) and takes the first
    // forward month with a row as the forward price.  LDS after the ring and the SH counters:
    // the batch's month prices [HU][RS] and each wave's list of cells to walk.
    constexpr int HU = HALO_BATCH;
    const int64_t* ms = month_start;
    const int H = ha.H, F = ha.F, HF = H + F;
    const int64_t as = live ? a0 : 0;
    const int lane = tid & 63, wv = tid >> 6;
    const int64_t aw = a0 - 2 * lane;   // the wave's first asset
    double* hpw = ring_lds + (size_t)W * RS + (size_t)(3 * RS) / 2;
    uint16_t* wl = reinterpret_cast<uint16_t*>(hpw + HU * RS) + wv * (HU * 128);
    int nh[VEC], fv[VEC], lv[VEC];
#pragma unroll
    for (int c = 0; c < VEC; ++c) { nh[c] = 0; fv[c] = -1; lv[c] = -1; npmh[c] = absent_val(); }
    for (int j0 = 0; j0 < HF; j0 += HU) {   // (block-uniform)
      double2 xl[HU];
#pragma unroll
      for (int u = 0; u < HU; ++u) {
        const int j = j0 + u;
        const int m = j < H ? j : j + T_m;   // halo month j, or forward month j - H
        xl[u] = make_double2(absent_val(), absent_val());
        if (j < HF) {
          const int64_t d0 = ms[m], d1 = ms[m + 1];
          if (d1 > d0) xl[u] = *reinterpret_cast<const double2*>(P + (d1 - 1) * N + as);
        }
      }
      int nit = 0;   // wave-uniform
#pragma unroll
      for (int u = 0; u < HU; ++u) {
        *reinterpret_cast<double2*>(hpw + u * RS + 2 * tid) = xl[u];
#pragma unroll
        for (int c = 0; c < VEC; ++c) {
          const double x = comp(xl[u], c);
          const bool need = live && j0 + u < HF && !(x == x);
          const uint64_t mk = __ballot(need);
          if (need) wl[nit + lane_prefix(mk)] = (uint16_t)(u * 128 + 2 * lane + c);
          nit += __popcll(mk);
        }
      }
      __builtin_amdgcn_wave_barrier();
      // the walks, a cell per lane and two cells per lane at once: the month's day rows before
      // its last (known to hold no price) in one batch of loads per cell, all in flight
      for (int it0 = 0; it0 < nit; it0 += 128) {   // (wave-uniform)
        int item[2], u[2];
        int64_t d0[2], d1[2];
        double xs[2][HALO_WALK];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int it = it0 + 64 * h + lane;
          item[h] = it < nit ? (int)wl[it] : -1;
          u[h] = item[h] >> 7;
          const int j = j0 + (item[h] < 0 ? 0 : u[h]);
          const int m = j < H ? j : j + T_m;
          d0[h] = ms[m];
          d1[h] = ms[m + 1];
          const int64_t a = aw + (item[h] & 127);
#pragma unroll
          for (int k = 0; k < HALO_WALK; ++k) {
            const int64_t d = d1[h] - 2 - k;
            xs[h][k] = (item[h] >= 0 && d >= d0[h]) ? P[d * N + a] : absent_val();
          }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          if (item[h] < 0) continue;
          const int64_t a = aw + (item[h] & 127);
          const double xlast = hpw[u[h] * RS + 128 * wv + (item[h] & 127)];
          bool p = !is_absent(xlast), got = false;
          double x = 0.0;
#pragma unroll
          for (int k = 0; k < HALO_WALK; ++k) {
            if (!got && xs[h][k] == xs[h][k]) { x = xs[h][k]; got = true; }
            p |= !is_absent(xs[h][k]);
          }
          if (!got && d1[h] - 1 - HALO_WALK > d0[h]) {   // months longer than the batch (rare)
            const double y = halo_month_price(P, d0[h], d1[h] - 1 - HALO_WALK, N, a);
            if (y == y) { x = y; got = true; }
            p |= !is_absent(y);
          }
          hpw[u[h] * RS + 128 * wv + (item[h] & 127)] = got ? x : (p ? qnan() : absent_val());
        }
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < HU; ++u) {
        const int j = j0 + u;
        if (j >= HF) break;
#pragma unroll
        for (int c = 0; c < VEC; ++c) {
          const double x = hpw[u * RS + 2 * tid + c];
          if (j < H) {
            if (live && !is_absent(x)) {
              if (!isnan_d(x)) { if (fv[c] < 0) fv[c] = nh[c]; lv[c] = nh[c]; }
              ++nh[c];
              scan_shadow(sl[c], x, j, ring_lds + VEC * tid + c, RS, W, J);
            }
          } else if (is_absent(npmh[c])) {
            npmh[c] = x;
          }
        }
      }
      __syncthreads();   // (the batch's LDS is the next batch's)
    }
#pragma unroll
    for (int c = 0; c < VEC; ++c) {
      sl[c].prev = -1;   // (the halo's pending row is the previous rank's: scan_init's state)
      uint8_t fl = 0;
      if (ha.before && !(fv[c] >= 0 && lv[c] - fv[c] >= W)) fl |= 1;
      if (ha.after && is_absent(npmh[c])) fl |= 2;
      if (live && ha.flags) ha.flags[a0 + c] = fl;
    }
    month_start += H;   // the shard's months from here on
  }
  const double* base = P + (live ? a0 : 0);
  const int64_t rstride = N;
  // Loads are issued unconditionally (months past the end re-load the last month: cache
  // hits) so every wait is a counted vmcnt; only the processing is guarded.
  // BL: raw buffer loads over a per-month resource that ends at the month's last day row, so
  // the padding loads past it are out of range: counted by vmcnt like any load, but they return
  // 0 without a memory request (process masks them by the wave-uniform row count).
  static_assert(!BL || VEC == 2, "buffer loads: paired lanes");
  const int voff = (int)((live ? a0 : 0) * 8);
  auto load_month = [&](VT (&buf)[MAXD], int mm) {
    mm = mm < T_m ? mm : T_m - 1;
    const int64_t f0 = month_start[mm], nn = month_start[mm + 1] - f0;
    if constexpr (BL) {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(P + f0 * N), (short)0, (int)(nn * N * 8), 0x00020000);
#pragma unroll
      for (int k = 0; k < MAXD; ++k) {
        const u32x4 w = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + k * (int)(N * 8), 0, 0);
        buf[k] = *reinterpret_cast<const VT*>(&w);
      }
    } else {
#pragma unroll
      for (int k = 0; k < MAXD; ++k)
        buf[k] = *reinterpret_cast<const VT*>(base + (f0 + (k < nn ? k : nn - 1)) * rstride);
    }
  };
  auto process = [&](const VT (&X)[MAXD], int m) {
    double pm[VEC];
    const int nnm = BL ? (int)(month_start[m + 1] - month_start[m]) : MAXD;
#pragma unroll
    for (int c = 0; c < VEC; ++c) {
      double last = 0.0;
      bool p = false, v = false;
#pragma unroll
      for (int k = 0; k < MAXD; ++k) {
        const double x = comp(X[k], c);
        const bool in = !BL || k < nnm;   // wave-uniform
        const bool ok = in && x == x;  // a valid price (ABSENT and missing are NaN)
        p |= in && !is_absent(x);
        v |= ok;
        last = ok ? x : last;
      }
      pm[c] = p ? (v ? last : qnan()) : absent_val();
      if (SH && p) {
        int* q = shc + VEC * tid + c;
        q[0] += 1;
        if (q[RS] < 0) q[RS] = m;
        q[2 * RS] = m;
      }
    }
    if (live) {
      if (PMo && (!SH || shard_pm_kept(m, T_m, W))) {
        if (VEC == 2) *reinterpret_cast<double2*>(PMo + (int64_t)m * N + a0) = make_double2(pm[0], pm[VEC - 1]);
        else PMo[(int64_t)m * N + a0] = pm[0];
      }
      double mom[VEC];
      if constexpr (VEC == 2) {   // paired 16-B stores (R / M / NR are 16-B aligned)
        scan_step_pair<JC>(reinterpret_cast<ScanLane (&)[2]>(sl), reinterpret_cast<const double (&)[2]>(pm),
                       m, ring_lds + VEC * tid, RS, W, J, N, a0, R, M, NR,
                       reinterpret_cast<double (&)[2]>(mom));
      } else {
#pragma unroll
        for (int c = 0; c < VEC; ++c)
          mom[c] = scan_step(sl[c], pm[c], m, ring_lds + VEC * tid + c, RS, W, J, N, a0 + c, R, M, NR);
      }
      if (IDS) {   // fixed-map bucket ids for the decile pass (csm_signal_ids)
#ifdef SIG_HIST
        // A/B only (verdict r05 #4): the cost of a per-month id histogram built here by
        // integer atomics ([T_m][8192] u32, the decile pass's bucket of each ranked id)
        if (g_sig_hist) {
#pragma unroll
          for (int c = 0; c < VEC; ++c) {
            const uint32_t id = csm_fid(mom[c]);
            if (id != CSM_FB_NAN) atomicAdd(g_sig_hist + (int64_t)m * 8192 + (id >> 3), 1u);
          }
        }
#endif
        if (VEC == 2)
          *reinterpret_cast<uint32_t*>(IDS + (int64_t)m * N + a0) =
              csm_fid(mom[0]) | (csm_fid(mom[VEC - 1]) << 16);
        else
          IDS[(int64_t)m * N + a0] = (uint16_t)csm_fid(mom[0]);
      }
    }
  };
  static_assert(NBUF == 2 || NBUF == 4, "two or four month buffers");
  VT A[MAXD], B[MAXD];
  if (NBUF == 2) {
    // month m+1 in flight while month m is reduced (half the registers: two waves per SIMD)
    load_month(A, 0);
    for (int m = 0; m < T_m; m += 2) {
      load_month(B, m + 1);
      process(A, m);
      load_month(A, m + 2);
      if (m + 1 < T_m) process(B, m + 1);
    }
  } else {
    // months m+1..m+3 in flight (the whole-history-per-wave pattern needs ~3 months in
    // flight to approach the row-stream rate, see scripts/mb)
    VT C[MAXD], D[MAXD];
    load_month(A, 0);
    load_month(B, 1);
    load_month(C, 2);
    for (int m = 0; m < T_m; m += 4) {
      load_month(D, m + 3);
      process(A, m);
      load_month(A, m + 4);
      if (m + 1 < T_m) process(B, m + 1);
      load_month(B, m + 5);
      if (m + 2 < T_m) process(C, m + 2);
      load_month(C, m + 6);
      if (m + 3 < T_m) process(D, m + 3);
    }
  }
  if (live) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      if constexpr (HALO) {   // scan_finish's pending row, with the prologue's forward price
        if (sl[k].prev >= 0) {
          double nr = qnan();
          const double x = npmh[k];
          if (!is_absent(x)) {
            const double ps_new = isnan_d(x) ? sl[k].psff : x;
            nr = ps_new / sl[k].psff - 1.0;
          }
          NR[(int64_t)sl[k].prev * N + a0 + k] = nr;
        }
      } else {
        scan_finish(sl[k], ring_lds + VEC * tid + k, RS, W, N, a0 + k, NR, next_pm,
                    SH ? nullptr : carry_out);
      }
      if (SH) {
        const int* q = shc + VEC * tid + k;
        carry_out[a0 + k] = (double)q[0];
        carry_out[N + a0 + k] = (double)sl[k].prev;
        carry_out[2 * N + a0 + k] = sl[k].psff;
        carry_out[3 * N + a0 + k] = (double)q[RS];
        carry_out[4 * N + a0 + k] = (double)q[2 * RS];
      }
    }
  }
}

// =====================================================================================
#define DEC_THREADS 512
#define HB 8192
#define CAP 4096
// label pass: 8 x 32 B of M / NR in flight per lane (128 VGPRs: still two 512-thread
// workgroups per CU): labels 117 -> 110 us per row at C4.  Row sweeps keep ROW_U = 8 (10 made
// the histogram pass 3 us slower; profiles/r01/experiments/dec_unroll_ab.log)
#ifndef DEC_LU
#define DEC_LU 8
#endif
namespace dec_wide {
#include "deciles.inc"
}  // namespace dec_wide
using dec_wide::k_deciles;
#undef DEC_THREADS
#undef HB
#undef CAP
#undef DEC_LU

// =====================================================================================
// Kernel E: long-short series (one workgroup; T_m * n_bins is tiny).  LS_THREADS threads: a
// thread's first month's counts and means are loaded before the leg-presence barrier and kept
// for its long-short (one round trip where T_m <= LS_THREADS, instead of a flag pass and a
// second pass over the months).
// =====================================================================================
#define LS_THREADS 512
__global__ __launch_bounds__(LS_THREADS) void k_long_short(const double* __restrict__ EW,
                                                           const int32_t* __restrict__ CNT,
                                                           int T_m, int nb,
                                                           double* __restrict__ LS) {
  __shared__ int has_lo, has_hi;
  const int t0 = threadIdx.x;
  int cv[MAXQ - 1];
  double ev[MAXQ - 1];
  auto load_row = [&](int t) {
    const double* e = EW + (int64_t)t * nb;
    const int32_t* c = CNT + (int64_t)t * nb;
#pragma unroll
    for (int d = 0; d < MAXQ - 1; ++d) {   // the row's counts and means, all loads in flight
      cv[d] = d < nb ? c[d] : 0;
      ev[d] = d < nb ? e[d] : 0.0;
    }
  };
  auto legs_of = [&](int& lo_c, int& hi_c) {   // the row's decile-0 / decile-(nb-1) counts
#pragma unroll
    for (int d = 0; d < MAXQ - 1; ++d) {
      if (d == 0) lo_c = cv[d];
      if (d == nb - 1) hi_c = cv[d];
    }
  };
  auto ls_of = [&](bool both) {
    bool any = false;
    double mx = -INFINITY, mn = INFINITY, lo = 0.0, hi = 0.0;
#pragma unroll
    for (int d = 0; d < MAXQ - 1; ++d) {
      if (cv[d] > 0) { any = true; mx = fmax(mx, ev[d]); mn = fmin(mn, ev[d]); }
      if (d == 0) lo = ev[d];
      if (d == nb - 1) hi = ev[d];
    }
    double v = qnan();
    if (any) v = both ? (hi - lo) : (mx - mn);
    return v;
  };
  if (t0 < T_m) load_row(t0);
  if (t0 == 0) { has_lo = 0; has_hi = 0; }
  __syncthreads();
  if (t0 < T_m) {
    int lc = 0, hc = 0;
    legs_of(lc, hc);
    if (lc > 0) atomicOr(&has_lo, 1);
    if (hc > 0) atomicOr(&has_hi, 1);
  }
  for (int t = t0 + LS_THREADS; t < T_m; t += LS_THREADS) {
    if (CNT[(int64_t)t * nb] > 0) atomicOr(&has_lo, 1);
    if (CNT[(int64_t)t * nb + nb - 1] > 0) atomicOr(&has_hi, 1);
  }
  __syncthreads();
  const bool both = has_lo && has_hi;
  if (t0 < T_m) LS[t0] = ls_of(both);
  for (int t = t0 + LS_THREADS; t < T_m; t += LS_THREADS) {
    load_row(t);
    LS[t] = ls_of(both);
  }
}

// =====================================================================================
// Date-shard exchange records (multi-GPU date sharding).
// =====================================================================================
#define SUM_SCALARS 6

__global__ __launch_bounds__(256) void k_shard_summary(const double* __restrict__ PM, int T_m,
                                                       int64_t N, int T, double* __restrict__ out) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= N) return;
  int64_t n = 0, fv = -1, lvi = -1;
  double lv = qnan(), first = absent_val();
  for (int m = 0; m < T_m; ++m) {
    const double x = PM[(int64_t)m * N + a];
    if (is_absent(x)) continue;
    if (n == 0) first = x;
    if (!isnan_d(x)) { if (fv < 0) fv = n; lvi = n; lv = x; }
    ++n;
  }
  // tail: last T present rows, oldest first; head: last valid among rows [0, n-T)
  const int k = (int)(n < T ? n : T);
  int got = 0;
  double head = qnan();
  for (int j = 0; j < T - k; ++j) out[(int64_t)(SUM_SCALARS + j) * N + a] = absent_val();
  int m = T_m - 1;
  for (; m >= 0 && got < k; --m) {
    const double x = PM[(int64_t)m * N + a];
    if (is_absent(x)) continue;
    out[(int64_t)(SUM_SCALARS + T - 1 - got) * N + a] = x;
    ++got;
  }
  for (; m >= 0; --m) {
    const double x = PM[(int64_t)m * N + a];
    if (is_absent(x)) continue;
    if (!isnan_d(x)) { head = x; break; }
  }
  out[0 * N + a] = (double)n;
  out[1 * N + a] = (double)fv;
  out[2 * N + a] = (double)lvi;
  out[3 * N + a] = lv;
  out[4 * N + a] = head;
  out[5 * N + a] = first;
}

// Month loads in batches of SUM_U (independent loads issued together; the walks below were
// one dependent round trip per month: C2 summary 15.5 us, fold 28.3 us).
#define SUM_U 8
__global__ __launch_bounds__(256) void k_shard_summary_chunked(const double* __restrict__ PM,
                                                               int T_m, int64_t N, int T, int G,
                                                               double* __restrict__ out) {
  const int g = blockIdx.y;
  int m0, m1;
  chunk_range(T_m, G, g, m0, m1);
  const int S = SUM_SCALARS + T;
  // reuse the single-shard body through pointer offsets (grid.x covers the assets)
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= N) return;
  const double* pm = PM + (int64_t)m0 * N;
  double* o = out + (int64_t)g * S * N;
  const int tm = m1 - m0;
  int64_t n = 0, fv = -1, lvi = -1;
  double lv = qnan(), first = absent_val();
  for (int mb = 0; mb < tm; mb += SUM_U) {
    double xs[SUM_U];
#pragma unroll
    for (int u = 0; u < SUM_U; ++u) xs[u] = mb + u < tm ? pm[(int64_t)(mb + u) * N + a] : absent_val();
#pragma unroll
    for (int u = 0; u < SUM_U; ++u) {
      const double x = xs[u];
      if (is_absent(x)) continue;
      if (n == 0) first = x;
      if (!isnan_d(x)) { if (fv < 0) fv = n; lvi = n; lv = x; }
      ++n;
    }
  }
  const int k = (int)(n < T ? n : T);
  int got = 0;
  double head = qnan();
  for (int j = 0; j < T - k; ++j) o[(int64_t)(SUM_SCALARS + j) * N + a] = absent_val();
  // backward: the last k present rows (oldest first in the record), then the last valid price
  // before them
  bool done = false;
  for (int mb = tm - 1; mb >= 0 && !done; mb -= SUM_U) {
    double xs[SUM_U];
#pragma unroll
    for (int u = 0; u < SUM_U; ++u) xs[u] = mb - u >= 0 ? pm[(int64_t)(mb - u) * N + a] : absent_val();
#pragma unroll
    for (int u = 0; u < SUM_U; ++u) {
      const double x = xs[u];
      if (done || mb - u < 0 || is_absent(x)) continue;
      if (got < k) {
        o[(int64_t)(SUM_SCALARS + T - 1 - got) * N + a] = x;
        ++got;
      } else if (!isnan_d(x)) {
        head = x;
        done = true;
      }
    }
  }
  o[0 * N + a] = (double)n;
  o[1 * N + a] = (double)fv;
  o[2 * N + a] = (double)lvi;
  o[3 * N + a] = lv;
  o[4 * N + a] = head;
  o[5 * N + a] = first;
}

// psq (csm_momentum_multi_chunked): also the subset-ffilled price of every look-back jq.J[q]
// of the multi-J scan (the ranked subset starts J + skip present rows after the first valid
// price), [G][MJ_MAX][N]; the ring and pff are J's own for J = max(J) and shared by the others.
struct FoldJs {
  int n;
  int J[MJ_MAX];
};
// The fold of k_fold_carry for asset (column) a: the scan state at shard g's first month from
// the exchange records of shards < g (ring factors oldest first, then pff, psff: rows 0..W + 1
// through store(row, value)), and the first present price after shard g (returned).
template <class Store>
__device__ __forceinline__ double fold_body(const double* __restrict__ sm, int G, int g,
                                            int64_t N, int64_t a, int J, int skip,
                                            const double* __restrict__ tail_pm, Store store,
                                            const FoldJs& jq, double* __restrict__ psq) {
  const int W = J + skip, T = W + 1, S = SUM_SCALARS + T;
  const double NaN = qnan();
  // the neighbours' scalars in one round trip (the walks below start there and usually end
  // there): chunk g - 1's record scalars, chunk g + 1's count and first price
  double pg[SUM_SCALARS], ng0 = 0.0, ng5 = absent_val();
#pragma unroll
  for (int r = 0; r < SUM_SCALARS; ++r) pg[r] = g > 0 ? sm[((int64_t)(g - 1) * S + r) * N + a] : NaN;
  if (g + 1 < G) {
    ng0 = sm[((int64_t)(g + 1) * S) * N + a];
    ng5 = sm[((int64_t)(g + 1) * S + 5) * N + a];
  }
  auto at = [&](int h, int r) -> double { return sm[((int64_t)h * S + r) * N + a]; };
  // a record scalar (r a constant < SUM_SCALARS): chunk g - 1's from registers
  auto sc = [&](int h, int r) -> double { return h == g - 1 ? pg[r] : at(h, r); };
  // next_pm: first present row after shard g
  double npm = (tail_pm && g == G - 1) ? tail_pm[a] : absent_val();
  if (g + 1 < G) {
    if (ng0 > 0.0) npm = ng5;
    else for (int h = g + 2; h < G; ++h) if (sc(h, 0) > 0.0) { npm = sc(h, 5); break; }
  }
  if (tail_pm && g < G - 1 && is_absent(npm)) npm = tail_pm[a];
  // locate the oldest of the last T present rows of shards < g
  int nv = 0, src_h = -1, src_j = -1;
  for (int h = g - 1; h >= 0 && nv < T; --h) {
    const int k = (int)fmin(sc(h, 0), (double)T);
    const int take = k < T - nv ? k : T - nv;
    if (take > 0) { nv += take; src_h = h; src_j = T - take; }
  }
  double pff_before = NaN;
  if (nv > 0) {
    const int k0 = (int)fmin(sc(src_h, 0), (double)T);
    for (int j = src_j - 1; j > T - 1 - k0; --j) { const double x = at(src_h, SUM_SCALARS + j); if (!isnan_d(x)) { pff_before = x; break; } }
    if (isnan_d(pff_before)) pff_before = sc(src_h, 4);
    if (isnan_d(pff_before))
      for (int h = src_h - 1; h >= 0; --h) if (!isnan_d(sc(h, 3))) { pff_before = sc(h, 3); break; }
  }
  // replay oldest -> newest; the newest W rets become the ring (as factors fl(1+ret))
  double pff = pff_before;
  for (int k = 0; k < W; ++k) store(k, NaN);
  int c = 0;
  for (int h = src_h; h >= 0 && h < g; ++h) {
    const int kh = (int)fmin(sc(h, 0), (double)T);
    for (int jb = (h == src_h) ? src_j : T - kh; jb < T; jb += SUM_U) {   // SUM_U rows in flight
      double xs[SUM_U];
#pragma unroll
      for (int u = 0; u < SUM_U; ++u) xs[u] = jb + u < T ? at(h, SUM_SCALARS + jb + u) : NaN;
#pragma unroll
      for (int u = 0; u < SUM_U; ++u) {
        if (jb + u >= T) break;
        const double x = xs[u];
        const double nx = isnan_d(x) ? pff : x;
        const double ret = nx / pff - 1.0;
        pff = nx;
        const int pos = c - (nv - W);
        if (pos >= 0) store(pos, 1.0 + ret);
        ++c;
      }
    }
  }
  double lastv = NaN;
  for (int h = g - 1; h >= 0; --h) if (!isnan_d(sc(h, 3))) { lastv = sc(h, 3); break; }
  store(W, lastv);
  int64_t off = 0, f = -1;
  for (int hb = 0; hb < g; hb += SUM_U) {   // every earlier chunk's counts, SUM_U in flight
    double cn[SUM_U], fi[SUM_U];
#pragma unroll
    for (int u = 0; u < SUM_U; ++u) {
      cn[u] = hb + u < g ? at(hb + u, 0) : 0.0;
      fi[u] = hb + u < g ? at(hb + u, 1) : -1.0;
    }
#pragma unroll
    for (int u = 0; u < SUM_U; ++u) {
      if (hb + u >= g) break;
      if (f < 0 && fi[u] >= 0.0) f = off + (int64_t)fi[u];
      off += (int64_t)cn[u];
    }
  }
  // last valid price among the ranked rows of look-back Jq (rows >= f + Jq + skip)
  auto psff_of = [&](int Jq) {
    double ps = NaN;
    if (f >= 0) {
      int64_t offh = off;
      for (int h = g - 1; h >= 0; --h) {
        offh -= (int64_t)sc(h, 0);
        if (sc(h, 2) >= 0.0) {
          const int64_t li = offh + (int64_t)sc(h, 2);
          if (li >= f + Jq + skip) ps = sc(h, 3);
          break;
        }
      }
    }
    return ps;
  };
  store(W + 1, psff_of(J));
  if (psq)
    for (int q = 0; q < jq.n; ++q) psq[((int64_t)g * MJ_MAX + q) * N + a] = psff_of(jq.J[q]);
  return npm;
}

__global__ __launch_bounds__(256) void k_fold_carry(const double* __restrict__ sm, int G, int g,
                                                    int64_t N, int J, int skip,
                                                    double* __restrict__ carry,
                                                    double* __restrict__ next_pm,
                                                    const double* __restrict__ tail_pm,
                                                    FoldJs jq, double* __restrict__ psq) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= N) return;
  const int W = J + skip;
  if (g < 0) {  // batched over all chunks: chunk blockIdx.y, outputs stacked per chunk
    g = blockIdx.y;
    carry += (int64_t)g * (W + 2) * N;
    next_pm += (int64_t)g * N;
  }
  next_pm[a] = fold_body(sm, G, g, N, a, J, skip, tail_pm,
                         [&](int k, double v) { carry[(int64_t)k * N + a] = v; }, jq, psq);
}

// =====================================================================================
// Kernel AB-TC: month-end + time-chunked scan in ONE launch, for narrow panels (C2: 5,000
// assets, where one wave per 128 assets walking all 300 months leaves the chip idle and the
// unfused path costs four launches: k_month_end, k_shard_summary_chunked, k_fold_carry,
// k_momentum_chunked).  A workgroup owns (chunk g, 256-asset column x).
//   1. Its eight waves reduce the chunk's daily rows to month prices in LDS (wave w: asset
//      half w % 2, months w / 2, w / 2 + 4, ...: four months of each half in flight).
//   2. Its first four waves (one asset per lane) build the chunk's exchange record from them
//      (k_shard_summary_chunked's fields + the last present month) and publish it.
//   3. They wait for the records of chunks 0..g-1 of the column and
//   4. fold them into the scan state at the chunk's first month: the newest T = W + 1
//      present month prices (k_fold_carry's window) are replayed into the ring.  WR > 0
//      (compile-time W): the window is located from the present-row counts, 16 chunks per
//      load trip, and read from at most three chunks' tails (two trips for a dense asset);
//      histories it does not settle (a window over four or more chunks, a last present month
//      with no valid price, a NaN window start with no earlier price in the loaded rows) take
//      k_fold_carry's general walk, as WR = 0 does for every asset.
//   5. They scan the chunk's months from LDS (WR > 0: the ring in registers).
// The pending ranked row at a chunk's end is not finished with a forward price: the chunk with
// the asset's next present row writes its next_ret (the fold hands it the pending month when
// the rebuilt ring says that row ranked -- exactly when the chunk that scanned it left it
// pending, so one writer per cell), as the sequential scan does; the last chunk writes NaN for
// one still pending.  Same factors, same order, same divisions as k_month_end -> k_momentum:
// bit-identical R / M / NR / ids.
// Hand-off (MI355X_MICROARCH.md, visibility, row 1): records stored write-through (agent
// relaxed atomic stores), every storing wave drains (vmcnt 0), a barrier, ONE lane stores the
// flag; the consumer polls the flags with relaxed agent loads (one wave, a lane per flag: all
// of them in one load per trip), ONE agent acquire, a barrier, plain loads.  Workgroups take tickets in arrival order and ticket t is chunk t / nbx, so
// every record a workgroup waits for belongs to an earlier ticket -- a workgroup already
// running: no residency assumption.  Spins are bounded (timeout word).  The last workgroup to
// finish zeroes the flags; the ticket and done counters wrap to 0 themselves, so the sync
// words are zero again for the next launch (or graph replay).
// sync [0] ticket, [1] done, [2] timeout, [3] pad, [4 ..) flags [G][nbx].  Records
// [G][nbx][SR][256] f64: one (chunk, column)'s record is whole cache lines of its own.
// =====================================================================================
#ifndef TC_THREADS
#define TC_THREADS 512   // eight waves reduce months; the first four fold and scan
#endif
#ifndef TC_COLS
#define TC_COLS 256      // assets per workgroup (a multiple of 128)
#endif
#define TC_HALVES (TC_COLS / 128)                    // 128-asset slices of a column
#define TC_MONTH_WAVES (TC_THREADS / 64 / TC_HALVES)   // month slots per slice
#define TC_MAXD 23       // day rows per month (a business month)
#define TC_MAXG 64       // chunks
#define TC_MAXC 32       // months per chunk
#define TC_SYNC0 4       // sync words before the flags
#define TC_SPINS (1u << 21)
#define TC_NC 16         // chunk counts per load trip of the window search
#ifndef TC_GW
#define TC_GW 4          // chunks per load trip of the general fold walk
#endif
#ifndef TC_LBW
#define TC_LBW 4         // launch bound: waves per SIMD the VGPR budget must allow
#endif
#ifndef TC_REC2
#define TC_REC2 1        // the record's forward and backward fields by the two wave halves
#endif
// -DTC_TIMING (experiment builds, scripts/build_variant.py): per-workgroup phase stamps
// (wall clock, 100 MHz) in 8 u64 words per ticket after the records (workspace grows)
#ifdef TC_TIMING
#define TC_STAMP(k) do { if (tid == 0) stamp[k] = wall_clock64(); } while (0)
#else
#define TC_STAMP(k) do { } while (0)
#endif

typedef __attribute__((address_space(1))) unsigned int tc_gu32;
typedef __attribute__((address_space(1))) unsigned long long tc_gu64;

__device__ __forceinline__ void tc_put(double* p, double v) {   // write-through (sc1) store
  __hip_atomic_store((tc_gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// scan_step with the ring in registers, oldest first (the same factors, product order and
// stores as scan_step's LDS ring).  JC > 0: J is the compile-time JC (the product's factor
// count folds: no per-factor select).
template <int WR, int JC = 0>
__device__ __forceinline__ double scan_step_reg(ScanLane& s, double x, int m, double (&fr)[WR],
                                                int J, int64_t N, int64_t a,
                                                double* __restrict__ R, double* __restrict__ M,
                                                double* __restrict__ NR) {
  const double NaN = qnan();
  const int64_t o = (int64_t)m * N + a;
  if (is_absent(x)) {
    if (R) R[o] = NaN;
    M[o] = NaN;
    NR[o] = NaN;
    return NaN;
  }
  const bool xv = !isnan_d(x);
  const double pnew = xv ? x : s.pff;
  const double ret = pnew / s.pff - 1.0;
  s.pff = pnew;
#pragma unroll
  for (int k = 0; k + 1 < WR; ++k) fr[k] = fr[k + 1];
  fr[WR - 1] = 1.0 + ret;
  double acc = fr[0];
#pragma unroll
  for (int k = 1; k < WR; ++k)
    if (k < (JC > 0 ? JC : J)) acc = acc * fr[k];
  const double mom = acc - 1.0;
  const bool ranked = !isnan_d(mom);
  const double ps_new = xv ? x : s.psff;
  if (s.prev >= 0) NR[(int64_t)s.prev * N + a] = ps_new / s.psff - 1.0;
  if (ranked) {
    s.psff = ps_new;
    s.prev = m;
  } else {
    NR[o] = NaN;
    s.prev = -1;
  }
  if (R) R[o] = ret;
  M[o] = mom;
  return mom;
}

// k_fold_carry's general walk for chunk g of one asset (column pointer cp, chunk stride hs):
// the ring into LDS (ring[k * RS], oldest first), returns pff / psff / the pending month.
__device__ __forceinline__ void tc_fold_general(const double* cp, int64_t hs, int g, int W,
                                                int J, double* ring, int RS, ScanLane& sl) {
  const int T = W + 1, SR = SUM_SCALARS + T + 1;
  const double NaN = qnan();
  auto at = [&](int h, int r) -> double { return cp[(int64_t)h * hs + (int64_t)r * TC_COLS]; };
  for (int k = 0; k < W; ++k) ring[k * RS] = NaN;
  int64_t s = 0;          // present rows of chunks h..g-1
  int64_t frel = 0, lrel = 0;
  bool hasf = false, haslv = false, below = false;
  double lvlast = NaN, lvbelow = NaN;
  int lpm = -1, nv = 0, src_h = -1, src_j = -1;
  for (int hb = g - 1; hb >= 0; hb -= TC_GW) {   // one backward pass, TC_GW chunks per trip
    double n4[TC_GW], f4[TC_GW], li4[TC_GW], lv4[TC_GW], lp4[TC_GW];
#pragma unroll
    for (int u = 0; u < TC_GW; ++u) {
      const int h = hb - u >= 0 ? hb - u : 0;
      n4[u] = at(h, 0); f4[u] = at(h, 1); li4[u] = at(h, 2); lv4[u] = at(h, 3);
      lp4[u] = at(h, SR - 1);
    }
#pragma unroll
    for (int u = 0; u < TC_GW; ++u) {
      const int h = hb - u;
      if (h < 0) break;
      const int64_t n = (int64_t)n4[u];
      bool took = false;
      if (nv < T) {
        const int k = (int)(n < T ? n : T);
        const int take = k < T - nv ? k : T - nv;
        if (take > 0) { nv += take; src_h = h; src_j = T - take; took = true; }
      }
      if (took) below = false;
      else if (src_h >= 0 && !below && li4[u] >= 0.0) { below = true; lvbelow = lv4[u]; }
      if (lpm < 0 && n > 0) lpm = (int)lp4[u];
      if (!haslv && li4[u] >= 0.0) { haslv = true; lvlast = lv4[u]; lrel = (int64_t)li4[u] - (s + n); }
      if (f4[u] >= 0.0) { hasf = true; frel = (int64_t)f4[u] - (s + n); }
      s += n;
    }
  }
  const int64_t off = s, f = hasf ? off + frel : -1;
  double pff = NaN;   // the price before the window's oldest row
  if (nv > 0) {
    const int k0 = (int)fmin(at(src_h, 0), (double)T);
    for (int j = src_j - 1; j > T - 1 - k0; --j) {
      const double xv = at(src_h, SUM_SCALARS + j);
      if (!isnan_d(xv)) { pff = xv; break; }
    }
    if (isnan_d(pff)) pff = at(src_h, 4);
    if (isnan_d(pff) && below) pff = lvbelow;
  }
  int cc = 0;   // replay oldest -> newest; the newest W rets become the ring
  for (int h = src_h; h >= 0 && h < g; ++h) {
    const int kh = (int)fmin(at(h, 0), (double)T);
    for (int jb = (h == src_h) ? src_j : T - kh; jb < T; jb += SUM_U) {
      double xs[SUM_U];
#pragma unroll
      for (int u = 0; u < SUM_U; ++u) xs[u] = jb + u < T ? at(h, SUM_SCALARS + jb + u) : NaN;
#pragma unroll
      for (int u = 0; u < SUM_U; ++u) {
        if (jb + u >= T) break;
        const double xv = xs[u];
        const double nx = isnan_d(xv) ? pff : xv;
        const double ret = nx / pff - 1.0;
        pff = nx;
        const int pos = cc - (nv - W);
        if (pos >= 0) ring[pos * RS] = 1.0 + ret;
        ++cc;
      }
    }
  }
  sl.pff = lvlast;
  const int64_t li = off + lrel;
  sl.psff = (f >= 0 && haslv && li >= f + W) ? lvlast : NaN;   // (k_fold_carry's psff)
  // the last present row's mom_J from the rebuilt ring, in scan_step's order: ranked (its
  // next_ret still pending) exactly when the chunk that scanned it left it pending
  double acc = ring[0];
  for (int k = 1; k < J; ++k) acc = acc * ring[k * RS];
  sl.prev = (lpm >= 0 && !isnan_d(acc - 1.0)) ? lpm : -1;
}

// The window search of WR > 0 (see the kernel's comment): true when it settled the state (ring
// factors in fr, sl), false when the general walk must run.  win: this lane's LDS column of T
// rows (stride RS).
template <int WR>
__device__ __forceinline__ bool tc_fold_fast(const double* cp, int64_t hs, int g, int J,
                                             double* win, int RS, double (&fr)[WR],
                                             ScanLane& sl) {
  constexpr int T = WR + 1, SR = SUM_SCALARS + T + 1;
  const double NaN = qnan();
  auto at = [&](int h, int r) -> double { return cp[(int64_t)h * hs + (int64_t)r * TC_COLS]; };
  // trip 1: chunk g - 1's record and the counts of the 16 chunks before it
  double r1[SR], nc[TC_NC];
#pragma unroll
  for (int r = 0; r < SR; ++r) r1[r] = at(g - 1, r);
#pragma unroll
  for (int u = 0; u < TC_NC; ++u) nc[u] = g - 2 - u >= 0 ? at(g - 2 - u, 0) : 0.0;
  const int k1 = (int)fmin(r1[0], (double)T);
  const double h1 = r1[4], lp1 = r1[SR - 1], n1 = r1[0];
  int nv = k1;
  // the older chunks in the window (newest first): index, rows taken, window rows before it
  int c0 = -1, t0 = 0, b0 = 0, c1 = -1, t1 = 0, b1 = 0;
  bool over = false;
  for (int base = g - 2; base >= 0 && nv < T && !over; base -= TC_NC) {
    if (base != g - 2) {   // later trips (long absences): the next 16 counts
#pragma unroll
      for (int u = 0; u < TC_NC; ++u) nc[u] = base - u >= 0 ? at(base - u, 0) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < TC_NC; ++u) {   // (guards, not breaks: nc stays in registers)
      const int h = base - u;
      const int k = (int)fmin(nc[u], (double)T);
      if (h >= 0 && nv < T && !over && k > 0) {
        const int take = k < T - nv ? k : T - nv;
        if (c0 < 0) { c0 = h; t0 = take; b0 = nv; }
        else if (c1 < 0) { c1 = h; t1 = take; b1 = nv; }
        else over = true;
        if (!over) nv += take;
      }
    }
  }
  if (over) return false;
  if (nv == 0) {   // no present month before the chunk: the empty state
#pragma unroll
    for (int k = 0; k < WR; ++k) fr[k] = NaN;
    sl.pff = NaN; sl.psff = NaN; sl.prev = -1; sl.head = 0;
    return true;
  }
  // the window in LDS: chunk g - 1's newest k1 rows, then the older chunks' (trip 2)
#pragma unroll
  for (int j = 0; j < T; ++j)
    if (j >= T - k1) win[j * RS] = r1[SUM_SCALARS + j];   // (r1 is dead from here)
  // trip 2: the older window chunks' tails, head, last present month and count
  double x0[T + 3], x1[T + 3];
#pragma unroll
  for (int j = 0; j < T; ++j) {
    x0[j] = c0 >= 0 ? at(c0, SUM_SCALARS + j) : NaN;
    x1[j] = c1 >= 0 ? at(c1, SUM_SCALARS + j) : NaN;
  }
  x0[T] = c0 >= 0 ? at(c0, 4) : NaN;
  x1[T] = c1 >= 0 ? at(c1, 4) : NaN;
  x0[T + 1] = c0 >= 0 ? at(c0, SR - 1) : -1.0;
  x1[T + 1] = -1.0;
  x0[T + 2] = c0 >= 0 ? at(c0, 0) : 0.0;
  x1[T + 2] = c1 >= 0 ? at(c1, 0) : 0.0;
#pragma unroll
  for (int j = 0; j < T; ++j) {
    if (c0 >= 0 && j >= T - t0) win[(j - b0) * RS] = x0[j];
    if (c1 >= 0 && j >= T - t1) win[(j - b1) * RS] = x1[j];
  }
  const int lpm = k1 > 0 ? (int)lp1 : (int)x0[T + 1];
  // the last present month must hold a valid price (else the general walk's psff rule)
  const double last = win[(T - 1) * RS];
  if (isnan_d(last)) return false;
  // the price before the window's oldest row: needed when the window is the whole history
  // (its first factor is kept) or when that row has no valid price.  With nv < T every window
  // chunk gave all its rows and the count walk saw every earlier chunk empty: NaN.  Else the
  // oldest window chunk's rows before the window (newest first), then its head; not found:
  // the general walk (a valid price further back).
  const double first = win[(T - nv) * RS];
  double pff = NaN;
  if (nv == T && isnan_d(first)) {
    const int kc = (int)fmin(c1 >= 0 ? x1[T + 2] : c0 >= 0 ? x0[T + 2] : n1, (double)T);
    const int tk = c1 >= 0 ? t1 : c0 >= 0 ? t0 : k1;
    bool found = false;
#pragma unroll
    for (int j = T - 1; j >= 0; --j) {
      // (a window of chunk g - 1 alone took all its tail: no row before it to search)
      const double xv = c1 >= 0 ? x1[j] : x0[j];
      if (!found && j < T - tk && j >= T - kc && !isnan_d(xv)) { pff = xv; found = true; }
    }
    if (!found) {
      const double hd = c1 >= 0 ? x1[T] : c0 >= 0 ? x0[T] : h1;
      if (!isnan_d(hd)) { pff = hd; found = true; }
    }
    if (!found) return false;
  }
  // replay the window oldest -> newest into the ring (factor of window row j at slot j - 1)
#pragma unroll
  for (int k = 0; k < WR; ++k) fr[k] = NaN;
#pragma unroll
  for (int j = 0; j < T; ++j) {
    if (j >= T - nv) {
      const double xv = win[j * RS];
      const double nx = isnan_d(xv) ? pff : xv;
      const double ret = nx / pff - 1.0;
      pff = nx;
      if (j >= 1) fr[j - 1] = 1.0 + ret;
    }
  }
  double acc = fr[0];
#pragma unroll
  for (int k = 1; k < WR; ++k)
    if (k < J) acc = acc * fr[k];
  const bool ranked = !isnan_d(acc - 1.0);
  sl.pff = last;
  sl.psff = ranked ? last : NaN;
  sl.prev = ranked ? lpm : -1;
  sl.head = 0;
  return true;
}

template <int WR, int JC = 0>
__global__ __launch_bounds__(TC_THREADS, TC_LBW) void k_signal_tc(
    const double* __restrict__ P, const int64_t* __restrict__ month_start, int T_m, int64_t N,
    int J, int skip, int G, int nbx, double* __restrict__ R, double* __restrict__ M,
    double* __restrict__ NR, uint16_t* __restrict__ IDS, double* __restrict__ rec,
    unsigned* __restrict__ sync, unsigned spin_limit) {
  extern __shared__ __attribute__((aligned(16))) double tc_lds[];   // ring [T][256], pm [C][256]
  __shared__ int s_t, s_last;
  const int tid = threadIdx.x;
  const int W = WR > 0 ? WR : J + skip, T = W + 1, SR = SUM_SCALARS + T + 1;
  const unsigned total = (unsigned)G * (unsigned)nbx;
#ifdef TC_TIMING
  unsigned long long stamp[8];
#endif
  TC_STAMP(0);
  if (tid == 0) s_t = (int)atomicInc(sync, total - 1u);   // wraps to 0 after the last ticket
  __syncthreads();
  const int t = s_t, g = t / nbx, x = t - g * nbx;
  int m0, m1;
  chunk_range(T_m, G, g, m0, m1);
  const int RS = TC_COLS;
  double* ring = tc_lds;            // [T][256]: the general walk's ring, the fast window
  double* pmL = tc_lds + T * RS;    // [C][256]: the chunk's month prices
  const int wv = tid >> 6, lane = tid & 63;
  const bool worker = tid < TC_COLS;   // folds and scans asset la = tid (wave-uniform)
  const int la = worker ? tid : 0;
  const int64_t a = (int64_t)x * TC_COLS + la;
  const bool live = worker && a < N;
  const double NaN = qnan();

  // ---- 1. month prices of the chunk (k_signal's reduction), into LDS ----
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const int lm = 128 * (wv % TC_HALVES) + 2 * lane;   // this lane's asset pair in phase 1
  const int64_t am = (int64_t)x * TC_COLS + lm;
  const int voff = (int)((am < N ? am : 0) * 8);
  const int rowb = (int)(N * 8);
  for (int m = m0 + wv / TC_HALVES; m < m1; m += TC_MONTH_WAVES) {
    const int64_t f0 = month_start[m], nn = month_start[m + 1] - f0;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(P + f0 * N), (short)0, (int)(nn * N * 8), 0x00020000);
    double2 X[TC_MAXD];
#pragma unroll
    for (int k = 0; k < TC_MAXD; ++k) {   // rows past the month: out of range, no request
      const u32x4 w = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + k * rowb, 0, 0);
      X[k] = *reinterpret_cast<const double2*>(&w);
    }
    const int nnm = (int)nn;
    double pm[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      double last = 0.0;
      bool p = false, v = false;
#pragma unroll
      for (int k = 0; k < TC_MAXD; ++k) {
        const double xv = comp(X[k], c);
        const bool in = k < nnm;   // wave-uniform
        const bool ok = in && xv == xv;
        p |= in && !is_absent(xv);
        v |= ok;
        last = ok ? xv : last;
      }
      pm[c] = p ? (v ? last : qnan()) : absent_val();
    }
    *reinterpret_cast<double2*>(pmL + (m - m0) * RS + lm) = make_double2(pm[0], pm[1]);
  }
  __syncthreads();
  TC_STAMP(1);

  // ---- 2. this chunk's record (k_shard_summary_chunked's fields + last present month) ----
  const int64_t hstride = (int64_t)nbx * SR * RS;   // chunk stride of a column's records
  double* cp = rec + (int64_t)x * SR * RS + la;     // this asset's column of records
  const int tm = m1 - m0;
  // the forward fields (count, first valid / last valid index, last valid price, first present
  // price) by the folding waves, the backward ones (the newest T present prices, the head, the
  // last present month) by the other waves at once (TC_REC2; else one wave does both)
  constexpr bool REC2 = TC_REC2 && TC_THREADS == 2 * TC_COLS;
  const int lr = worker ? la : tid - TC_COLS;   // the record column this lane writes
  const bool fwd = worker, bwd = REC2 ? !worker : worker;
  if (worker || REC2) {
    const double* col = pmL + lr;
    double* o = rec + (int64_t)x * SR * RS + lr + (int64_t)g * hstride;
    if (fwd) {
      int n = 0, fv = -1, lvi = -1;
      double lv = NaN, first = absent_val();
      for (int j0 = 0; j0 < tm; j0 += 8) {   // 8 months' LDS loads in flight per trip
        double xs[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) xs[u] = j0 + u < tm ? col[(j0 + u) * RS] : absent_val();
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const double xv = xs[u];
          if (!is_absent(xv)) {
            if (n == 0) first = xv;
            if (!isnan_d(xv)) { if (fv < 0) fv = n; lvi = n; lv = xv; }
            ++n;
          }
        }
      }
      tc_put(o + 0 * RS, (double)n);
      tc_put(o + 1 * RS, (double)fv);
      tc_put(o + 2 * RS, (double)lvi);
      tc_put(o + 3 * RS, lv);
      tc_put(o + 5 * RS, first);
    }
    if (bwd) {
      // the newest min(n, T) present prices into the tail rows, absent fill below them
      int got = 0, lpm = -1;
      double head = NaN;
      int j = tm - 1;
      for (; j >= 0 && got < T; --j) {
        const double xv = col[j * RS];
        if (is_absent(xv)) continue;
        if (got == 0) lpm = m0 + j;
        tc_put(o + (SUM_SCALARS + T - 1 - got) * RS, xv);
        ++got;
      }
      for (int i = 0; i < T - got; ++i) tc_put(o + (SUM_SCALARS + i) * RS, absent_val());
      for (; j >= 0; --j) {
        const double xv = col[j * RS];
        if (is_absent(xv)) continue;
        if (!isnan_d(xv)) { head = xv; break; }
      }
      tc_put(o + 4 * RS, head);
      tc_put(o + (int64_t)(SR - 1) * RS, (double)lpm);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains
  __syncthreads();
  // Publication.  Every record word is itself an agent-scope atomic store (tc_put: written
  // through to the agent coherence point, never left dirty in this XCD's L2), and every storing
  // wave has waited for its stores to complete (vmcnt(0)) before the barrier, so the records are
  // visible at agent scope before the flag is issued.  That is all a release would add for
  // atomic stores on gfx950; an __ATOMIC_RELEASE store also emits buffer_wbl2 (an L2 write-back
  // of every dirty line of the XCD, the other workgroups' M / NR among them): measured +3.5 us
  // per C2 launch (k_signal_tc 76.5 -> 80.0 us, same box, round 6), so the flag stays relaxed.
  // The consumer acquires (agent fence) after it sees every flag.
  if (tid == 0)
    __hip_atomic_store((tc_gu32*)(sync + TC_SYNC0 + (int64_t)g * nbx + x), 1u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  TC_STAMP(2);

  // ---- 3. wait for the records of chunks 0..g-1 of this column ----
  if (g > 0) {
    if (tid < 64) {   // wave 0: lane h polls chunk h's flag, all g flags in one load per trip
      bool got = lane >= g;
      unsigned spins = 0;
      while (true) {
        // never expected (spin_limit 0 forces it: the tests of the failure report): give up and
        // mark the launch; csm_signal_chunked_status reports the mark as CSM_E_TIMEOUT
        if (spins >= spin_limit) {
          if (lane == 0)
            __hip_atomic_store((tc_gu32*)(sync + 2), 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        if (!got)
          got = __hip_atomic_load((const tc_gu32*)(sync + TC_SYNC0 + (int64_t)lane * nbx + x),
                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
        if (__ballot(!got) == 0ull) break;   // (wave-uniform)
        __builtin_amdgcn_s_sleep(2);
        ++spins;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  }
  TC_STAMP(3);

  // ---- 4. the scan state at month m0 ----
  ScanLane sl;
  sl.head = 0; sl.pff = NaN; sl.psff = NaN; sl.prev = -1;
  double fr[WR > 0 ? WR : 1];
#pragma unroll
  for (int k = 0; k < (WR > 0 ? WR : 1); ++k) fr[k] = NaN;
  if (worker) {
    double* rl = ring + la;
    if (g > 0 && live) {
      bool done = false;
      if constexpr (WR > 0) done = tc_fold_fast<WR>(cp, hstride, g, J, rl, RS, fr, sl);
      if (!done) {
        tc_fold_general(cp, hstride, g, W, J, rl, RS, sl);
        if constexpr (WR > 0) {
#pragma unroll
          for (int k = 0; k < WR; ++k) fr[k] = rl[k * RS];
        }
      }
    } else if (WR == 0) {
      for (int k = 0; k < W; ++k) rl[k * RS] = NaN;
    }
  }
  TC_STAMP(4);

  // ---- 5. scan the chunk's months from LDS (the next month's price read a step ahead) ----
  if (live) {
    double xn = pmL[la];
    for (int m = m0; m < m1; ++m) {
      const double xv = xn;
      if (m + 1 < m1) xn = pmL[(m + 1 - m0) * RS + la];
      double mom;
      if constexpr (WR > 0) mom = scan_step_reg<WR, JC>(sl, xv, m, fr, J, N, a, R, M, NR);
      else mom = scan_step(sl, xv, m, ring + la, RS, W, J, N, a, R, M, NR);
      if (IDS) IDS[(int64_t)m * N + a] = (uint16_t)csm_fid(mom);
    }
    if (g == G - 1 && sl.prev >= 0) NR[(int64_t)sl.prev * N + a] = NaN;   // (scan_finish)
  }

  // ---- 6. the last workgroup out zeroes the flags for the next launch ----
  __syncthreads();
  TC_STAMP(5);
#ifdef TC_TIMING
  if (tid == 0) {
    stamp[6] = (unsigned long long)g;
    stamp[7] = (unsigned long long)x;
    unsigned long long* o = reinterpret_cast<unsigned long long*>(
        rec + (int64_t)total * SR * RS) + (int64_t)t * 8;
    for (int k = 0; k < 8; ++k) o[k] = stamp[k];
  }
#endif
  if (tid == 0) s_last = atomicInc(sync + 1, total - 1u) == total - 1u;
  __syncthreads();
  if (s_last)
    for (unsigned i = tid; i < total; i += TC_THREADS) sync[TC_SYNC0 + i] = 0u;
}

// =====================================================================================
// Speculative date shards (the fused multi-GPU pass).  A rank runs k_signal<SH>
// on its month range from an EMPTY scan state (trajectory F) before the earlier shards' carry
// is known, writing PM and a [5][N] end-state record (present months, pending row, its psff,
// first / last present month).  k_shard_summary_state builds the exchange record from PM with
// short walks from both ends (no full pass).  After the all-gather and k_fold_carry,
// k_shard_repair replays each asset from the true carry (trajectory T) beside F, rewriting
// R / M / NR, until the two states are bit-identical -- from then on every output k_signal
// wrote is T's -- or the asset has no present month left; then it finishes the pending ranked
// row with next_pm (k_signal ran without it).  A dense asset converges after its first
// J + skip + 1 present months.  Bit-identical to the unfused k_month_end -> k_shard_summary ->
// k_fold_carry -> k_momentum(carry) pass.
// =====================================================================================
#define REPAIR_THREADS 64
#ifndef WALK_CHUNK
#define WALK_CHUNK 8   // months per load round of the summary / repair walks
#endif
#define REPAIR_CHUNK WALK_CHUNK

// Month price of asset a in month m of a speculative shard: PM where k_signal<SH> kept it,
// else the month-end of the daily rows (k_signal's reduction: last valid price, NaN if the
// month has rows but no price, ABSENT if none).
__device__ __forceinline__ double shard_pm_at(const double* __restrict__ PM,
                                              const double* __restrict__ P,
                                              const int64_t* __restrict__ ms, int m, int T_m,
                                              int W, int64_t N, int64_t a) {
  if (shard_pm_kept(m, T_m, W)) return PM[(int64_t)m * N + a];
  // the month's day rows are loaded together (one latency per month, not one per day)
  constexpr int KD = 24;
  const int64_t d0 = ms[m], d1 = ms[m + 1];
  double last = 0.0;
  bool p = false, v = false;
  double xs[KD];
#pragma unroll
  for (int k = 0; k < KD; ++k) xs[k] = (d0 + k < d1) ? P[(d0 + k) * N + a] : absent_val();
#pragma unroll
  for (int k = 0; k < KD; ++k) {
    const double x = xs[k];
    const bool ok = x == x;
    p |= !is_absent(x);
    v |= ok;
    last = ok ? x : last;
  }
  for (int64_t d = d0 + KD; d < d1; ++d) {
    const double x = P[d * N + a];
    const bool ok = x == x;
    p |= !is_absent(x);
    v |= ok;
    last = ok ? x : last;
  }
  return p ? (v ? last : qnan()) : absent_val();
}

// WALK_CHUNK month prices of asset a, months m0, m0 + dm, m0 + 2 dm, ... within [lo, hi]
// (ABSENT outside): the kept months' PM loads are issued together first, the rare months PM
// does not keep are re-derived after them -- one memory round trip per chunk, not per month.
__device__ __forceinline__ void shard_pm_chunk(const double* __restrict__ PM,
                                               const double* __restrict__ P,
                                               const int64_t* __restrict__ ms, int m0, int dm,
                                               int lo, int hi, int T_m, int W, int64_t N,
                                               int64_t a, double (&buf)[WALK_CHUNK]) {
#pragma unroll
  for (int q = 0; q < WALK_CHUNK; ++q) {
    const int m = m0 + q * dm;
    const bool in = m >= lo && m <= hi;
    buf[q] = (in && shard_pm_kept(m, T_m, W)) ? PM[(int64_t)m * N + a] : absent_val();
  }
#pragma unroll
  for (int q = 0; q < WALK_CHUNK; ++q) {
    const int m = m0 + q * dm;
    if (m >= lo && m <= hi && !shard_pm_kept(m, T_m, W)) buf[q] = shard_pm_at(PM, P, ms, m, T_m, W, N, a);
  }
}

// Same record as k_shard_summary (n, fv, lvi, lv, head, first; tail of the last T present
// month prices, ABSENT-padded at the front) from the SH state's n / first / last month.
// idx (the halo pass's fallback columns): output column j < ncol is asset idx[j] (record rows
// ncol apart); columns past the list's length *cnt get the record of an asset with no present
// month (a neutral column for k_fold_carry).
// The record body over a month source: chunk(m0, dm, lo, hi, buf) fills WALK_CHUNK month
// prices (ABSENT outside [lo, hi]) and one(m) gives one month's price.
template <class Chunk, class One>
__device__ __forceinline__ void shard_summary_body(Chunk chunk, One one, int64_t n, int fm, int lm,
                                                   int T, int64_t os, double* __restrict__ out) {
  int64_t fv = -1, lvi = -1;
  double lv = qnan(), head = qnan(), first = absent_val();
  const int k = (int)(n < T ? n : T);
  for (int q = 0; q < T - k; ++q) out[(int64_t)(SUM_SCALARS + q) * os] = absent_val();
  if (n > 0) {
    // forward from the first present month: first price, index of the first valid row
    first = one(fm);
    int64_t ix = 0;
    bool found = false;
    for (int m0 = fm; m0 <= lm && !found; m0 += WALK_CHUNK) {
      double buf[WALK_CHUNK];
      chunk(m0, 1, fm, lm, buf);
#pragma unroll
      for (int q = 0; q < WALK_CHUNK; ++q) {
        const double x = buf[q];
        if (found || is_absent(x)) continue;
        if (!isnan_d(x)) { fv = ix; found = true; }
        ++ix;
      }
    }
    // backward from the last present month: tail, last valid (lv, lvi), head
    int got = 0;
    int64_t seen = 0;          // present rows passed, newest first
    bool have_lv = false, done = false;
    for (int m0 = lm; m0 >= fm && !done; m0 -= WALK_CHUNK) {
      double buf[WALK_CHUNK];
      chunk(m0, -1, fm, lm, buf);
#pragma unroll
      for (int q = 0; q < WALK_CHUNK; ++q) {
        const double x = buf[q];
        if (done || is_absent(x)) continue;
        const bool valid = !isnan_d(x);
        if (valid && !have_lv) { lv = x; lvi = n - 1 - seen; have_lv = true; }
        if (got < k) {
          out[(int64_t)(SUM_SCALARS + T - 1 - got) * os] = x;
          ++got;
        } else if (valid) {
          head = x;
          done = true;
        }
        ++seen;
      }
    }
  }
  out[0 * os] = (double)n;
  out[1 * os] = (double)fv;
  out[2 * os] = (double)lvi;
  out[3 * os] = lv;
  out[4 * os] = head;
  out[5 * os] = first;
}

// Same record as k_shard_summary (n, fv, lvi, lv, head, first; tail of the last T present
// month prices, ABSENT-padded at the front) from the SH state's n / first / last month.
// idx (the halo pass's fallback columns): output column j < ncol is asset idx[j] (record rows
// ncol apart); columns past the list's length *cnt get the record of an asset with no present
// month (a neutral column for k_fold_carry).
__global__ __launch_bounds__(256) void k_shard_summary_state(const double* __restrict__ PM,
                                                             const double* __restrict__ P,
                                                             const int64_t* __restrict__ ms,
                                                             int T_m, int64_t N, int T,
                                                             const double* __restrict__ st,
                                                             double* __restrict__ out,
                                                             const int32_t* __restrict__ idx,
                                                             const int32_t* __restrict__ cnt,
                                                             int64_t ncol) {
  const int W = T - 1;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= (idx ? ncol : N)) return;
  const int64_t os = idx ? ncol : N;   // output row stride
  const bool listed = !idx || j < (int64_t)*cnt;
  const int64_t a = idx ? (listed ? (int64_t)idx[j] : 0) : j;
  const int64_t n = listed ? (int64_t)st[a] : 0;
  const int fm = listed ? (int)st[3 * N + a] : -1, lm = listed ? (int)st[4 * N + a] : -1;
  shard_summary_body(
      [&](int m0, int dm, int lo, int hi, double (&buf)[WALK_CHUNK]) {
        shard_pm_chunk(PM, P, ms, m0, dm, lo, hi, T_m, W, N, a, buf);
      },
      [&](int m) { return shard_pm_at(PM, P, ms, m, T_m, W, N, a); }, n, fm, lm, T, os, out + j);
}

// The listed columns of the halo pass, ONE WORKGROUP PER COLUMN (COLS_THREADS): its threads
// derive the column's T_m month prices together (PM where kept, else the month-end of the
// daily rows: one round trip for all months instead of one per re-derived month), into LDS; one
// lane then builds the record from LDS exactly as k_shard_summary_state does.  The grid is
// min(ncol, 2 n_CU) workgroups striding over the ncol columns (the listed count is on the
// device): a listed column as above, a column past the list gets the neutral record (no present
// month: k_shard_summary_state's, written by the workgroup's first T + SUM_SCALARS lanes).
#define COLS_THREADS 64
__global__ __launch_bounds__(COLS_THREADS) void k_shard_summary_cols(
    const double* __restrict__ PM, const double* __restrict__ P, const int64_t* __restrict__ ms,
    int T_m, int64_t N, int T, const double* __restrict__ st, double* __restrict__ out,
    const int32_t* __restrict__ idx, const int32_t* __restrict__ cnt, int64_t ncol) {
  extern __shared__ __attribute__((aligned(16))) double pmc[];   // [T_m]
  const int W = T - 1;
  const int64_t nl = *cnt;
  for (int64_t j = blockIdx.x; j < ncol; j += gridDim.x) {   // (workgroup-uniform)
    if (j >= nl) {   // the neutral record: shard_summary_body with n = 0
      const int r = threadIdx.x;
      if (r < SUM_SCALARS + T) {
        double v = absent_val();   // the tail rows and `first`
        if (r == 0) v = 0.0;
        else if (r == 1 || r == 2) v = -1.0;
        else if (r == 3 || r == 4) v = qnan();
        out[(int64_t)r * ncol + j] = v;
      }
      continue;
    }
    const int64_t a = (int64_t)idx[j];
    __syncthreads();   // (the previous column's lane 0 is done with pmc)
    for (int m = threadIdx.x; m < T_m; m += COLS_THREADS) pmc[m] = shard_pm_at(PM, P, ms, m, T_m, W, N, a);
    __syncthreads();
    if (threadIdx.x != 0) continue;
    const int64_t n = (int64_t)st[a];
    const int fm = (int)st[3 * N + a], lm = (int)st[4 * N + a];
    shard_summary_body(
        [&](int m0, int dm, int lo, int hi, double (&buf)[WALK_CHUNK]) {
#pragma unroll
          for (int q = 0; q < WALK_CHUNK; ++q) {
            const int m = m0 + q * dm;
            buf[q] = (m >= lo && m <= hi) ? pmc[m] : absent_val();
          }
        },
        [&](int m) { return pmc[m]; }, n, fm, lm, T, ncol, out + j);
  }
}

__device__ __forceinline__ bool same_bits(double x, double y) {
  return __double_as_longlong(x) == __double_as_longlong(y);
}

// fcarry: F's initial state (the halo pass's carry, [W+2][N]); NULL = empty (the speculative
// pass).  idx (the halo pass's fallback columns): thread j repairs asset idx[j] for j < *cnt,
// with carry / next_pm column j (rows ncol apart); NULL = every asset, carry / next_pm [.][N].
// The repair body for asset a over a month source chunk(m0, buf) (REPAIR_CHUNK months from m0,
// ABSENT past T_m - 1); rt / rf: T's and F's rings (stride RS).
template <class Chunk>
__device__ __forceinline__ void shard_repair_body(
    Chunk chunk, int T_m, int64_t N, int J, int skip, const double* __restrict__ carry,
    const double* __restrict__ next_pm, const double* __restrict__ st, double* __restrict__ R,
    double* __restrict__ M, double* __restrict__ NR, uint16_t* __restrict__ IDS,
    const double* __restrict__ fcarry, int64_t a, int64_t cs, int64_t cj, double* rt,
    double* rf, int RS) {
  const int W = J + skip;
  ScanLane t, f;
  scan_init(t, rt, RS, W, carry, cs, cj, true);
  scan_init(f, rf, RS, W, fcarry, N, a, true);
  auto same = [&]() -> bool {
    if (!same_bits(t.pff, f.pff) || !same_bits(t.psff, f.psff) || t.prev != f.prev) return false;
    for (int k = 0; k < W; ++k)
      if (!same_bits(rt[k * RS], rf[k * RS])) return false;
    return true;
  };
  const int64_t npres = (int64_t)st[a];
  const int fm = (int)st[3 * N + a];  // months before the first present one change no state
  int64_t seen = 0;
  bool conv = same();
  bool done = conv || npres == 0;
  static_assert(REPAIR_CHUNK == WALK_CHUNK, "the repair walks months in shard_pm_chunk's batches");
  for (int m0 = fm < 0 ? 0 : fm; m0 < T_m && !done; m0 += REPAIR_CHUNK) {
    double buf[REPAIR_CHUNK];
    chunk(m0, buf);
#pragma unroll
    for (int q = 0; q < REPAIR_CHUNK; ++q) {
      const int m = m0 + q;
      if (m >= T_m || done) break;
      const double x = buf[q];
      const double mom = scan_step(t, x, m, rt, RS, W, J, N, a, R, M, NR);
      if (IDS) IDS[(int64_t)m * N + a] = (uint16_t)csm_fid(mom);   // the rewritten cell's bucket id
      scan_shadow(f, x, m, rf, RS, W, J);
      if (!is_absent(x)) ++seen;
      conv = same();
      done = conv || seen >= npres;
    }
  }
  // the pending ranked row at the shard's end: F's (= T's once converged) or T's own
  const int prev = conv ? (int)st[N + a] : t.prev;
  const double psff = conv ? st[2 * N + a] : t.psff;
  if (prev >= 0) {
    double nr = qnan();
    const double x = next_pm[cj];
    if (!is_absent(x)) {
      const double ps_new = isnan_d(x) ? psff : x;
      nr = ps_new / psff - 1.0;
    }
    NR[(int64_t)prev * N + a] = nr;
  }
}

__global__ __launch_bounds__(REPAIR_THREADS) void k_shard_repair(
    const double* __restrict__ PM, const double* __restrict__ P, const int64_t* __restrict__ ms,
    int T_m, int64_t N, int J, int skip,
    const double* __restrict__ carry, const double* __restrict__ next_pm,
    const double* __restrict__ st, double* __restrict__ R, double* __restrict__ M,
    double* __restrict__ NR, uint16_t* __restrict__ IDS, const double* __restrict__ fcarry,
    const int32_t* __restrict__ idx, const int32_t* __restrict__ cnt, int64_t ncol) {
  extern __shared__ __attribute__((aligned(16))) double lds[];  // [2][W][REPAIR_THREADS]
  const int W = J + skip, RS = REPAIR_THREADS;
  const int tid = threadIdx.x;
  const int64_t j = (int64_t)blockIdx.x * REPAIR_THREADS + tid;
  if (idx ? (j >= ncol || j >= (int64_t)*cnt) : j >= N) return;  // no barriers below
  const int64_t a = idx ? (int64_t)idx[j] : j;
  const int64_t cs = idx ? ncol : N, cj = idx ? j : a;   // carry / next_pm stride and column
  shard_repair_body(
      [&](int m0, double (&buf)[REPAIR_CHUNK]) {
        shard_pm_chunk(PM, P, ms, m0, 1, 0, T_m - 1, T_m, W, N, a, buf);
      },
      T_m, N, J, skip, carry, next_pm, st, R, M, NR, IDS, fcarry, a, cs, cj, lds + tid,
      lds + W * RS + tid, RS);
}

// The listed columns of the halo pass, one workgroup per column (k_shard_summary_cols' month
// prices into LDS by all its threads, then one lane repairs from them; rings in LDS too).
__global__ __launch_bounds__(COLS_THREADS) void k_shard_repair_cols(
    const double* __restrict__ PM, const double* __restrict__ P, const int64_t* __restrict__ ms,
    int T_m, int64_t N, int J, int skip,
    const double* __restrict__ carry, const double* __restrict__ next_pm,
    const double* __restrict__ st, double* __restrict__ R, double* __restrict__ M,
    double* __restrict__ NR, uint16_t* __restrict__ IDS, const double* __restrict__ fcarry,
    const int32_t* __restrict__ idx, const int32_t* __restrict__ cnt, int64_t ncol) {
  extern __shared__ __attribute__((aligned(16))) double lds[];  // pm [T_m], rings [2][W]
  const int W = J + skip;
  const int64_t j = blockIdx.x;
  if (j >= (int64_t)*cnt) return;   // (workgroup-uniform: before the barrier)
  const int64_t a = (int64_t)idx[j];
  double* pmc = lds;
  for (int m = threadIdx.x; m < T_m; m += COLS_THREADS) pmc[m] = shard_pm_at(PM, P, ms, m, T_m, W, N, a);
  __syncthreads();
  if (threadIdx.x != 0) return;
  shard_repair_body(
      [&](int m0, double (&buf)[REPAIR_CHUNK]) {
#pragma unroll
        for (int q = 0; q < REPAIR_CHUNK; ++q) buf[q] = m0 + q < T_m ? pmc[m0 + q] : absent_val();
      },
      T_m, N, J, skip, carry, next_pm, st, R, M, NR, IDS, fcarry, a, ncol, j, lds + T_m,
      lds + T_m + W, 1);
}

// The halo pass's listed columns after collective 1b, in ONE launch: a workgroup per listed
// column (a grid-stride loop over the device-side count, so an empty list costs one wave per
// workgroup) folds the column's exchange records (fold_body, k_fold_carry's walk) into the
// true scan state at the shard's first month and the first present price after the shard,
// derives the column's month prices into LDS (shard_pm_at, all lanes), and one lane replays
// every month from that state -- the sequential scan itself, so every output of the column is
// the unsharded pass's (no convergence test against the halo trajectory: nothing the halo
// state wrote is trusted).  Replaces k_fold_carry + k_shard_repair_cols.
template <int WR, int JC>
__global__ __launch_bounds__(COLS_THREADS) void k_shard_fix_cols(
    const double* __restrict__ PM, const double* __restrict__ P, const int64_t* __restrict__ ms,
    int T_m, int64_t N, int J, int skip, const double* __restrict__ recs, int G, int g,
    double* __restrict__ R, double* __restrict__ M, double* __restrict__ NR,
    uint16_t* __restrict__ IDS, const int32_t* __restrict__ idx, const int32_t* __restrict__ cnt,
    int64_t ncol) {
  // LDS: pm [T_m], carry [W + 2], ring [W] (runtime W), the column's records [G][S]
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int W = J + skip, S = SUM_SCALARS + W + 1;
  double* pmc = lds;
  double* cy = lds + T_m;
  double* ring = cy + W + 2;
  double* rec = ring + W;
  const int64_t n = (int64_t)*cnt < ncol ? (int64_t)*cnt : ncol;
  for (int64_t j = blockIdx.x; j < n; j += gridDim.x) {   // (workgroup-uniform)
    const int64_t a = (int64_t)idx[j];
    for (int q = threadIdx.x; q < G * S; q += COLS_THREADS) rec[q] = recs[(int64_t)q * ncol + j];
    for (int m = threadIdx.x; m < T_m; m += COLS_THREADS) pmc[m] = shard_pm_at(PM, P, ms, m, T_m, W, N, a);
    __syncthreads();
    if (threadIdx.x == 0) {
      const double npm = fold_body(rec, G, g, 1, 0, J, skip, (const double*)nullptr,
                                   [&](int k, double v) { cy[k] = v; }, FoldJs{0, {0, 0, 0, 0}},
                                   (double*)nullptr);
      ScanLane t;
      if constexpr (WR > 0) {   // the ring in registers, oldest first (k_signal_tc's scan)
        double fr[WR];
#pragma unroll
        for (int k = 0; k < WR; ++k) fr[k] = cy[k];
        t.pff = cy[WR];
        t.psff = cy[WR + 1];
        t.head = 0;
        t.prev = -1;
        double xn = pmc[0];
        for (int m = 0; m < T_m; ++m) {
          const double x = xn;
          if (m + 1 < T_m) xn = pmc[m + 1];
          const double mom = scan_step_reg<WR, JC>(t, x, m, fr, J, N, a, R, M, NR);
          if (IDS) IDS[(int64_t)m * N + a] = (uint16_t)csm_fid(mom);
        }
      } else {
        scan_init(t, ring, 1, W, cy, 1, 0, true);
        for (int m = 0; m < T_m; ++m) {
          const double mom = scan_step(t, pmc[m], m, ring, 1, W, J, N, a, R, M, NR);
          if (IDS) IDS[(int64_t)m * N + a] = (uint16_t)csm_fid(mom);
        }
      }
      if (t.prev >= 0) {   // the pending ranked row at the shard's end (scan_finish)
        double nr = qnan();
        if (!is_absent(npm)) {
          const double ps_new = isnan_d(npm) ? t.psff : npm;
          nr = ps_new / t.psff - 1.0;
        }
        NR[(int64_t)t.prev * N + a] = nr;
      }
    }
    __syncthreads();   // (the LDS is the next column's)
  }
}

// =====================================================================================
// Halo date shards (the default multi-GPU pass; north_star's "J + skip lookback
// halo").  A rank holds its shard's daily rows plus H calendar months before it and the first
// month after it.  k_shard_halo builds the scan state the halo months leave (from an empty
// state) and the forward month's price; the state is EXACT -- equal to the one the whole
// history leaves -- whenever the halo holds two valid prices W = J + skip present months apart
// (fv, lv below): the ring's W factors then all follow a valid price, and the last valid price
// is a ranked row in both histories.  k_signal<SH> starts from that state and the forward
// price, so a dense asset's outputs are final after one pass and no record is exchanged for
// it.  The other assets (listed inside the halo or the shard, long gaps, a forward month with
// no row) are flagged; only they take the exchange-and-repair path, over a column list.
// =====================================================================================
#define HALO_THREADS 256
#define HALO_U 8
// The halo months' and the forward months' prices, one thread per (asset, month): PMh[j][N],
// j < H halo month j, j = H + f forward month f < F.  A wave whose lanes walk a month back (no
// price on its last day: listings, delistings, absent months) does not hold up the others.
__global__ __launch_bounds__(HALO_THREADS) void k_halo_pm(const double* __restrict__ P,
                                                          const int64_t* __restrict__ ms, int H,
                                                          int T_m, int64_t N,
                                                          double* __restrict__ PMh) {
  const int64_t a = (int64_t)blockIdx.x * HALO_THREADS + threadIdx.x;
  const int j = blockIdx.y;
  if (a >= N) return;
  const int m = j < H ? j : j + T_m;
  PMh[(int64_t)j * N + a] = halo_month_price(P, ms[m], ms[m + 1], N, a);
}

// months [0, H) of ms are the halo, [H, H + T_m) the shard, [H + T_m, H + T_m + F) the forward
// months, their prices in PMh (k_halo_pm).  before: the panel has months before the halo (else
// the halo is the whole history and its state exact); after: the panel has months after the
// forward months (else an asset with no row in them has next_pm ABSENT, exactly).  carry
// [W+2][N] (csm_signal's layout), next_pm [N] (the first forward month with a row), flags [N]:
// bit 0 the carry may differ from the whole history's, bit 1 next_pm may.
__global__ __launch_bounds__(HALO_THREADS) void k_shard_halo(
    const double* __restrict__ PMh, int H, int F, int before, int after, int64_t N, int J,
    int skip, double* __restrict__ carry, double* __restrict__ next_pm,
    uint8_t* __restrict__ flags) {
  extern __shared__ __attribute__((aligned(16))) double hring[];  // [W][HALO_THREADS]
  const int W = J + skip, RS = HALO_THREADS;
  const int64_t a = (int64_t)blockIdx.x * HALO_THREADS + threadIdx.x;
  if (a >= N) return;  // no barriers below
  double* ring = hring + threadIdx.x;
  ScanLane s;
  scan_init(s, ring, RS, W, nullptr, N, a, true);
  int n = 0, fv = -1, lv = -1;
  for (int m0 = 0; m0 < H; m0 += HALO_U) {
    double xs[HALO_U];   // HALO_U month prices in flight
#pragma unroll
    for (int u = 0; u < HALO_U; ++u)
      xs[u] = m0 + u < H ? PMh[(int64_t)(m0 + u) * N + a] : absent_val();
#pragma unroll
    for (int u = 0; u < HALO_U; ++u) {
      const double x = xs[u];
      if (m0 + u >= H || is_absent(x)) continue;
      if (!isnan_d(x)) { if (fv < 0) fv = n; lv = n; }
      ++n;
      scan_shadow(s, x, m0 + u, ring, RS, W, J);
    }
  }
  int ix = s.head;
  for (int k = 0; k < W; ++k) {   // ring factors, oldest first (scan_finish's carry_out)
    carry[(int64_t)k * N + a] = ring[ix * RS];
    ix = (ix + 1 == W) ? 0 : ix + 1;
  }
  carry[(int64_t)W * N + a] = s.pff;
  carry[(int64_t)(W + 1) * N + a] = s.psff;
  uint8_t fl = 0;
  if (before && !(fv >= 0 && lv - fv >= W)) fl |= 1;
  double npm = absent_val();
  for (int f = 0; f < F && is_absent(npm); ++f) npm = PMh[(int64_t)(H + f) * N + a];
  if (after && is_absent(npm)) fl |= 2;
  next_pm[a] = npm;
  flags[a] = fl;
}

// This rank's exchange bits, one per asset, 64 per word (a wave's ballot), rows of nw words:
// 0 an uncertain carry and a present month in the shard; 1 an uncertain forward price and a
// pending ranked row at the shard's end; 2 a present month in the shard; 3 a present month
// before the shard's last Hn months (those in the next rank's halo).  The union below decides
// from every rank's rows which assets really need the exchange.
__global__ __launch_bounds__(256) void k_shard_need(const uint8_t* __restrict__ flags,
                                                    const double* __restrict__ st, int64_t N,
                                                    int T_m, int Hn, int64_t nw,
                                                    uint64_t* __restrict__ mask) {
  const int64_t a = (int64_t)blockIdx.x * 256 + threadIdx.x;
  bool c0 = false, c1 = false, pa = false, ph = false;
  if (a < N) {
    const uint8_t f = flags[a];
    pa = st[a] > 0.0;
    c0 = (f & 1) && pa;
    c1 = (f & 2) && st[N + a] >= 0.0;
    const double fm = st[3 * N + a];
    ph = fm >= 0.0 && fm < (double)(T_m - Hn);
  }
  const uint64_t b0 = __ballot(c0), b1 = __ballot(c1), b2 = __ballot(pa), b3 = __ballot(ph);
  if ((threadIdx.x & 63) == 0 && a < N) {
    const int64_t w = a >> 6;
    mask[w] = b0;
    mask[nw + w] = b1;
    mask[2 * nw + w] = b2;
    mask[3 * nw + w] = b3;
  }
}

// The assets that need the exchange on some rank, from every rank's k_shard_need rows
// [G][4][nw]: rank g needs asset a when its carry is uncertain and the asset has a row before
// g's halo (a row in a shard before g - 1, or in shard g - 1 before its last H months), or its
// forward price is uncertain and a later shard has a row -- otherwise the halo's state / ABSENT
// IS the whole history's.  The union as an ascending list of asset indices (the same on every
// rank): idx[0 .. min(count, cap)), *count = its full length (> cap: the list overflowed and
// the pass must take the all-gather path).  One workgroup.
#define UNION_THREADS 1024
__global__ __launch_bounds__(UNION_THREADS) void k_shard_union(const uint64_t* __restrict__ masks,
                                                               int G, int64_t nw, int64_t cap,
                                                               int32_t* __restrict__ idx,
                                                               int32_t* __restrict__ count) {
  __shared__ int32_t wsum[UNION_THREADS / 64];
  __shared__ int64_t base;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) base = 0;
  __syncthreads();
  auto row = [&](int g, int r, int64_t w) -> uint64_t { return masks[((int64_t)g * 4 + r) * nw + w]; };
  for (int64_t w0 = 0; w0 < nw; w0 += UNION_THREADS) {
    const int64_t w = w0 + tid;
    uint64_t u = 0;
    if (w < nw) {
      uint64_t later[HALO_MAXG];   // a row in a shard after g
      uint64_t suf = 0;
      for (int g = G - 1; g >= 0; --g) { later[g] = suf; suf |= row(g, 2, w); }
      uint64_t A = 0, B = 0, hp = 0;   // rows in shards < g - 1 / in g - 1 / in g - 1's head
      for (int g = 0; g < G; ++g) {
        const uint64_t hist = A | hp;   // a row before g's halo
        u |= (row(g, 0, w) & hist) | (row(g, 1, w) & later[g]);
        A |= B;
        B = row(g, 2, w);
        hp = row(g, 3, w);
      }
    }
    const int c = __popcll(u);
    int inc = c;   // wave inclusive scan, then the waves in order
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(inc, o, 64);
      if (lane >= o) inc += v;
    }
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    int64_t off = base + inc - c;
    for (int q = 0; q < wid; ++q) off += wsum[q];
    while (u) {
      const int b = __builtin_ctzll(u);
      u &= u - 1;
      if (off < cap) idx[off] = (int32_t)(w * 64 + b);
      ++off;
    }
    __syncthreads();
    if (tid == UNION_THREADS - 1) base = off;
    __syncthreads();
  }
  if (tid == 0) *count = (int32_t)(base < 0x7FFFFFFF ? base : 0x7FFFFFFF);
}

// =====================================================================================
// C ABI
// =====================================================================================
// Process-wide knobs (csm_tune).  Every one selects between PRODUCT paths that give identical
// results (the fallbacks odd widths / unaligned buffers / narrow panels take), so tests can
// drive each path on inputs that would not reach it by default.  The measured variants that
// lost their A/B (profiles/r0*/experiments) are not in the library.
static int g_tune_signal_vec = 2;      // k_signal assets per lane: 2 (paired 16-B rows) | 1 (odd N)
static int g_tune_signal_bwf = 0;      // k_signal blocks: 0 auto | 1 one wave | 4 four barrier-free waves x 2 month buffers (buffer loads)
static int g_tune_signal_j12 = 1;      // wide shard k_signal: J = 12 with its product length fixed at compile time (0: runtime J)
static int g_tune_cols_wg = 1;          // halo pass's listed columns: one workgroup per column (month prices into LDS) | 0 one thread per column
#define SIGNAL_BWF_MIN_N (180 * 512)   // auto: 4-wave blocks once the grid still covers >= 180 CUs
static int64_t* g_dec_timing = nullptr;
// PRE decile pass (csm_deciles_ids): 1 the merged sweep, then the general kernel for the rows it
// leaves | 0 the general kernel only
static int g_tune_dec_merge = 1;
// wide rows on ids: 2 (auto) the split decile pass (plan, chunked sweep, finish; deciles.inc) for
// launches of fewer rows than half the CUs (short date shards), else the merged
// one-workgroup-per-row pass | 1 always split | 0 never.  Same labels and counts; decile means in
// another fixed order
static int g_tune_dec_split = 2;
static int64_t g_tune_dec_split_cells = SPLIT_CELLS;   // cells per split-sweep chunk
// the split sweep: 0 the two-workgroups-per-CU variant (no prefetch) | 1 the prefetching one
// workgroup per CU | 2 prefetch when the launch has no more (chunk, date) pairs than CUs.
// C4 rank rehearsals, deciles_ids ms: 4-way 0.1162 / 0.1338 / 0.1165, 8-way 0.0998 / 0.1019 /
// 0.1014 (profiles/r06/experiments/split_pf)
static int g_tune_dec_split_pf = 0;
// csm_momentum_multi: 2 register shift ring, two assets per lane (even N, aligned) | 1 one asset
// per lane | 0 the shared-memory ring (max(J) + skip > 16 always takes it)
static int g_tune_mj_reg = 2;
// rows with at most this many assets take the narrow-row decile kernels
static int64_t g_tune_dec_narrow_max = 16384;
// k_signal_tc: polling trips a waiting workgroup makes before it gives up and marks the launch
// (0: give up at once -- only the tests of the failure report set it)
static unsigned g_tune_tc_spins = TC_SPINS;

extern "C" {

int csm_abi_version(void) { return CSM_ABI_VERSION; }

int csm_tune_portfolio(const char* key, int value);  // portfolio.hip
int csm_tune_ptr_portfolio(const char* key, void* p);  // portfolio.hip

int csm_tune(const char* key, int value) {
  if (!key) return CSM_E_INVAL;
  if (!strcmp(key, "cohort_lds") || !strcmp(key, "cohort_seg") || !strcmp(key, "turn_want") ||
      !strcmp(key, "overlap_rows") || !strcmp(key, "turn_gen_grid") || !strcmp(key, "gen_reset") ||
      !strcmp(key, "turn_vwg") || !strcmp(key, "turn_mask") || !strcmp(key, "ls_opt"))
    return csm_tune_portfolio(key, value);
  if (!strcmp(key, "signal_vec") && (value == 1 || value == 2)) { g_tune_signal_vec = value; return CSM_OK; }
  if (!strcmp(key, "signal_bwf") && (value == 0 || value == 1 || value == 4)) { g_tune_signal_bwf = value; return CSM_OK; }
  if (!strcmp(key, "signal_j12") && (value == 0 || value == 1)) { g_tune_signal_j12 = value; return CSM_OK; }
  if (!strcmp(key, "cols_wg") && (value == 0 || value == 1)) { g_tune_cols_wg = value; return CSM_OK; }
  if (!strcmp(key, "dec_merge") && (value == 0 || value == 1)) { g_tune_dec_merge = value; return CSM_OK; }
  if (!strcmp(key, "mj_reg") && value >= 0 && value <= 2) { g_tune_mj_reg = value; return CSM_OK; }
  if (!strcmp(key, "dec_narrow_max") && value >= 0) { g_tune_dec_narrow_max = value; return CSM_OK; }
  if (!strcmp(key, "dec_split") && value >= 0 && value <= 2) { g_tune_dec_split = value; return CSM_OK; }
  if (!strcmp(key, "dec_split_pf") && value >= 0 && value <= 2) { g_tune_dec_split_pf = value; return CSM_OK; }
  if (!strcmp(key, "tc_spins") && value >= 0) { g_tune_tc_spins = (unsigned)value; return CSM_OK; }
  if (!strcmp(key, "dec_split_cells") && value >= SPLIT_TRIP && value % SPLIT_TRIP == 0) {
    g_tune_dec_split_cells = value;
    return CSM_OK;
  }
  return CSM_E_INVAL;
}

int csm_tune_ptr(const char* key, void* p) {
  if (!key) return CSM_E_INVAL;
  if (!strcmp(key, "dec_timing")) { g_dec_timing = (int64_t*)p; return CSM_OK; }
  return csm_tune_ptr_portfolio(key, p);
}

int csm_create(int device, csm_ctx** out) {
  if (!out) return CSM_E_INVAL;
  *out = nullptr;
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || device < 0 || device >= nd) return CSM_E_HIP;
  if (hipSetDevice(device) != hipSuccess) return CSM_E_HIP;
  csm_ctx* c = (csm_ctx*)calloc(1, sizeof(csm_ctx));
  if (!c) return CSM_E_INVAL;
  c->device = device;
  c->stream = nullptr;
  if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    c->n_cu = 256;
  c->dec_flg_n = 1 << 16;
  if (hipMalloc(&c->dec_flg, (size_t)c->dec_flg_n * sizeof(int32_t)) != hipSuccess) {
    free(c);
    return CSM_E_HIP;
  }
  // the fused long-short's arrival counter: allocated and zeroed here, so a captured pipeline
  // never allocates; each decile launch's last workgroup leaves it zero again
  if (hipMalloc(&c->ticket, 256) != hipSuccess) {
    (void)hipFree(c->dec_flg);
    free(c);
    return CSM_E_HIP;
  }
  if (hipMemset(c->ticket, 0, 256) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    (void)hipFree(c->ticket);
    (void)hipFree(c->dec_flg);
    free(c);
    return CSM_E_HIP;
  }
  *out = c;
  return CSM_OK;
}

int csm_destroy(csm_ctx* ctx) {
  if (ctx) (void)csm_allgather_free(ctx);
  if (ctx && (ctx->scratch || ctx->dec_flg || ctx->ticket || ctx->dsplit)) {
    (void)hipSetDevice(ctx->device);
    if (ctx->scratch) (void)hipFree(ctx->scratch);
    if (ctx->dec_flg) (void)hipFree(ctx->dec_flg);
    if (ctx->ticket) (void)hipFree(ctx->ticket);
    if (ctx->dsplit) (void)hipFree(ctx->dsplit);
  }
  free(ctx);
  return CSM_OK;
}

const char* csm_last_error(const csm_ctx* ctx) { return ctx ? ctx->err : "null context"; }

int csm_set_stream(csm_ctx* ctx, void* stream) {
  if (!ctx) return CSM_E_INVAL;
  ctx->stream = (hipStream_t)stream;
  return CSM_OK;
}

int csm_sync(csm_ctx* ctx) {
  int r = prep(ctx);
  if (r) return r;
  HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
  return CSM_OK;
}

int csm_month_end(csm_ctx* ctx, const double* P, const double* V, int64_t T_d, int64_t N,
                  const int64_t* month_start, int32_t T_m, double* PM, double* VOL) {
  int r = prep(ctx);
  if (r) return r;
  if (!P || !month_start || !PM || N <= 0 || T_d < 0 || T_m < 0 || T_m > 65535)
    return set_err(ctx, CSM_E_INVAL, "csm_month_end: bad arguments (N=%lld T_d=%lld T_m=%d)",
                   (long long)N, (long long)T_d, T_m);
  if ((V == nullptr) != (VOL == nullptr))
    return set_err(ctx, CSM_E_INVAL, "csm_month_end: V and VOL must both be given or both NULL");
  if (T_m == 0) return CSM_OK;
  const bool v2 = (N % 2 == 0) && aligned16(P) && aligned16(PM) && (!V || aligned16(V));
  const int vec = v2 ? 2 : 1;
  dim3 grid((unsigned)((N + 256LL * vec - 1) / (256LL * vec)), (unsigned)T_m);
  if (v2) {
    if (V) hipLaunchKernelGGL((k_month_end<2, true>), grid, dim3(256), 0, ctx->stream, P, V, month_start, N, PM, VOL);
    else hipLaunchKernelGGL((k_month_end<2, false>), grid, dim3(256), 0, ctx->stream, P, V, month_start, N, PM, VOL);
  } else {
    if (V) hipLaunchKernelGGL((k_month_end<1, true>), grid, dim3(256), 0, ctx->stream, P, V, month_start, N, PM, VOL);
    else hipLaunchKernelGGL((k_month_end<1, false>), grid, dim3(256), 0, ctx->stream, P, V, month_start, N, PM, VOL);
  }
  LAUNCH_CHECK(ctx, "k_month_end");
  return CSM_OK;
}

int csm_momentum(csm_ctx* ctx, const double* PM, int32_t T_m, int64_t N, int32_t J, int32_t skip,
                 double* R, double* M, double* NR, const double* carry, const double* next_pm,
                 double* carry_out) {
  int r = prep(ctx);
  if (r) return r;
  if (!PM || !M || !NR || N <= 0 || T_m < 0 || J < 1 || skip < 0 || J + skip > 256)
    return set_err(ctx, CSM_E_INVAL, "csm_momentum: bad arguments (N=%lld T_m=%d J=%d skip=%d)",
                   (long long)N, T_m, J, skip);
  const int W = J + skip;
  const int tpb = W <= 64 ? SCAN_THREADS : 64;  // ring = W * tpb doubles of LDS (<= 128 KiB)
  const size_t lds = (size_t)W * tpb * sizeof(double);
  const unsigned blocks = (unsigned)((N + tpb - 1) / tpb);
  if (lds > 65536)
    HIP_CHECK(ctx, hipFuncSetAttribute((const void*)k_momentum,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(k_momentum, dim3(blocks), dim3(tpb), lds, ctx->stream, PM, T_m, N, J,
                     skip, R, M, NR, carry, next_pm, carry_out);
  LAUNCH_CHECK(ctx, "k_momentum");
  return CSM_OK;
}

static bool mj_fixed_grid(const int32_t* Js, int nJ, int skip) {
  return nJ == 4 && skip == 1 && Js[0] == 3 && Js[1] == 6 && Js[2] == 9 && Js[3] == 12;
}

static int momentum_multi(csm_ctx* ctx, const double* PM, int32_t T_m, int64_t N,
                          const int32_t* Js, int32_t nJ, int32_t skip, double* const* M,
                          double* const* NR, uint16_t* const* IDS) {
  int r = prep(ctx);
  if (r) return r;
  if (!PM || !Js || !M || !NR || N <= 0 || T_m < 0 || nJ < 1 || nJ > MJ_MAX || skip < 0)
    return set_err(ctx, CSM_E_INVAL, "csm_momentum_multi: bad arguments (N=%lld T_m=%d nJ=%d "
                   "skip=%d; 1 <= nJ <= %d)", (long long)N, T_m, nJ, skip, MJ_MAX);
  MJSet mj;
  int Jmax = 0;
  for (int q = 0; q < MJ_MAX; ++q) {
    mj.J[q] = q < nJ ? Js[q] : 1;
    mj.M[q] = q < nJ ? M[q] : nullptr;
    mj.NR[q] = q < nJ ? NR[q] : nullptr;
    mj.IDS[q] = (q < nJ && IDS) ? IDS[q] : nullptr;
    if (q < nJ && IDS && !IDS[q])
      return set_err(ctx, CSM_E_INVAL, "csm_momentum_multi_ids: ids[%d] is NULL", q);
    if (q < nJ && (Js[q] < 1 || !M[q] || !NR[q]))
      return set_err(ctx, CSM_E_INVAL, "csm_momentum_multi: J[%d]=%d or its outputs invalid", q,
                     q < nJ ? Js[q] : 0);
    if (q < nJ && Js[q] > Jmax) Jmax = Js[q];
  }
  const int W = Jmax + skip;
  if (W > 64)
    return set_err(ctx, CSM_E_INVAL, "csm_momentum_multi: max(J) + skip = %d > 64", W);
  if (T_m == 0) return CSM_OK;
  const int tpb = SCAN_THREADS;
  const unsigned blocks = (unsigned)((N + tpb - 1) / tpb);
  bool al = (N % 2) == 0 && aligned16(PM);
  for (int q = 0; q < nJ; ++q)
    al = al && aligned16(M[q]) && aligned16(NR[q]) && (!IDS || ((uintptr_t)IDS[q] & 3u) == 0);
  if (W <= MJ_REG_W && g_tune_mj_reg == 2 && al) {   // register shift ring, two assets per lane
    if (mj_fixed_grid(Js, nJ, skip))
      hipLaunchKernelGGL((k_momentum_multi_reg2<13, false, true>), dim3((unsigned)((N / 2 + tpb - 1) / tpb)),
                         dim3(tpb), 0, ctx->stream, PM, T_m, N, nJ, skip, mj, 1,
                         (const double*)nullptr, (const double*)nullptr, (const double*)nullptr);
    else
      hipLaunchKernelGGL(k_momentum_multi_reg2<MJ_REG_W>, dim3((unsigned)((N / 2 + tpb - 1) / tpb)),
                         dim3(tpb), 0, ctx->stream, PM, T_m, N, nJ, skip, mj, 1,
                         (const double*)nullptr, (const double*)nullptr, (const double*)nullptr);
    LAUNCH_CHECK(ctx, "k_momentum_multi_reg2");
    return CSM_OK;
  }
  if (W <= MJ_REG_W && g_tune_mj_reg) {   // register shift ring
    hipLaunchKernelGGL(k_momentum_multi_reg<MJ_REG_W>, dim3(blocks), dim3(tpb), 0, ctx->stream,
                       PM, T_m, N, nJ, skip, mj);
    LAUNCH_CHECK(ctx, "k_momentum_multi_reg");
    return CSM_OK;
  }
  const size_t lds = (size_t)W * tpb * sizeof(double);   // <= 64 KiB
  hipLaunchKernelGGL(k_momentum_multi, dim3(blocks), dim3(tpb), lds, ctx->stream, PM, T_m, N,
                     nJ, skip, W, mj);
  LAUNCH_CHECK(ctx, "k_momentum_multi");
  return CSM_OK;
}

int csm_momentum_multi(csm_ctx* ctx, const double* PM, int32_t T_m, int64_t N,
                       const int32_t* Js, int32_t nJ, int32_t skip, double* const* M,
                       double* const* NR) {
  return momentum_multi(ctx, PM, T_m, N, Js, nJ, skip, M, NR, nullptr);
}

int csm_momentum_multi_ids(csm_ctx* ctx, const double* PM, int32_t T_m, int64_t N,
                           const int32_t* Js, int32_t nJ, int32_t skip, double* const* M,
                           double* const* NR, uint16_t* const* IDS) {
  if (!IDS) return set_err(ctx, CSM_E_INVAL, "csm_momentum_multi_ids: ids is NULL");
  return momentum_multi(ctx, PM, T_m, N, Js, nJ, skip, M, NR, IDS);
}

static int signal_launch(csm_ctx* ctx, const char* who, const double* P, int64_t T_d,
                         int64_t N, const int64_t* month_start, int32_t T_m,
                         int32_t max_month_days, int32_t J, int32_t skip, double* PM, double* R,
                         double* M, double* NR, const double* carry, const double* next_pm,
                         double* carry_out, bool sh = false, uint16_t* ids = nullptr,
                         const HaloArgs* halo = nullptr) {
  int r = prep(ctx);
  if (r) return r;
  // (a shard pass starts from an empty state, or -- the halo pass -- from the halo's carry
  // and forward price)
  if (sh && (!PM || !carry_out || T_m < 1))
    return set_err(ctx, CSM_E_INVAL, "%s: a shard pass needs PM and state, and at least one month",
                   who);
  if (!P || !month_start || !M || !NR || N <= 0 || T_d < 0 || T_m < 0 || J < 1 || skip < 0 ||
      J + skip > 256 || max_month_days < 1)
    return set_err(ctx, CSM_E_INVAL, "%s: bad arguments (N=%lld T_m=%d J=%d skip=%d)", who,
                   (long long)N, T_m, J, skip);
  if (max_month_days > 32)
    return set_err(ctx, CSM_E_INVAL, "%s: months longer than 32 days are not supported "
                   "(use csm_month_end + csm_momentum)", who);
  if (T_m == 0) return CSM_OK;
  const int W = J + skip;
  const bool can2 = (N % 2 == 0) && aligned16(P) && (!PM || aligned16(PM)) && aligned16(M) &&
                    aligned16(NR) && (!R || aligned16(R));
  const int vec = (g_tune_signal_vec == 1 || !can2) ? 1 : 2;
  // Barrier-free 4-wave blocks (adjacent 1-KiB column slices walked independently, 2 month
  // buffers, raw buffer loads with the padding rows out of range): the wide-panel default
  // (C4 1.75-1.85 -> 1.63-1.78 ms, then buffer loads 1.695 -> 1.674, profiles/r02/experiments).
  // Rows of at most 2 GiB / 32 (buffer offsets), months of at most 23 days.
  const bool fits4 = vec == 2 && max_month_days <= 23 && N * 8 * 32 < ((int64_t)1 << 31);
  const bool wide4 = fits4 && (g_tune_signal_bwf == 4 ||
                               (g_tune_signal_bwf == 0 && N >= (int64_t)SIGNAL_BWF_MIN_N));
  const int bw = wide4 ? 4 : 1;
  const size_t lds = (size_t)W * 64 * vec * bw * sizeof(double) +
                     (sh ? (size_t)3 * 64 * vec * bw * sizeof(int) : 0) +
                     (halo ? (size_t)HALO_BATCH * 64 * vec * bw * sizeof(double) +
                             (size_t)bw * HALO_BATCH * 128 * sizeof(uint16_t) : 0);
  const unsigned blocks = (unsigned)((N / vec + 64 * bw - 1) / (64 * bw));
  const void* fn = nullptr;
  // one-wave blocks, four month buffers: 23 / 24 / 32 day rows (the longest month)
#define SIG1(V, SH_)                                                                            \
  (max_month_days <= 23 && V == 2 ? (const void*)k_signal<23, V, 4, 1, SH_, false>              \
   : max_month_days <= 24         ? (const void*)k_signal<24, V, 4, 1, SH_, false>              \
                                  : (const void*)k_signal<32, V, 4, 1, SH_, false>)
  // date shards: the default look-back J = 12 with its product length fixed at compile time
  // (8-way halo rank: shard kernel 0.237 -> 0.231 ms; the full C4 pass measured 0.3 % slower
  // with it, so the one-GPU kernel keeps the runtime J)
  const bool j12 = sh && J == 12 && g_tune_signal_j12;
  if (halo && !(sh && wide4))
    return set_err(ctx, CSM_E_INVAL, "%s: the fused halo prologue runs in the wide shard kernel "
                   "(even N >= %d, months of <= 23 days); use csm_shard_halo + "
                   "csm_signal_shard_halo", who, SIGNAL_BWF_MIN_N);
  if (halo)
    fn = j12 ? (const void*)k_signal<23, 2, 2, 4, true, true, 12, true>
             : (const void*)k_signal<23, 2, 2, 4, true, true, 0, true>;
  else if (wide4 && j12)
    fn = (const void*)k_signal<23, 2, 2, 4, true, true, 12>;
  else if (wide4)
    fn = sh ? (const void*)k_signal<23, 2, 2, 4, true, true> : (const void*)k_signal<23, 2, 2, 4, false, true>;
  else if (vec == 2)
    fn = sh ? SIG1(2, true) : SIG1(2, false);
  else
    fn = sh ? SIG1(1, true) : SIG1(1, false);
#undef SIG1
  if (lds > 65536)
    HIP_CHECK(ctx, hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  {
    int T_m_ = T_m, J_ = J, skip_ = skip;
    int64_t N_ = N, T_d_ = T_d;
    HaloArgs ha = halo ? *halo : HaloArgs{0, 0, 0, 0, nullptr};
    void* args[] = {(void*)&P, (void*)&month_start, &T_m_, &N_, &J_, &skip_, (void*)&PM, (void*)&R,
                    (void*)&M, (void*)&NR, (void*)&carry, (void*)&next_pm, (void*)&carry_out, &T_d_,
                    (void*)&ids, (void*)&ha};
    HIP_CHECK(ctx, hipLaunchKernel(fn, dim3(blocks), dim3(64 * bw), args, lds, ctx->stream));
  }
  LAUNCH_CHECK(ctx, who);
  return CSM_OK;
}

int csm_signal(csm_ctx* ctx, const double* P, int64_t T_d, int64_t N, const int64_t* month_start,
               int32_t T_m, int32_t max_month_days, int32_t J, int32_t skip, double* PM, double* R,
               double* M, double* NR, const double* carry, const double* next_pm,
               double* carry_out) {
  return signal_launch(ctx, "csm_signal", P, T_d, N, month_start, T_m, max_month_days, J,
                       skip, PM, R, M, NR, carry, next_pm, carry_out);
}

int csm_signal_ids(csm_ctx* ctx, const double* P, int64_t T_d, int64_t N,
                   const int64_t* month_start, int32_t T_m, int32_t max_month_days,
                   int32_t min_month_days, int32_t J, int32_t skip, double* PM, double* R,
                   double* M, double* NR, uint16_t* ids) {
  if (!ids || (N % 4) != 0 || ((uintptr_t)ids & 7u) != 0)
    return set_err(ctx, CSM_E_INVAL, "csm_signal_ids: ids must be non-NULL and 8-B aligned, N %% 4 == 0 "
                   "(N=%lld)", (long long)N);
  (void)min_month_days;   // kept in the ABI (host hint for fixed day batches; no kernel uses it)
#ifdef SIG_HIST
  {   // A/B build only: a zeroed [T_m][8192] histogram per launch
    static uint32_t* hist = nullptr;
    static int64_t cap = 0;
    const int64_t need = (int64_t)T_m * 8192;
    if (need > cap) {
      if (hist) hipFree(hist);
      HIP_CHECK(ctx, hipMalloc(&hist, need * 4));
      cap = need;
      HIP_CHECK(ctx, hipMemcpyToSymbol(HIP_SYMBOL(g_sig_hist), &hist, sizeof(hist)));
    }
    HIP_CHECK(ctx, hipMemsetAsync(hist, 0, need * 4, ctx->stream));
  }
#endif
  return signal_launch(ctx, "csm_signal_ids", P, T_d, N, month_start, T_m, max_month_days, J,
                       skip, PM, R, M, NR, nullptr, nullptr, nullptr, false, ids);
}

int csm_signal_shard(csm_ctx* ctx, const double* P, int64_t T_d, int64_t N,
                     const int64_t* month_start, int32_t T_m, int32_t max_month_days, int32_t J,
                     int32_t skip, double* PM, double* R, double* M, double* NR, double* state) {
  return signal_launch(ctx, "csm_signal_shard", P, T_d, N, month_start, T_m,
                       max_month_days, J, skip, PM, R, M, NR, nullptr, nullptr, state, true);
}

int csm_signal_shard_ids(csm_ctx* ctx, const double* P, int64_t T_d, int64_t N,
                         const int64_t* month_start, int32_t T_m, int32_t max_month_days,
                         int32_t J, int32_t skip, double* PM, double* R, double* M, double* NR,
                         double* state, uint16_t* ids) {
  if (!ids || (N % 4) != 0 || ((uintptr_t)ids & 7u) != 0)
    return set_err(ctx, CSM_E_INVAL, "csm_signal_shard_ids: needs ids, N %% 4 == 0, 8-B aligned ids");
  return signal_launch(ctx, "csm_signal_shard_ids", P, T_d, N, month_start, T_m,
                       max_month_days, J, skip, PM, R, M, NR, nullptr, nullptr, state, true, ids);
}

}  // extern "C"

template <int NB>
static void launch_deciles(bool v2, int T_m, hipStream_t st, const double* M, const double* NR,
                           int64_t N, int nbins, const QTab& q, int8_t* L, double* EW,
                           int32_t* CNT, int32_t* NV, uint16_t* ids, bool pre = false,
                           int32_t* flg = nullptr, double* LS = nullptr,
                           int32_t* ticket = nullptr) {
  int64_t* tm = g_dec_timing;
  if (pre) {   // ids written by csm_signal_ids / csm_momentum_multi_ids (fixed map): M is read only for a few cells
    if (N <= g_tune_dec_narrow_max)   // sweep rows: 2048 buckets (the fixed map's ids >> 2)
      launch_deciles_pre_narrow<NB>(T_m, st, M, NR, N, nbins, q, L, EW, CNT, NV, tm, ids,
                                    g_tune_dec_merge ? flg : nullptr, LS, ticket);
    else
      launch_deciles_pre<NB>(T_m, st, M, NR, N, nbins, q, L, EW, CNT, NV, tm, ids,
                             g_tune_dec_merge ? flg : nullptr, LS, ticket, g_tune_dec_split_cells);
    return;
  }
  if (N <= g_tune_dec_narrow_max) {   // rows of a few thousand assets (C2/C3/C5)
    launch_deciles_narrow<NB>(v2, T_m, st, M, NR, N, nbins, q, L, EW, CNT, NV, tm);
    return;
  }
  if (v2) hipLaunchKernelGGL((k_deciles<NB, true>), dim3(T_m), dim3(dec_wide::kThreads), 0, st, M, NR, N, nbins, q, L, EW, CNT, NV, tm, ids);
  else hipLaunchKernelGGL((k_deciles<NB, false>), dim3(T_m), dim3(dec_wide::kThreads), 0, st, M, NR, N, nbins, q, L, EW, CNT, NV, tm, ids);
}

extern "C" {

int csm_deciles(csm_ctx* ctx, const double* M, const double* NR, int32_t T_m, int64_t N,
                int32_t n_bins, const double* qtable, int8_t* L, double* EW, int32_t* CNT,
                int32_t* NV) {
  int r = prep(ctx);
  if (r) return r;
  if (!M || !L || !qtable || N <= 0 || T_m < 0 || n_bins < 1 || n_bins > MAXQ - 1 || N > 0x7FFFFFFFLL)
    return set_err(ctx, CSM_E_INVAL, "csm_deciles: bad arguments (N=%lld T_m=%d n_bins=%d)",
                   (long long)N, T_m, n_bins);
  if (NR && (!EW || !CNT))
    return set_err(ctx, CSM_E_INVAL, "csm_deciles: EW and CNT are required when NR is given");
  if (T_m == 0) return CSM_OK;
  QTab q;
  for (int i = 0; i < MAXQ; ++i) q.q[i] = i <= n_bins ? qtable[i] : 1.0;
  const bool v2 = (N % 2 == 0) && aligned16(M) && (!NR || aligned16(NR)) && (((uintptr_t)L & 1u) == 0);
  uint16_t* ids = nullptr;
  if (!NR) {
    launch_deciles<0>(v2, T_m, ctx->stream, M, nullptr, N, n_bins, q, L, nullptr, nullptr, NV, ids);
  } else {
    switch (n_bins) {
      case 2: launch_deciles<2>(v2, T_m, ctx->stream, M, NR, N, n_bins, q, L, EW, CNT, NV, ids); break;
      case 3: launch_deciles<3>(v2, T_m, ctx->stream, M, NR, N, n_bins, q, L, EW, CNT, NV, ids); break;
      case 4: launch_deciles<4>(v2, T_m, ctx->stream, M, NR, N, n_bins, q, L, EW, CNT, NV, ids); break;
      case 5: launch_deciles<5>(v2, T_m, ctx->stream, M, NR, N, n_bins, q, L, EW, CNT, NV, ids); break;
      case 10: launch_deciles<10>(v2, T_m, ctx->stream, M, NR, N, n_bins, q, L, EW, CNT, NV, ids); break;
      case 20: launch_deciles<20>(v2, T_m, ctx->stream, M, NR, N, n_bins, q, L, EW, CNT, NV, ids); break;
      default:
        return set_err(ctx, CSM_E_INVAL, "csm_deciles: n_bins=%d unsupported with NR (use 2,3,4,5,10,20)", n_bins);
    }
  }
  LAUNCH_CHECK(ctx, "k_deciles");
  return CSM_OK;
}

int csm_long_short(csm_ctx* ctx, const double* EW, const int32_t* CNT, int32_t T_m,
                   int32_t n_bins, double* LS) {
  int r = prep(ctx);
  if (r) return r;
  if (!EW || !CNT || !LS || T_m < 0 || n_bins < 1)
    return set_err(ctx, CSM_E_INVAL, "csm_long_short: bad arguments");
  if (T_m == 0) return CSM_OK;
  hipLaunchKernelGGL(k_long_short, dim3(1), dim3(LS_THREADS), 0, ctx->stream, EW, CNT, T_m, n_bins, LS);
  LAUNCH_CHECK(ctx, "k_long_short");
  return CSM_OK;
}

// The split decile pass's workspace for T_m rows of N cells (csm_common.h DecSplit), carved
// from one context buffer; sized for n_bins up to MAXQ so one buffer serves every NB.
static size_t dsplit_layout(int32_t T_m, int64_t N, DecSplit* sp, char* base) {
  const int64_t CC = g_tune_dec_split_cells;
  const int64_t C = (N + CC - 1) / CC;
  auto al = [](size_t x) { return (x + 255) / 256 * 256; };
  size_t o = 0;
  const size_t plan = o; o = al(o + (size_t)T_m * DSPLAN_BYTES);
  const size_t tab = o;  o = al(o + (size_t)T_m * CSM_FB_BUCKETS);
  const size_t lp = o;   o = al(o + (size_t)T_m * C * (MAXQ - 1) * SPLIT_THREADS * 8);
  const size_t pc = o;   o = al(o + (size_t)T_m * C * MAXQ * 4);
  const size_t uc = o;   o = al(o + (size_t)T_m * C * SPLIT_WAVES * 4);
  const size_t ul = o;   o = al(o + (size_t)T_m * C * SPLIT_WAVES * SPLIT_FL * 4);
  if (sp) {
    sp->plan = base + plan;
    sp->tab = (int8_t*)(base + tab);
    sp->lp = (double*)(base + lp);
    sp->pc = (int32_t*)(base + pc);
    sp->ucnt = (int32_t*)(base + uc);
    sp->ulist = (uint32_t*)(base + ul);
    sp->C = (int)C;
    sp->cells = CC;
  }
  return o;
}

static int deciles_dispatch(csm_ctx* ctx, const char* who, bool v2, int32_t T_m,
                            const double* M, const double* NR, int64_t N, int32_t n_bins,
                            const QTab& q, int8_t* L, double* EW, int32_t* CNT, int32_t* NV,
                            uint16_t* ids, bool pre, double* LS = nullptr) {
  // LS (the ids path only): narrow rows form the long-short in the decile launch (its last
  // workgroup); wide rows (C4) with k_long_short after it -- measured the same there
  // (1.968 vs 1.971 ms/step), and the general kernel stays free of the per-workgroup fence
  double* LSw = (LS && N > g_tune_dec_narrow_max) ? LS : nullptr;
  if (LSw) LS = nullptr;
  int32_t* tk = LS ? ctx->ticket : nullptr;
  int32_t* flg = nullptr;
  if (pre) {
    if (ctx->dec_flg_n < T_m) {   // beyond the create-time capacity
      if (capturing(ctx))           // a captured graph would keep the freed buffer's address
        return set_err(ctx, CSM_E_INVAL, "%s: %d rows exceed the context's row-flag buffer (%d) "
                       "during stream capture; run the call once before capturing", who, T_m,
                       ctx->dec_flg_n);
      if (ctx->dec_flg) HIP_CHECK(ctx, hipFree(ctx->dec_flg));
      ctx->dec_flg = nullptr;
      ctx->dec_flg_n = 0;
      HIP_CHECK(ctx, hipMalloc(&ctx->dec_flg, (size_t)T_m * sizeof(int32_t)));
      ctx->dec_flg_n = T_m;
    }
    flg = ctx->dec_flg;
    // wide rows of a short date shard (fewer rows than half the CUs: one workgroup per row
    // leaves most of the chip idle): the split pass (plan, chunked sweep over the whole chip,
    // finish with the fused long-short) when the row's (chunk, wave) lists fit the finish
    // launch's merge.  Same labels and counts as the merged pass; means in another fixed order.
    const int64_t C = (N + g_tune_dec_split_cells - 1) / g_tune_dec_split_cells;
    const bool split = g_tune_dec_split == 1 ||
                       (g_tune_dec_split == 2 && (int64_t)T_m * 2 <= (int64_t)ctx->n_cu);
    if (split && g_tune_dec_merge && !q.legs && N > g_tune_dec_narrow_max &&
        C * SPLIT_WAVES <= DSPLIT_MAXL) {
      const size_t need = dsplit_layout(T_m, N, nullptr, nullptr);
      if (ctx->dsplit_bytes < need) {
        if (capturing(ctx))
          return set_err(ctx, CSM_E_INVAL, "%s: the split decile workspace (%zu B) must grow to %zu B "
                         "during stream capture; run the call once before capturing", who,
                         ctx->dsplit_bytes, need);
        if (ctx->dsplit) HIP_CHECK(ctx, hipFree(ctx->dsplit));
        ctx->dsplit = nullptr;
        ctx->dsplit_bytes = 0;
        HIP_CHECK(ctx, hipMalloc(&ctx->dsplit, need));
        ctx->dsplit_bytes = need;
      }
      DecSplit sp;
      dsplit_layout(T_m, N, &sp, (char*)ctx->dsplit);
      sp.pf = g_tune_dec_split_pf == 2 ? (C * T_m <= (int64_t)ctx->n_cu) : g_tune_dec_split_pf;
      int64_t* tm = g_dec_timing;
      double* lsx = NR ? LSw : nullptr;
      int32_t* tkx = lsx ? ctx->ticket : nullptr;
      switch (NR ? n_bins : 0) {
#define DS_CASE(NBV) case NBV: launch_deciles_split<NBV>(T_m, ctx->stream, M, NR, N, n_bins, q, L, EW, CNT, NV, tm, ids, flg, sp, lsx, tkx); break;
        DS_CASE(0) DS_CASE(2) DS_CASE(3) DS_CASE(4) DS_CASE(5) DS_CASE(10) DS_CASE(20)
#undef DS_CASE
        default:
          return set_err(ctx, CSM_E_INVAL, "%s: n_bins=%d unsupported with NR (use 2,3,4,5,10,20)", who, n_bins);
      }
      LAUNCH_CHECK(ctx, who);
      return CSM_OK;
    }
  }
  if (!NR) {
    launch_deciles<0>(v2, T_m, ctx->stream, M, nullptr, N, n_bins, q, L, nullptr, nullptr, NV, ids, pre, flg);
  } else {
    switch (n_bins) {
      case 2: launch_deciles<2>(v2, T_m, ctx->stream, M, NR, N, n_bins, q, L, EW, CNT, NV, ids, pre, flg, LS, tk); break;
      case 3: launch_deciles<3>(v2, T_m, ctx->stream, M, NR, N, n_bins, q, L, EW, CNT, NV, ids, pre, flg, LS, tk); break;
      case 4: launch_deciles<4>(v2, T_m, ctx->stream, M, NR, N, n_bins, q, L, EW, CNT, NV, ids, pre, flg, LS, tk); break;
      case 5: launch_deciles<5>(v2, T_m, ctx->stream, M, NR, N, n_bins, q, L, EW, CNT, NV, ids, pre, flg, LS, tk); break;
      case 10: launch_deciles<10>(v2, T_m, ctx->stream, M, NR, N, n_bins, q, L, EW, CNT, NV, ids, pre, flg, LS, tk); break;
      case 20: launch_deciles<20>(v2, T_m, ctx->stream, M, NR, N, n_bins, q, L, EW, CNT, NV, ids, pre, flg, LS, tk); break;
      default:
        return set_err(ctx, CSM_E_INVAL, "%s: n_bins=%d unsupported with NR (use 2,3,4,5,10,20)", who, n_bins);
    }
  }
  LAUNCH_CHECK(ctx, who);
  if (LSw) {
    hipLaunchKernelGGL(k_long_short, dim3(1), dim3(LS_THREADS), 0, ctx->stream, EW, CNT, T_m, n_bins, LSw);
    LAUNCH_CHECK(ctx, "k_long_short");
  }
  return CSM_OK;
}

static bool ids_ok(int64_t N, const double* M, const double* NR, const int8_t* L, const uint16_t* ids) {
  return ids && (N % 4) == 0 && ((uintptr_t)ids & 7u) == 0 && aligned16(M) && (!NR || aligned16(NR)) &&
         (((uintptr_t)L & 3u) == 0);
}

int csm_deciles_ids(csm_ctx* ctx, const double* M, const double* NR, const uint16_t* ids,
                    int32_t T_m, int64_t N, int32_t n_bins, const double* qtable, int8_t* L,
                    double* EW, int32_t* CNT, int32_t* NV) {
  int r = prep(ctx);
  if (r) return r;
  if (!M || !L || !qtable || N <= 0 || T_m < 0 || n_bins < 1 || n_bins > MAXQ - 1 || N > 0x7FFFFFFFLL)
    return set_err(ctx, CSM_E_INVAL, "csm_deciles_ids: bad arguments (N=%lld T_m=%d n_bins=%d)",
                   (long long)N, T_m, n_bins);
  if (NR && (!EW || !CNT))
    return set_err(ctx, CSM_E_INVAL, "csm_deciles_ids: EW and CNT are required when NR is given");
  if (!ids_ok(N, M, NR, L, ids))
    return set_err(ctx, CSM_E_INVAL, "csm_deciles_ids: needs N %% 4 == 0, 8-B aligned ids, 16-B aligned "
                   "M / NR, 4-B aligned L (N=%lld)", (long long)N);
  if (T_m == 0) return CSM_OK;
  QTab q;
  for (int i = 0; i < MAXQ; ++i) q.q[i] = i <= n_bins ? qtable[i] : 1.0;
  return deciles_dispatch(ctx, "csm_deciles_ids", true, T_m, M, NR, N, n_bins, q, L, EW, CNT, NV,
                          const_cast<uint16_t*>(ids), true);
}

int csm_deciles_ids_legs(csm_ctx* ctx, const double* M, const uint16_t* ids, int32_t T_m,
                         int64_t N, int32_t n_bins, const double* qtable, int8_t* L, int32_t* NV) {
  int r = prep(ctx);
  if (r) return r;
  if (!M || !L || !qtable || N <= 0 || T_m < 0 || n_bins < 1 || n_bins > MAXQ - 1 || N > 0x7FFFFFFFLL)
    return set_err(ctx, CSM_E_INVAL, "csm_deciles_ids_legs: bad arguments (N=%lld T_m=%d n_bins=%d)",
                   (long long)N, T_m, n_bins);
  if (!ids_ok(N, M, nullptr, L, ids))
    return set_err(ctx, CSM_E_INVAL, "csm_deciles_ids_legs: needs N %% 4 == 0, 8-B aligned ids, "
                   "16-B aligned M, 4-B aligned L (N=%lld)", (long long)N);
  if (T_m == 0) return CSM_OK;
  QTab q;
  for (int i = 0; i < MAXQ; ++i) q.q[i] = i <= n_bins ? qtable[i] : 1.0;
  q.legs = 1;
  return deciles_dispatch(ctx, "csm_deciles_ids_legs", true, T_m, M, nullptr, N, n_bins, q, L,
                          nullptr, nullptr, NV, const_cast<uint16_t*>(ids), true);
}

int csm_deciles_ids_ls(csm_ctx* ctx, const double* M, const double* NR, const uint16_t* ids,
                       int32_t T_m, int64_t N, int32_t n_bins, const double* qtable, int8_t* L,
                       double* EW, int32_t* CNT, int32_t* NV, double* LS) {
  int r = prep(ctx);
  if (r) return r;
  if (!M || !NR || !EW || !CNT || !LS || !L || !qtable || N <= 0 || T_m < 0 || n_bins < 1 ||
      n_bins > MAXQ - 1 || N > 0x7FFFFFFFLL)
    return set_err(ctx, CSM_E_INVAL, "csm_deciles_ids_ls: bad arguments (N=%lld T_m=%d n_bins=%d; "
                   "NR, EW, CNT and LS required)", (long long)N, T_m, n_bins);
  if (!ids_ok(N, M, NR, L, ids))
    return set_err(ctx, CSM_E_INVAL, "csm_deciles_ids_ls: needs N %% 4 == 0, 8-B aligned ids, 16-B "
                   "aligned M / NR, 4-B aligned L (N=%lld)", (long long)N);
  if (T_m == 0) return CSM_OK;
  QTab q;
  for (int i = 0; i < MAXQ; ++i) q.q[i] = i <= n_bins ? qtable[i] : 1.0;
  return deciles_dispatch(ctx, "csm_deciles_ids_ls", true, T_m, M, NR, N, n_bins, q, L, EW, CNT,
                          NV, const_cast<uint16_t*>(ids), true, LS);
}

int csm_pipeline(csm_ctx* ctx, const double* P, int64_t T_d, int64_t N, const int64_t* month_start,
                 int32_t T_m, int32_t max_month_days, int32_t min_month_days, int32_t J,
                 int32_t skip, int32_t n_bins,
                 const double* qtable, double* PM, double* R, double* M, double* NR, int8_t* L,
                 double* EW, int32_t* CNT, int32_t* NV, double* LS) {
  int r = prep(ctx);
  if (r) return r;
  if (!P || !month_start || !qtable || !M || !NR || !L || !EW || !CNT || !LS || N <= 0 ||
      T_m < 0 || n_bins < 1 || n_bins > MAXQ - 1 || N > 0x7FFFFFFFLL)
    return set_err(ctx, CSM_E_INVAL, "csm_pipeline: bad arguments (N=%lld T_m=%d n_bins=%d)",
                   (long long)N, T_m, n_bins);
  if (T_m == 0) return CSM_OK;
  // the id path needs 4-aligned rows and the wide decile kernel; otherwise signal + deciles
  uint16_t* ids = nullptr;
  const bool want_ids = (N % 4) == 0 && N > g_tune_dec_narrow_max && aligned16(P) && aligned16(M) &&
                        aligned16(NR) && (((uintptr_t)L & 3u) == 0) && (!PM || aligned16(PM)) &&
                        (!R || aligned16(R));
  if (want_ids) {
    const size_t need = (size_t)T_m * (size_t)N * sizeof(uint16_t);
    if (ctx->scratch_bytes < need) {
      if (capturing(ctx))
        return set_err(ctx, CSM_E_INVAL, "csm_pipeline: the bucket-id scratch (%zu B) must grow to "
                       "%zu B during stream capture; run the call once before capturing",
                       ctx->scratch_bytes, need);
      if (ctx->scratch) HIP_CHECK(ctx, hipFree(ctx->scratch));
      ctx->scratch = nullptr;
      ctx->scratch_bytes = 0;
      HIP_CHECK(ctx, hipMalloc(&ctx->scratch, need));
      ctx->scratch_bytes = need;
    }
    ids = (uint16_t*)ctx->scratch;
  }
  (void)min_month_days;
  r = signal_launch(ctx, "csm_pipeline", P, T_d, N, month_start, T_m, max_month_days, J,
                    skip, PM, R, M, NR, nullptr, nullptr, nullptr, false, ids);
  if (r) return r;
  QTab q;
  for (int i = 0; i < MAXQ; ++i) q.q[i] = i <= n_bins ? qtable[i] : 1.0;
  const bool v2 = (N % 2 == 0) && aligned16(M) && aligned16(NR) && (((uintptr_t)L & 1u) == 0);
  // the id path: labels, decile means and the long-short in one launch
  r = deciles_dispatch(ctx, "csm_pipeline", v2, T_m, M, NR, N, n_bins, q, L, EW, CNT, NV, ids,
                       ids != nullptr, ids ? LS : nullptr);
  if (r || ids) return r;
  hipLaunchKernelGGL(k_long_short, dim3(1), dim3(LS_THREADS), 0, ctx->stream, EW, CNT, T_m, n_bins, LS);
  LAUNCH_CHECK(ctx, "k_long_short");
  return CSM_OK;
}

int csm_shard_summary(csm_ctx* ctx, const double* PM, int32_t T_m, int64_t N, int32_t J,
                      int32_t skip, double* out) {
  int r = prep(ctx);
  if (r) return r;
  if (!PM || !out || N <= 0 || T_m < 0 || J < 1 || skip < 0 || J + skip > 256)
    return set_err(ctx, CSM_E_INVAL, "csm_shard_summary: bad arguments");
  const unsigned blocks = (unsigned)((N + 255) / 256);
  hipLaunchKernelGGL(k_shard_summary, dim3(blocks), dim3(256), 0, ctx->stream, PM, T_m, N,
                     J + skip + 1, out);
  LAUNCH_CHECK(ctx, "k_shard_summary");
  return CSM_OK;
}

int csm_fold_carry(csm_ctx* ctx, const double* summaries, int32_t G, int32_t g, int64_t N,
                   int32_t J, int32_t skip, double* carry, double* next_pm) {
  int r = prep(ctx);
  if (r) return r;
  if (!summaries || !carry || !next_pm || N <= 0 || G < 1 || g < 0 || g >= G || J < 1 ||
      skip < 0 || J + skip > 256)
    return set_err(ctx, CSM_E_INVAL, "csm_fold_carry: bad arguments");
  const unsigned blocks = (unsigned)((N + 255) / 256);
  hipLaunchKernelGGL(k_fold_carry, dim3(blocks), dim3(256), 0, ctx->stream, summaries, G, g, N, J,
                     skip, carry, next_pm, (const double*)nullptr, FoldJs{0, {0, 0, 0, 0}},
                     (double*)nullptr);
  LAUNCH_CHECK(ctx, "k_fold_carry");
  return CSM_OK;
}

int csm_shard_summary_state(csm_ctx* ctx, const double* P, const int64_t* month_start,
                            const double* PM, int32_t T_m, int64_t N, int32_t J, int32_t skip,
                            const double* state, double* out) {
  int r = prep(ctx);
  if (r) return r;
  if (!P || !month_start || !PM || !state || !out || N <= 0 || T_m < 1 || J < 1 || skip < 0 ||
      J + skip > 256)
    return set_err(ctx, CSM_E_INVAL, "csm_shard_summary_state: bad arguments");
  hipLaunchKernelGGL(k_shard_summary_state, dim3((unsigned)((N + 255) / 256)), dim3(256), 0,
                     ctx->stream, PM, P, month_start, T_m, N, J + skip + 1, state, out,
                     (const int32_t*)nullptr, (const int32_t*)nullptr, (int64_t)0);
  LAUNCH_CHECK(ctx, "k_shard_summary_state");
  return CSM_OK;
}

static int shard_repair(csm_ctx* ctx, const double* P, const int64_t* month_start, const double* PM,
                     int32_t T_m, int64_t N, int32_t J, int32_t skip, const double* carry,
                     const double* next_pm, const double* state, double* R, double* M,
                     double* NR, uint16_t* ids) {
  int r = prep(ctx);
  if (r) return r;
  if (!P || !month_start || !PM || !carry || !next_pm || !state || !M || !NR || N <= 0 ||
      T_m < 1 || J < 1 ||
      skip < 0 || J + skip > 128)
    return set_err(ctx, CSM_E_INVAL, "csm_shard_repair: bad arguments (J + skip <= 128)");
  const int W = J + skip;
  const size_t lds = (size_t)2 * W * REPAIR_THREADS * sizeof(double);
  if (lds > 65536)
    HIP_CHECK(ctx, hipFuncSetAttribute((const void*)k_shard_repair,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(k_shard_repair, dim3((unsigned)((N + REPAIR_THREADS - 1) / REPAIR_THREADS)),
                     dim3(REPAIR_THREADS), lds, ctx->stream, PM, P, month_start, T_m, N, J, skip,
                     carry, next_pm, state, R, M, NR, ids, (const double*)nullptr,
                     (const int32_t*)nullptr, (const int32_t*)nullptr, (int64_t)0);
  LAUNCH_CHECK(ctx, "k_shard_repair");
  return CSM_OK;
}

int csm_shard_repair(csm_ctx* ctx, const double* P, const int64_t* month_start, const double* PM,
                     int32_t T_m, int64_t N, int32_t J, int32_t skip, const double* carry,
                     const double* next_pm, const double* state, double* R, double* M,
                     double* NR) {
  return shard_repair(ctx, P, month_start, PM, T_m, N, J, skip, carry, next_pm, state, R, M, NR,
                      nullptr);
}

int csm_shard_repair_ids(csm_ctx* ctx, const double* P, const int64_t* month_start,
                         const double* PM, int32_t T_m, int64_t N, int32_t J, int32_t skip,
                         const double* carry, const double* next_pm, const double* state,
                         double* R, double* M, double* NR, uint16_t* ids) {
  if (!ids) return set_err(ctx, CSM_E_INVAL, "csm_shard_repair_ids: ids is NULL");
  return shard_repair(ctx, P, month_start, PM, T_m, N, J, skip, carry, next_pm, state, R, M, NR,
                      ids);
}

// ---- halo date shards (k_shard_halo above; include/csmom.h) -------------------------------
int csm_shard_halo(csm_ctx* ctx, const double* P, int64_t T_d, int64_t N,
                   const int64_t* month_start, int32_t H, int32_t T_m, int32_t F,
                   int32_t before, int32_t after, int32_t J, int32_t skip, double* halo_pm,
                   double* carry, double* next_pm, uint8_t* flags) {
  int r = prep(ctx);
  if (r) return r;
  if (!P || !month_start || !carry || !next_pm || !flags || (H + F > 0 && !halo_pm) || N <= 0 ||
      T_d <= 0 || H < 0 || T_m < 1 || F < 0 || F > 8 || J < 1 || skip < 0 || J + skip > 64)
    return set_err(ctx, CSM_E_INVAL, "csm_shard_halo: bad arguments (H >= 0, T_m >= 1, 0 <= F <= 8, "
                   "J + skip <= 64, halo_pm [H + F][N])");
  const int W = J + skip;
  const unsigned bx = (unsigned)((N + HALO_THREADS - 1) / HALO_THREADS);
  if (H + F > 0) {
    hipLaunchKernelGGL(k_halo_pm, dim3(bx, (unsigned)(H + F)), dim3(HALO_THREADS), 0, ctx->stream,
                       P, month_start, H, T_m, N, halo_pm);
    LAUNCH_CHECK(ctx, "k_halo_pm");
  }
  const size_t lds = (size_t)W * HALO_THREADS * sizeof(double);
  if (lds > 65536)
    HIP_CHECK(ctx, hipFuncSetAttribute((const void*)k_shard_halo,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(k_shard_halo, dim3(bx), dim3(HALO_THREADS), lds, ctx->stream,
                     (const double*)halo_pm, H, F, before ? 1 : 0, after ? 1 : 0, N, J, skip, carry,
                     next_pm, flags);
  LAUNCH_CHECK(ctx, "k_shard_halo");
  return CSM_OK;
}

int csm_signal_halo(csm_ctx* ctx, const double* P, int64_t T_d, int64_t N,
                    const int64_t* month_start, int32_t H, int32_t T_m, int32_t F, int32_t before,
                    int32_t after, int32_t max_month_days, int32_t J, int32_t skip, double* PM,
                    double* R, double* M, double* NR, double* state, uint16_t* ids,
                    uint8_t* flags) {
  if (!flags || H < 0 || F < 0 || F > 8 || J + skip > 64)
    return set_err(ctx, CSM_E_INVAL, "csm_signal_halo: bad arguments (flags [N], H >= 0, "
                   "0 <= F <= 8, J + skip <= 64)");
  if (ids && ((N % 4) != 0 || ((uintptr_t)ids & 7u) != 0))
    return set_err(ctx, CSM_E_INVAL, "csm_signal_halo: ids need N %% 4 == 0, 8-B alignment");
  const HaloArgs ha{H, F, before ? 1 : 0, after ? 1 : 0, flags};
  return signal_launch(ctx, "csm_signal_halo", P, T_d, N, month_start, T_m, max_month_days, J,
                       skip, PM, R, M, NR, nullptr, nullptr, state, true, ids, &ha);
}

int csm_signal_shard_halo(csm_ctx* ctx, const double* P, int64_t T_d, int64_t N,
                          const int64_t* month_start, int32_t T_m, int32_t max_month_days,
                          int32_t J, int32_t skip, const double* carry, const double* next_pm,
                          double* PM, double* R, double* M, double* NR, double* state,
                          uint16_t* ids) {
  if (!carry || !next_pm)
    return set_err(ctx, CSM_E_INVAL, "csm_signal_shard_halo: needs the halo's carry and next_pm");
  if (ids && ((N % 4) != 0 || ((uintptr_t)ids & 7u) != 0))
    return set_err(ctx, CSM_E_INVAL, "csm_signal_shard_halo: ids need N %% 4 == 0, 8-B alignment");
  return signal_launch(ctx, "csm_signal_shard_halo", P, T_d, N, month_start, T_m, max_month_days,
                       J, skip, PM, R, M, NR, carry, next_pm, state, true, ids);
}

int csm_shard_need(csm_ctx* ctx, const uint8_t* flags, const double* state, int64_t N,
                   int32_t T_m, int32_t H, uint64_t* mask) {
  int r = prep(ctx);
  if (r) return r;
  if (!flags || !state || !mask || N <= 0 || T_m < 1 || H < 0)
    return set_err(ctx, CSM_E_INVAL, "csm_shard_need: bad arguments");
  hipLaunchKernelGGL(k_shard_need, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, ctx->stream,
                     flags, state, N, T_m, H, (N + 63) / 64, mask);
  LAUNCH_CHECK(ctx, "k_shard_need");
  return CSM_OK;
}

int csm_shard_union(csm_ctx* ctx, const uint64_t* masks, int32_t G, int64_t N, int64_t cap,
                    int32_t* idx, int32_t* count) {
  int r = prep(ctx);
  if (r) return r;
  if (!masks || !idx || !count || G < 1 || G > HALO_MAXG || N <= 0 || cap < 1 ||
      N > 0x7FFFFFFFLL)
    return set_err(ctx, CSM_E_INVAL, "csm_shard_union: bad arguments (1 <= G <= %d)", HALO_MAXG);
  hipLaunchKernelGGL(k_shard_union, dim3(1), dim3(UNION_THREADS), 0, ctx->stream, masks, G,
                     (N + 63) / 64, cap, idx, count);
  LAUNCH_CHECK(ctx, "k_shard_union");
  return CSM_OK;
}

int csm_shard_summary_cols(csm_ctx* ctx, const double* P, const int64_t* month_start,
                           const double* PM, int32_t T_m, int64_t N, int32_t J, int32_t skip,
                           const double* state, const int32_t* idx, const int32_t* count,
                           int64_t cap, double* out) {
  int r = prep(ctx);
  if (r) return r;
  if (!P || !month_start || !PM || !state || !idx || !count || !out || N <= 0 || T_m < 1 ||
      cap < 1 || J < 1 || skip < 0 || J + skip > 256)
    return set_err(ctx, CSM_E_INVAL, "csm_shard_summary_cols: bad arguments");
  // one workgroup per listed column, its month prices derived together into LDS
  if (g_tune_cols_wg && (size_t)T_m * sizeof(double) <= 65536 && cap <= 0x7FFFFFFF) {
    const int64_t grid = std::min<int64_t>(cap, 2 * (int64_t)ctx->n_cu);
    hipLaunchKernelGGL(k_shard_summary_cols, dim3((unsigned)grid), dim3(COLS_THREADS),
                       (size_t)T_m * sizeof(double), ctx->stream, PM, P, month_start, T_m, N,
                       J + skip + 1, state, out, idx, count, cap);
    LAUNCH_CHECK(ctx, "k_shard_summary_cols");
    return CSM_OK;
  }
  hipLaunchKernelGGL(k_shard_summary_state, dim3((unsigned)((cap + 255) / 256)), dim3(256), 0,
                     ctx->stream, PM, P, month_start, T_m, N, J + skip + 1, state, out, idx,
                     count, cap);
  LAUNCH_CHECK(ctx, "k_shard_summary_state (columns)");
  return CSM_OK;
}

int csm_shard_repair_cols(csm_ctx* ctx, const double* P, const int64_t* month_start,
                          const double* PM, int32_t T_m, int64_t N, int32_t J, int32_t skip,
                          const double* carry, const double* next_pm, const double* fcarry,
                          const double* state, const int32_t* idx, const int32_t* count,
                          int64_t cap, double* R, double* M, double* NR, uint16_t* ids) {
  int r = prep(ctx);
  if (r) return r;
  if (!P || !month_start || !PM || !carry || !next_pm || !fcarry || !state || !idx || !count ||
      !M || !NR || N <= 0 || T_m < 1 || cap < 1 || J < 1 || skip < 0 || J + skip > 128)
    return set_err(ctx, CSM_E_INVAL, "csm_shard_repair_cols: bad arguments (J + skip <= 128)");
  const int W = J + skip;
  const size_t ldsc = (size_t)(T_m + 2 * W) * sizeof(double);
  if (g_tune_cols_wg && ldsc <= 65536 && cap <= 0x7FFFFFFF) {
    hipLaunchKernelGGL(k_shard_repair_cols, dim3((unsigned)cap), dim3(COLS_THREADS), ldsc,
                       ctx->stream, PM, P, month_start, T_m, N, J, skip, carry, next_pm, state,
                       R, M, NR, ids, fcarry, idx, count, cap);
    LAUNCH_CHECK(ctx, "k_shard_repair_cols");
    return CSM_OK;
  }
  const size_t lds = (size_t)2 * W * REPAIR_THREADS * sizeof(double);
  if (lds > 65536)
    HIP_CHECK(ctx, hipFuncSetAttribute((const void*)k_shard_repair,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(k_shard_repair, dim3((unsigned)((cap + REPAIR_THREADS - 1) / REPAIR_THREADS)),
                     dim3(REPAIR_THREADS), lds, ctx->stream, PM, P, month_start, T_m, N, J, skip,
                     carry, next_pm, state, R, M, NR, ids, fcarry, idx, count, cap);
  LAUNCH_CHECK(ctx, "k_shard_repair (columns)");
  return CSM_OK;
}

int csm_shard_fix_cols(csm_ctx* ctx, const double* P, const int64_t* month_start,
                       const double* PM, int32_t T_m, int64_t N, int32_t J, int32_t skip,
                       const double* records, int32_t G, int32_t g, const int32_t* idx,
                       const int32_t* count, int64_t cap, double* R, double* M, double* NR,
                       uint16_t* ids) {
  int r = prep(ctx);
  if (r) return r;
  const int W = J + skip;
  const size_t lds = (size_t)(T_m + 2 * W + 2 + (size_t)G * (SUM_SCALARS + W + 1)) * sizeof(double);
  if (!P || !month_start || !PM || !records || !idx || !count || !M || !NR || N <= 0 ||
      T_m < 1 || cap < 1 || cap > 0x7FFFFFFF || G < 1 || g < 0 || g >= G || J < 1 || skip < 0 ||
      W > 128 || G > HALO_MAXG || lds > 65536)
    return set_err(ctx, CSM_E_INVAL, "csm_shard_fix_cols: bad arguments (J + skip <= 128, "
                   "0 <= g < G <= %d, months, rings and records within 64 KB of LDS)", HALO_MAXG);
  // a workgroup per listed column, at most two per CU (the list is short; the rest exit at once)
  const int64_t grid = cap < 2 * (int64_t)ctx->n_cu ? cap : 2 * (int64_t)ctx->n_cu;
  // (C4's look-back J = 12, skip = 1: the ring in registers and the product length fixed)
  const void* fn = (J == 12 && skip == 1) ? (const void*)k_shard_fix_cols<13, 12>
                                          : (const void*)k_shard_fix_cols<0, 0>;
  {
    int T_m_ = T_m, J_ = J, skip_ = skip, G_ = G, g_ = g;
    int64_t N_ = N, cap_ = cap;
    void* args[] = {(void*)&PM, (void*)&P, (void*)&month_start, &T_m_, &N_, &J_, &skip_,
                    (void*)&records, &G_, &g_, (void*)&R, (void*)&M, (void*)&NR, (void*)&ids,
                    (void*)&idx, (void*)&count, &cap_};
    HIP_CHECK(ctx, hipLaunchKernel(fn, dim3((unsigned)grid), dim3(COLS_THREADS), args, lds,
                                   ctx->stream));
  }
  LAUNCH_CHECK(ctx, "k_shard_fix_cols");
  return CSM_OK;
}

int64_t csm_momentum_chunked_workspace(int32_t T_m, int64_t N, int32_t J, int32_t skip,
                                       int32_t C) {
  if (N <= 0 || C < 1 || J < 1 || skip < 0) return 0;
  const int64_t S = SUM_SCALARS + J + skip + 1, W = J + skip;
  (void)T_m;
  return (int64_t)C * (S + (W + 2) + 1) * N * (int64_t)sizeof(double);
}

static int momentum_chunked(csm_ctx* ctx, const double* PM, int32_t T_m, int64_t N, int32_t J,
                            int32_t skip, int32_t C, double* R, double* M, double* NR,
                            const double* next_pm, void* workspace, uint16_t* IDS) {
  int r = prep(ctx);
  if (r) return r;
  if (!PM || !M || !NR || !workspace || N <= 0 || T_m < 0 || J < 1 || skip < 0 ||
      J + skip > 256 || C < 1 || C > 65535)
    return set_err(ctx, CSM_E_INVAL, "csm_momentum_chunked: bad arguments (N=%lld T_m=%d C=%d)",
                   (long long)N, T_m, C);
  if (T_m == 0) return CSM_OK;
  if (C > T_m) C = T_m;
  const int W = J + skip, T = W + 1, S = SUM_SCALARS + T;
  double* sm = (double*)workspace;
  double* carry = sm + (int64_t)C * S * N;
  double* npm = carry + (int64_t)C * (W + 2) * N;
  const unsigned bx = (unsigned)((N + 255) / 256);
  hipLaunchKernelGGL(k_shard_summary_chunked, dim3(bx, C), dim3(256), 0, ctx->stream, PM, T_m, N,
                     T, C, sm);
  LAUNCH_CHECK(ctx, "k_shard_summary_chunked");
  hipLaunchKernelGGL(k_fold_carry, dim3(bx, C), dim3(256), 0, ctx->stream, (const double*)sm, C,
                     -1, N, J, skip, carry, npm, next_pm, FoldJs{0, {0, 0, 0, 0}}, (double*)nullptr);
  LAUNCH_CHECK(ctx, "k_fold_carry");
  const int tpb = W <= 64 ? SCAN_THREADS : 64;
  const size_t lds = (size_t)W * tpb * sizeof(double);
  if (lds > 65536)
    HIP_CHECK(ctx, hipFuncSetAttribute((const void*)k_momentum_chunked,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(k_momentum_chunked, dim3((unsigned)((N + tpb - 1) / tpb), C), dim3(tpb), lds,
                     ctx->stream, PM, T_m, C, N, J, skip, R, M, NR, (const double*)carry,
                     (const double*)npm, IDS);
  LAUNCH_CHECK(ctx, "k_momentum_chunked");
  return CSM_OK;
}

int csm_momentum_chunked(csm_ctx* ctx, const double* PM, int32_t T_m, int64_t N, int32_t J,
                         int32_t skip, int32_t C, double* R, double* M, double* NR,
                         const double* next_pm, void* workspace) {
  return momentum_chunked(ctx, PM, T_m, N, J, skip, C, R, M, NR, next_pm, workspace, nullptr);
}

int64_t csm_momentum_multi_chunked_workspace(int32_t T_m, int64_t N, int32_t Jmax, int32_t skip,
                                             int32_t C) {
  if (N <= 0 || C < 1 || Jmax < 1 || skip < 0) return 0;
  const int64_t W = Jmax + skip, S = SUM_SCALARS + W + 1;
  (void)T_m;
  return (int64_t)C * (S + (W + 2) + 1 + MJ_MAX) * N * (int64_t)sizeof(double);
}

int csm_momentum_multi_chunked(csm_ctx* ctx, const double* PM, int32_t T_m, int64_t N,
                               const int32_t* Js, int32_t nJ, int32_t skip, int32_t C,
                               double* const* M, double* const* NR, uint16_t* const* IDS,
                               void* workspace) {
  int r = prep(ctx);
  if (r) return r;
  if (!PM || !Js || !M || !NR || !workspace || N <= 0 || T_m < 0 || nJ < 1 || nJ > MJ_MAX ||
      skip < 0 || C < 1 || C > 65535)
    return set_err(ctx, CSM_E_INVAL, "csm_momentum_multi_chunked: bad arguments (N=%lld T_m=%d "
                   "nJ=%d C=%d; 1 <= nJ <= %d)", (long long)N, T_m, nJ, C, MJ_MAX);
  MJSet mj;
  FoldJs fj;
  fj.n = nJ;
  int Jmax = 0;
  bool al = (N % 2) == 0 && aligned16(PM) && aligned16(workspace);
  for (int q = 0; q < MJ_MAX; ++q) {
    const bool on = q < nJ;
    mj.J[q] = fj.J[q] = on ? Js[q] : 1;
    mj.M[q] = on ? M[q] : nullptr;
    mj.NR[q] = on ? NR[q] : nullptr;
    mj.IDS[q] = (on && IDS) ? IDS[q] : nullptr;
    if (on && (Js[q] < 1 || !M[q] || !NR[q] || (IDS && !IDS[q])))
      return set_err(ctx, CSM_E_INVAL, "csm_momentum_multi_chunked: J[%d]=%d or its outputs invalid",
                     q, on ? Js[q] : 0);
    if (on) {
      al = al && aligned16(M[q]) && aligned16(NR[q]) && (!IDS || ((uintptr_t)IDS[q] & 3u) == 0);
      Jmax = Js[q] > Jmax ? Js[q] : Jmax;
    }
  }
  const int W = Jmax + skip;
  if (W > MJ_REG_W || !al)
    return set_err(ctx, CSM_E_INVAL, "csm_momentum_multi_chunked: needs max(J) + skip <= %d, even N "
                   "and 16-B aligned PM / M / NR / workspace, 4-B aligned ids (W=%d N=%lld)",
                   MJ_REG_W, W, (long long)N);
  if (T_m == 0) return CSM_OK;
  if (C > T_m) C = T_m;
  const int T = W + 1, S = SUM_SCALARS + T;
  double* sm = (double*)workspace;
  double* carry = sm + (int64_t)C * S * N;
  double* npm = carry + (int64_t)C * (W + 2) * N;
  double* psq = npm + (int64_t)C * N;
  const unsigned bx = (unsigned)((N + 255) / 256);
  hipLaunchKernelGGL(k_shard_summary_chunked, dim3(bx, C), dim3(256), 0, ctx->stream, PM, T_m, N,
                     T, C, sm);
  LAUNCH_CHECK(ctx, "k_shard_summary_chunked");
  hipLaunchKernelGGL(k_fold_carry, dim3(bx, C), dim3(256), 0, ctx->stream, (const double*)sm, C,
                     -1, N, Jmax, skip, carry, npm, (const double*)nullptr, fj, psq);
  LAUNCH_CHECK(ctx, "k_fold_carry");
  const int tpb = SCAN_THREADS;
  const dim3 grid((unsigned)((N / 2 + tpb - 1) / tpb), (unsigned)C);
  if (mj_fixed_grid(Js, nJ, skip))
    hipLaunchKernelGGL((k_momentum_multi_reg2<13, true, true>), grid, dim3(tpb), 0, ctx->stream,
                       PM, T_m, N, nJ, skip, mj, C, (const double*)carry, (const double*)npm,
                       (const double*)psq);
  else
    hipLaunchKernelGGL((k_momentum_multi_reg2<MJ_REG_W, true>), grid, dim3(tpb), 0, ctx->stream,
                       PM, T_m, N, nJ, skip, mj, C, (const double*)carry, (const double*)npm,
                       (const double*)psq);
  LAUNCH_CHECK(ctx, "k_momentum_multi_reg2 (chunked)");
  return CSM_OK;
}

int csm_momentum_chunked_ids(csm_ctx* ctx, const double* PM, int32_t T_m, int64_t N, int32_t J,
                             int32_t skip, int32_t C, double* R, double* M, double* NR,
                             const double* next_pm, uint16_t* ids, void* workspace) {
  if (!ids || (N % 4) != 0 || ((uintptr_t)ids & 7u) != 0)
    return set_err(ctx, CSM_E_INVAL, "csm_momentum_chunked_ids: ids must be non-NULL and 8-B "
                   "aligned, N %% 4 == 0 (N=%lld)", (long long)N);
  return momentum_chunked(ctx, PM, T_m, N, J, skip, C, R, M, NR, next_pm, workspace, ids);
}

// ---- the fused time-chunked signal (k_signal_tc, narrow panels) ----
static int64_t tc_sync_bytes(int G, int nbx) {
  return ((int64_t)(TC_SYNC0 + (int64_t)G * nbx) * 4 + 255) / 256 * 256;
}

int64_t csm_signal_chunked_workspace(int32_t T_m, int64_t N, int32_t J, int32_t skip, int32_t C) {
  if (N <= 0 || C < 1 || J < 1 || skip < 0) return 0;
  (void)T_m;
  const int64_t nbx = (N + TC_COLS - 1) / TC_COLS, SR = SUM_SCALARS + J + skip + 2;
  int64_t b = tc_sync_bytes(C, (int)nbx) + (int64_t)C * nbx * SR * TC_COLS * (int64_t)sizeof(double);
#ifdef TC_TIMING
  b += (int64_t)C * nbx * 64;
#endif
  return b;
}

int csm_signal_chunked(csm_ctx* ctx, const double* P, int64_t T_d, int64_t N,
                       const int64_t* month_start, int32_t T_m, int32_t max_month_days,
                       int32_t J, int32_t skip, int32_t C, double* R, double* M, double* NR,
                       uint16_t* ids, void* workspace) {
  int r = prep(ctx);
  if (r) return r;
  const int W = J + skip;
  if (!P || !month_start || !M || !NR || !workspace || N <= 0 || (N % 2) != 0 || T_d <= 0 ||
      T_m < 0 || J < 1 || skip < 0 || W > 32 || C < 1 || C > TC_MAXG || max_month_days < 0 ||
      max_month_days > TC_MAXD || !aligned16(P) || !aligned16(M) || !aligned16(NR) ||
      (R && !aligned16(R)) || (ids && ((uintptr_t)ids & 3u) != 0) || N * 8 * TC_MAXD > INT32_MAX ||
      ((uintptr_t)workspace & 255u) != 0)
    return set_err(ctx, CSM_E_INVAL, "csm_signal_chunked: bad arguments (N=%lld even, T_m=%d, "
                   "J + skip <= 32, 1 <= C <= %d, months of <= %d day rows, 16-B aligned P / M / "
                   "NR / R, 4-B aligned ids, 256-B aligned workspace)", (long long)N, T_m,
                   TC_MAXG, TC_MAXD);
  if (T_m == 0) return CSM_OK;
  if (C > T_m) C = T_m;
  const int maxc = (T_m + C - 1) / C;
  if (maxc > TC_MAXC)
    return set_err(ctx, CSM_E_INVAL, "csm_signal_chunked: %d months per chunk (at most %d: more "
                   "chunks)", maxc, TC_MAXC);
  const int nbx = (int)((N + TC_COLS - 1) / TC_COLS);
  unsigned* sync = (unsigned*)workspace;
  double* rec = (double*)((char*)workspace + tc_sync_bytes(C, nbx));
  const size_t lds = (size_t)(W + 1 + maxc) * TC_COLS * sizeof(double);
  // the C2 look-back (J = 12, skip = 1) with its ring in registers; any other, from LDS
  // (and the C2 window J = 12 with its product length fixed at compile time)
  const void* kfn = W == 13 ? (J == 12 ? (const void*)k_signal_tc<13, 12> : (const void*)k_signal_tc<13>)
                            : (const void*)k_signal_tc<0>;
  if (lds > 65536)
    HIP_CHECK(ctx, hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  if (W == 13 && J == 12)
    hipLaunchKernelGGL((k_signal_tc<13, 12>), dim3((unsigned)(C * nbx)), dim3(TC_THREADS), lds,
                       ctx->stream, P, month_start, T_m, N, J, skip, C, nbx, R, M, NR, ids, rec,
                       sync, g_tune_tc_spins);
  else if (W == 13)
    hipLaunchKernelGGL(k_signal_tc<13>, dim3((unsigned)(C * nbx)), dim3(TC_THREADS), lds,
                       ctx->stream, P, month_start, T_m, N, J, skip, C, nbx, R, M, NR, ids, rec,
                       sync, g_tune_tc_spins);
  else
    hipLaunchKernelGGL(k_signal_tc<0>, dim3((unsigned)(C * nbx)), dim3(TC_THREADS), lds,
                       ctx->stream, P, month_start, T_m, N, J, skip, C, nbx, R, M, NR, ids, rec,
                       sync, g_tune_tc_spins);
  LAUNCH_CHECK(ctx, "k_signal_tc");
  return CSM_OK;
}

int csm_signal_chunked_status(csm_ctx* ctx, void* workspace) {
  int r = prep(ctx);
  if (r) return r;
  if (!workspace || ((uintptr_t)workspace & 255u) != 0)
    return set_err(ctx, CSM_E_INVAL, "csm_signal_chunked_status: null or unaligned workspace");
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  HIP_CHECK(ctx, hipStreamIsCapturing(ctx->stream, &cs));
  if (cs != hipStreamCaptureStatusNone)
    return set_err(ctx, CSM_E_INVAL, "csm_signal_chunked_status: the stream is capturing (read "
                   "the status after the graph's replay)");
  unsigned w = 0;
  unsigned* word = (unsigned*)workspace + 2;
  HIP_CHECK(ctx, hipMemcpyAsync(&w, word, sizeof(w), hipMemcpyDeviceToHost, ctx->stream));
  HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
  if (w == 0u) return CSM_OK;
  // reported once: cleared for the workspace's next launch
  HIP_CHECK(ctx, hipMemsetAsync(word, 0, sizeof(unsigned), ctx->stream));
  HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
  return set_err(ctx, CSM_E_TIMEOUT, "csm_signal_chunked: a workgroup gave up waiting for an "
                 "earlier chunk's record (in-launch hand-off); the M / NR / R / ids of the "
                 "launches since the last status check are invalid");
}

}  // extern "C"
