// csm_common.h -- shared by the engine's translation units: the NaN-payload presence
// encoding, the context object and the status/error plumbing of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/csmom.h"

#define ABSENT_BITS 0x7FF4000000000001ULL
#define ABSENT_MASK 0x7FF7FFFFFFFFFFFFULL

__device__ __forceinline__ bool is_absent(double x) {
  return (((uint64_t)__double_as_longlong(x)) & ABSENT_MASK) == ABSENT_BITS;
}
__device__ __forceinline__ double absent_val() { return __longlong_as_double((long long)ABSENT_BITS); }
__device__ __forceinline__ double qnan() { return __longlong_as_double(0x7FF8000000000000LL); }
__device__ __forceinline__ bool isnan_d(double x) { return x != x; }


struct csm_ctx {
  int device;
  hipStream_t stream;
  char err[512];
  void* scratch;          // context-owned device workspace (k_deciles bucket ids), grown lazily
  size_t scratch_bytes;
  int n_cu;               // compute units of the device (decile kernel choice)
  int32_t* dec_flg;       // [dec_flg_n] rows the merged decile pass left to the general kernel
  int32_t dec_flg_n;      // (allocated at create, so a captured pipeline never allocates)
  int32_t* ticket;        // the fused long-short's arrival counter (zeroed at create; it wraps
                          // back to 0 on each decile launch's last increment)
  void* dsplit;           // the split decile pass's workspace (DecSplit), grown lazily
  size_t dsplit_bytes;
  void* comm;             // RCCL communicator of csm_allgather_init (collective.hip), or NULL
  int comm_rank, comm_size;
  // portfolio workspaces and what their last cohort pass wrote (portfolio.hip): bit 0 the leg
  // bitplanes -- the turnover pass reads bitplanes only from a workspace recorded here, whatever
  // the tune knobs say by then (a knob changed between the two calls falls back to the label
  // bytes) -- bit 1 legs-only cohort partials in the two-leg layout ([rows][K][C][2])
  void* planes_ws[32];
  unsigned char planes_bits[32];
  int planes_next;
};

static inline int set_err(csm_ctx* c, int code, const char* fmt, ...) {
  if (c) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(c->err, sizeof(c->err), fmt, ap);
    va_end(ap);
  }
  return code;
}

#define HIP_CHECK(ctx, call)                                                               \
  do {                                                                                     \
    hipError_t e_ = (call);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return set_err(ctx, CSM_E_HIP, "%s: %s", #call, hipGetErrorString(e_));              \
  } while (0)

#define LAUNCH_CHECK(ctx, name)                                                            \
  do {                                                                                     \
    hipError_t e_ = hipGetLastError();                                                     \
    if (e_ != hipSuccess) return set_err(ctx, CSM_E_HIP, "%s launch: %s", name, hipGetErrorString(e_)); \
  } while (0)

static inline int prep(csm_ctx* c) {
  if (!c) return CSM_E_INVAL;
  c->err[0] = 0;
  HIP_CHECK(c, hipSetDevice(c->device));
  return CSM_OK;
}

static inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// Whether the context's stream is being captured into a hipGraph.  Context-owned buffers are
// baked into a captured graph by address, so they are never (re)allocated while capturing.
static inline bool capturing(csm_ctx* c) {
  hipStreamCaptureStatus s = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(c->stream, &s) == hipSuccess && s != hipStreamCaptureStatusNone;
}

// Device counters / flags the library resets before a launch that accumulates into them are
// zeroed by a kernel, not by hipMemsetAsync: a kernel node replays the same way in a captured
// graph as eagerly (the turnover work-list counter, the boot-scan domain flag).
static __global__ void k_zero_i32(int32_t* __restrict__ p, int n) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i < n) p[i] = 0;
}
static inline hipError_t zero_i32_async(int32_t* p, int n, hipStream_t st) {
  hipLaunchKernelGGL(k_zero_i32, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, p, n);
  return hipGetLastError();
}

// ---- shared by the decile kernels (csmom.hip and deciles_narrow.hip) -------------------------
#define MAXQ 21  // n_bins + 1 <= 21
#define MAXT 42  // distinct target ranks (2 per interior quantile + min + max)
// Phase timestamps (profiling aid, csm_tune_ptr("dec_timing", buf)): per date row, wall-clock
// ticks at DEC_NPH phase boundaries, written by thread 0 when the pointer is set.
#define DEC_NPH 9
__device__ __forceinline__ void dec_mark(int64_t* tim, int t, int ph) {
  if (tim && threadIdx.x == 0) tim[(int64_t)t * DEC_NPH + ph] = (int64_t)wall_clock64();
}
struct QTab {
  double q[MAXQ];
  // legs mode (csm_deciles_ids_legs; labels-only merged pass, n_bins >= 4): only the first and
  // last decile are exact -- every other ranked cell gets some label in [1, n_bins - 2]
  int legs = 0;
};

// Fixed bucket map of the fused pipeline (csm_signal_ids writes one u16 id per asset-month,
// the decile pass histograms the ids instead of re-reading mom_J): y = fl(1 + x), 1024
// buckets per octave of y over [1/16, 16), clamped at both ends (x <= -15/16 -> 0, x >= 15
// -> 8191).  fl(1 + x) is monotone in x and so are the bits of a positive double, so the map is
// monotone non-decreasing: bucket order never contradicts value order, and the decile pass
// stays exact for ANY data -- the map only decides how many values share a bucket.  12-month
// momentum cross-sections (log-normal-ish in y) put ~5-10 of 100k values in a bulk bucket and
// almost none in the clamped end buckets (2048 per octave over [1/4, 4) halved the target
// buckets but left ~600-3000 values in the end buckets, whose exact min / max the pass needs);
// a row the map fits badly falls back to key-space refinement (slower, same labels).
#define CSM_FB_BUCKETS 8192
#define CSM_FB_NAN 0xFFFFu
// (bits >> 42 of the double, taken as the high word's arithmetic >> 10: the same value with
// 32-bit operations -- the id is computed for every asset-month by the VALU-bound scans)
__device__ __forceinline__ int csm_fbucket(double x) {
  const int b = __double2hiint(1.0 + x) >> 10;
  const int k = b - (0x3FB00000 >> 10);   // bits(1/16) >> 42
  return k < 0 ? 0 : (k > CSM_FB_BUCKETS - 1 ? CSM_FB_BUCKETS - 1 : k);
}
// set bits of a wave mask below this lane (v_mbcnt_lo / hi: 2 ops; the popcount of the masked
// ballot is 4)
__device__ __forceinline__ int lane_prefix(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint32_t csm_fid(double x) {
  return x == x ? (uint32_t)csm_fbucket(x) : CSM_FB_NAN;
}

// The split decile pass on ids (deciles.inc, wide rows): device workspace of the plan / sweep /
// finish launches, carved from the context's split buffer (csmom.hip dsplit_layout).  A chunk is
// a whole number of the merged pass's sweep trips (SPLIT_TRIP cells: 512 lanes x 4 groups x 4
// cells), and a sweep workgroup's lane owns the cells the merged pass's lane of that index owns
// there, so both passes sum next_ret in the same order (deciles.inc DEC_CHUNK_ORDER).
#define SPLIT_CELLS 32768   // default cells per sweep chunk (csm_tune "dec_split_cells"; the
                            // chunking depends on N and that knob only, never on the launch)
#define SPLIT_TRIP 8192     // cells of one merged-sweep trip: chunks are multiples of it
#define SPLIT_THREADS 512
#define SPLIT_WAVES (SPLIT_THREADS / 64)
#define SPLIT_FL 1024       // uncertain cells a sweep wave can list per chunk
#define DSPLAN_BYTES 4096   // one row's DsPlan
#define DSPLIT_MAXL 512     // (chunk, wave) lists per row the finish launch merges
struct DecSplit {
  char* plan;        // [T_m] DsPlan (slots, targets, ranked count)
  int8_t* tab;       // [T_m][8192] bucket -> label (-1 NaN, >= 0 certain, <= -2 uncertain)
  double* lp;        // [T_m][C][MAXQ - 1][SPLIT_THREADS] each lane's certain-cell next_ret sum
                     //   per label, per chunk (the merged pass's per-lane chunk partials)
  int32_t* pc;       // [T_m][C][MAXQ] certain-cell counts per label, per chunk
  int32_t* ucnt;     // [T_m][C][SPLIT_WAVES] uncertain cells listed per (chunk, wave)
  uint32_t* ulist;   // [T_m][C][SPLIT_WAVES][SPLIT_FL] their cell indices
  int C;             // chunks per row: ceil(N / cells)
  int64_t cells;     // cells per chunk (a multiple of SPLIT_TRIP)
  int pf;            // the sweep's prefetching variant (no more (chunk, date) pairs than CUs)
};

// narrow-row decile launcher (deciles_narrow.hip), NB in {0,2,3,4,5,10,20}
template <int NB>
void launch_deciles_narrow(bool v2, int T_m, hipStream_t st, const double* M, const double* NR,
                           int64_t N, int nbins, const QTab& q, int8_t* L, double* EW,
                           int32_t* CNT, int32_t* NV, int64_t* tim);

// fused-pipeline decile launcher on the bucket ids of csm_signal_ids (deciles_pre.hip),
// NB in {0,2,3,4,5,10,20}.  flg (T_m ints) non-NULL: the merged kernel first, then the general
// kernel for the rows it left (flg[t] = 1); NULL: the general kernel only.  LS non-NULL (NB > 0,
// with the context's ticket): the long-short by the general launch's last workgroup
template <int NB>
void launch_deciles_pre(int T_m, hipStream_t st, const double* M, const double* NR, int64_t N,
                        int nbins, const QTab& q, int8_t* L, double* EW, int32_t* CNT,
                        int32_t* NV, int64_t* tim, uint16_t* ids, int32_t* flg, double* LS,
                        int32_t* ticket, int64_t cells);

// the split pass (plan, chunked sweep, finish + the general path for the rows it leaves) on
// wide rows of short date shards; flg (T_m ints) required
template <int NB>
void launch_deciles_split(int T_m, hipStream_t st, const double* M, const double* NR, int64_t N,
                          int nbins, const QTab& q, int8_t* L, double* EW, int32_t* CNT,
                          int32_t* NV, int64_t* tim, uint16_t* ids, int32_t* flg,
                          const DecSplit& sp, double* LS, int32_t* ticket);

// the same on narrow rows (deciles_npre.hip: 2048 buckets = the fixed map's ids >> 2); flg
// non-NULL with decile sums: ONE launch, a row the merged pass gives up taking the general path
// in the same workgroup
template <int NB>
void launch_deciles_pre_narrow(int T_m, hipStream_t st, const double* M, const double* NR,
                               int64_t N, int nbins, const QTab& q, int8_t* L, double* EW,
                               int32_t* CNT, int32_t* NV, int64_t* tim, uint16_t* ids,
                               int32_t* flg, double* LS, int32_t* ticket);
