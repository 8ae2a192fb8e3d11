// deciles_pre.hip -- the per-date qcut kernel of the fused pipeline (csm_deciles_ids /
// csm_pipeline): the wide-row kernel of csrc/deciles.inc in PRE mode, reading the fixed-map
// bucket ids csm_signal_ids wrote (M is read only for the few cells near a bin edge).  Its own
// translation unit so the kernel builds in parallel with csmom.hip.
#include "csm_common.h"

// (overridable for same-box A/B builds: -DDEC_PRE_THREADS=256 -DDEC_PRE_HB=4096 ...)
#ifndef DEC_PRE_THREADS
#define DEC_PRE_THREADS 512
#endif
#ifndef DEC_PRE_HB
#define DEC_PRE_HB 8192
#endif
#ifndef DEC_PRE_CAP
#define DEC_PRE_CAP 4096
#endif
#define DEC_THREADS DEC_PRE_THREADS
#define HB DEC_PRE_HB
#define CAP DEC_PRE_CAP
#define DEC_LU 8
#define DEC_CHUNK_ORDER 1   // merged pass summed in the split pass's order (deciles.inc)
namespace dec_pre {
#include "deciles.inc"
}  // namespace dec_pre

template <int NB>
void launch_deciles_pre(int T_m, hipStream_t st, const double* M, const double* NR, int64_t N,
                        int nbins, const QTab& q, int8_t* L, double* EW, int32_t* CNT,
                        int32_t* NV, int64_t* tim, uint16_t* ids, int32_t* flg, double* LS,
                        int32_t* ticket, int64_t cells) {
  // merged pass first (flg): one sweep of ids + next_ret per row (deciles.inc, MG); then the
  // general kernel takes the rows it left (all rows without flg) -- and, LS given, its last
  // workgroup forms the long-short (csmom.hip launches k_long_short instead for these rows).
  // (The merged pass with the general path as an in-workgroup fallback needs more than the 128
  // VGPRs of two 512-thread workgroups per CU at this width.)
  // (the merged pass sums in the split pass's order: its chunks of `cells` cells)
  if (flg) {
    DecSplit sp{};
    sp.cells = cells;
    hipLaunchKernelGGL((dec_pre::k_deciles<NB, true, true, true>), dim3(T_m),
                       dim3(DEC_THREADS), 0, st, M, NR, N, nbins, q, L, EW, CNT, NV, tim,
                       ids, flg, (double*)nullptr, (int32_t*)nullptr, sp);
  }
  hipLaunchKernelGGL((dec_pre::k_deciles<NB, true, true, false>), dim3(T_m),
                     dim3(DEC_THREADS), 0, st, M, NR, N, nbins, q, L, EW, CNT, NV, tim,
                     ids, flg, LS, ticket);
}

// the split pass: plan -> chunked sweep -> finish (+ the general kernel for the rows the plan or
// a sweep chunk left, FLG = 1) -- deciles.inc's split section
template <int NB>
void launch_deciles_split(int T_m, hipStream_t st, const double* M, const double* NR, int64_t N,
                          int nbins, const QTab& q, int8_t* L, double* EW, int32_t* CNT,
                          int32_t* NV, int64_t* tim, uint16_t* ids, int32_t* flg,
                          const DecSplit& sp, double* LS, int32_t* ticket) {
  hipLaunchKernelGGL((dec_pre::k_deciles<NB, true, true, true, false, 1>), dim3(T_m),
                     dim3(DEC_THREADS), 0, st, M, NR, N, nbins, q, L, EW, CNT, NV, tim, ids, flg,
                     (double*)nullptr, (int32_t*)nullptr, sp);
  if (sp.pf)
    hipLaunchKernelGGL((dec_pre::k_dsplit_sweep<NB, true>), dim3((unsigned)sp.C, (unsigned)T_m),
                       dim3(SPLIT_THREADS), 0, st, NR, (const uint16_t*)ids, N, L, flg, sp);
  else
    hipLaunchKernelGGL((dec_pre::k_dsplit_sweep<NB, false>), dim3((unsigned)sp.C, (unsigned)T_m),
                       dim3(SPLIT_THREADS), 0, st, NR, (const uint16_t*)ids, N, L, flg, sp);
  // the finish launch: the listed cells of the rows the plan and sweep took, the general path
  // for the rows they left; LS given, its last workgroup forms the long-short
  hipLaunchKernelGGL((dec_pre::k_deciles<NB, true, true, false, false, 2>), dim3(T_m),
                     dim3(DEC_THREADS), 0, st, M, NR, N, nbins, q, L, EW, CNT, NV, tim, ids, flg,
                     LS, ticket, sp);
}

#define INST(NB)                                                                              \
  template void launch_deciles_split<NB>(int, hipStream_t, const double*, const double*,        \
                                         int64_t, int, const QTab&, int8_t*, double*, int32_t*, \
                                         int32_t*, int64_t*, uint16_t*, int32_t*,              \
                                         const DecSplit&, double*, int32_t*);                 \
  template void launch_deciles_pre<NB>(int, hipStream_t, const double*, const double*, int64_t, \
                                       int, const QTab&, int8_t*, double*, int32_t*, int32_t*,  \
                                       int64_t*, uint16_t*, int32_t*, double*, int32_t*, int64_t);
INST(0)
INST(2)
INST(3)
INST(4)
INST(5)
INST(10)
INST(20)
#undef INST
