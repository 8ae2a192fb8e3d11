// deciles_npre.hip -- the sweeps' decile pass on bucket ids (csm_momentum_multi_ids ->
// csm_deciles_ids on rows of <= dec_narrow_max assets): the narrow-row kernel of
// csrc/deciles.inc in PRE mode with 2048 buckets (the fixed map's ids >> 2).  Finer than the
// streaming narrow kernel's 1024 so that fewer cells share an edge's bucket: each of those costs
// a scattered 8-B read of mom_J (a cache line of HBM traffic).  Own translation unit: builds in
// parallel with the others.
#include "csm_common.h"

#define DEC_THREADS 256
#define HB 2048
#define CAP 512
#define DEC_MINB 4   // the general kernel and the merged pass with decile sums: no spills
#define DEC_MINB_MG0 8   // labels-only merged pass: 59 VGPRs, 20 KB LDS -> 8 workgroups per CU
namespace dec_npre {
#include "deciles.inc"
}  // namespace dec_npre

// the fused sweep path on bucket ids (csm_momentum_multi_ids -> csm_deciles_ids on rows of
// <= dec_narrow_max assets): merged pass, then the general PRE kernel for the rows it leaves
template <int NB>
void launch_deciles_pre_narrow(int T_m, hipStream_t st, const double* M, const double* NR,
                               int64_t N, int nbins, const QTab& q, int8_t* L, double* EW,
                               int32_t* CNT, int32_t* NV, int64_t* tim,
                               uint16_t* ids, int32_t* flg, double* LS,
                               int32_t* ticket) {
  // with decile sums (C2): ONE launch -- a row the merged pass gives up takes the general path
  // in the same workgroup, and LS (with the context's ticket) is formed by the last workgroup.
  // Labels only (the sweeps, NB = 0): the merged kernel keeps its 8 workgroups per CU only
  // without the general path beside it (64 VGPRs; with it the kernel spills), so the general
  // kernel follows as its own launch for the rows the merged pass left (flg[t] = 1).
  if constexpr (NB > 0) {
    if (flg) {
      hipLaunchKernelGGL((dec_npre::k_deciles<NB, true, true, true, true>), dim3(T_m),
                         dim3(DEC_THREADS), 0, st, M, NR, N, nbins, q, L, EW, CNT, NV, tim,
                         ids, (int32_t*)nullptr, LS, ticket);
      return;
    }
  }
  if (flg)
    hipLaunchKernelGGL((dec_npre::k_deciles<NB, true, true, true>), dim3(T_m),
                       dim3(DEC_THREADS), 0, st, M, NR, N, nbins, q, L, EW, CNT, NV, tim,
                       ids, flg, (double*)nullptr, (int32_t*)nullptr);
  hipLaunchKernelGGL((dec_npre::k_deciles<NB, true, true, false>), dim3(T_m),
                     dim3(DEC_THREADS), 0, st, M, NR, N, nbins, q, L, EW, CNT, NV, tim,
                     ids, flg, LS, ticket);
}

#define INST(NB)                                                                              \
  template void launch_deciles_pre_narrow<NB>(int, hipStream_t, const double*, const double*,  \
                                              int64_t, int, const QTab&, int8_t*, double*,       \
                                              int32_t*, int32_t*, int64_t*, uint16_t*,       \
                                              int32_t*, double*, int32_t*);
INST(0)
INST(2)
INST(3)
INST(4)
INST(5)
INST(10)
INST(20)
#undef INST
