// deciles_narrow.hip -- the per-date qcut kernel for rows of a few thousand assets (C2 / C3
// and the C5 bootstrap batches: 30k rows of 5k assets per launch).  Same algorithm and results
// as the wide-row kernel (csrc/deciles.inc); 256 threads, 1024 buckets and 1024 candidates
// use a quarter of its LDS, so four times as many rows are in flight per CU -- the per-row
// serial phases (range, targets, selection, edges) dominate at this width.
#include "csm_common.h"

#define DEC_THREADS 256
#define HB 1024
#define CAP 1024     // candidates of the target buckets (refinement splits beyond)
#define DEC_MINB 6   // 6 workgroups per CU (8: register spills, slower)
namespace dec_narrow {
#include "deciles.inc"
}  // namespace dec_narrow

template <int NB>
void launch_deciles_narrow(bool v2, int T_m, hipStream_t st, const double* M, const double* NR,
                           int64_t N, int nbins, const QTab& q, int8_t* L, double* EW,
                           int32_t* CNT, int32_t* NV, int64_t* tim) {
  uint16_t* ids = nullptr;
  if (v2)
    hipLaunchKernelGGL((dec_narrow::k_deciles<NB, true, false>), dim3(T_m), dim3(DEC_THREADS), 0,
                       st, M, NR, N, nbins, q, L, EW, CNT, NV, tim, ids);
  else
    hipLaunchKernelGGL((dec_narrow::k_deciles<NB, false, false>), dim3(T_m), dim3(DEC_THREADS), 0,
                       st, M, NR, N, nbins, q, L, EW, CNT, NV, tim, ids);
}

#define INST(NB)                                                                              \
  template void launch_deciles_narrow<NB>(bool, int, hipStream_t, const double*, const double*,  \
                                          int64_t, int, const QTab&, int8_t*, double*,           \
                                          int32_t*, int32_t*, int64_t*);
INST(0)
INST(2)
INST(3)
INST(4)
INST(5)
INST(10)
INST(20)
#undef INST
