// deciles_wave.hip -- the per-date qcut kernel with ONE WAVE per row, for the narrowest rows
// (the C5 bootstrap batches: 30k rows of 5k assets per launch).  Same algorithm and results as
// the wide- and narrow-row kernels (csrc/deciles.inc); a single-wave workgroup's barriers are
// free, and 1024 buckets + 512 candidates (~11 KB of LDS) let 14 rows share a CU, so the
// per-row serial phases of different rows overlap instead of running in lockstep.
#include "csm_common.h"

#define DEC_THREADS 64
#define HB 1024
#define CAP 512      // candidates of the target buckets (refinement splits beyond)
#define DEC_MINB 3   // 3 waves per SIMD (LDS allows ~10 of these workgroups per CU)
#define DEC_SCH 16   // a 1024-value range sample (16 per lane)
namespace dec_wave {
#include "deciles.inc"
}  // namespace dec_wave

template <int NB>
void launch_deciles_wave(bool v2, int T_m, hipStream_t st, const double* M, const double* NR,
                         int64_t N, int nbins, const QTab& q, int8_t* L, double* EW,
                         int32_t* CNT, int32_t* NV, int ablate, int64_t* tim) {
  uint16_t* ids = nullptr;
  if (v2)
    hipLaunchKernelGGL((dec_wave::k_deciles<NB, true, false>), dim3(T_m), dim3(DEC_THREADS), 0,
                       st, M, NR, N, nbins, q, L, EW, CNT, NV, ablate, tim, ids);
  else
    hipLaunchKernelGGL((dec_wave::k_deciles<NB, false, false>), dim3(T_m), dim3(DEC_THREADS), 0,
                       st, M, NR, N, nbins, q, L, EW, CNT, NV, ablate, tim, ids);
}

#define INST(NB)                                                                              \
  template void launch_deciles_wave<NB>(bool, int, hipStream_t, const double*, const double*,    \
                                        int64_t, int, const QTab&, int8_t*, double*, int32_t*,   \
                                        int32_t*, int, int64_t*);
INST(0)
INST(2)
INST(3)
INST(4)
INST(5)
INST(10)
INST(20)
#undef INST
