// deciles_reg.hip -- the wide-row qcut kernel (csrc/deciles.inc, 512 threads, 8192 buckets)
// with register-resident bucket ids (RI mode): each lane keeps the 16-bit bucket id of its
// 4 x RI cells from the histogram pass to the label pass, so the row of M is streamed from
// HBM once instead of three times (the gather and label passes re-read only the cells of
// target / edge buckets).  Rows with N even and N <= 1.25 x RI * 2048 (C4: 100k assets,
// 94208 cells in registers + a 5792-cell tail).  Bit-identical to the plain wide kernel.
#include "csm_common.h"

#define DEC_THREADS 512
#define HB 8192
#define CAP 4096
namespace dec_reg {
#include "deciles.inc"
}  // namespace dec_reg

// rows up to 1.25 x the register range (the tail cells are re-read like the plain kernel)
int deciles_reg_max_n() { return DEC_REG_RI * 4 * DEC_THREADS * 5 / 4; }

template <int NB>
void launch_deciles_reg(int T_m, hipStream_t st, const double* M, const double* NR, int64_t N,
                        int nbins, const QTab& q, int8_t* L, double* EW, int32_t* CNT,
                        int32_t* NV, int ablate, int64_t* tim) {
  hipLaunchKernelGGL((dec_reg::k_deciles<NB, true, false, DEC_REG_RI>), dim3(T_m),
                     dim3(DEC_THREADS), 0, st, M, NR, N, nbins, q, L, EW, CNT, NV, ablate, tim,
                     (uint16_t*)nullptr);
}

#define INST(NB)                                                                              \
  template void launch_deciles_reg<NB>(int, hipStream_t, const double*, const double*, int64_t, \
                                       int, const QTab&, int8_t*, double*, int32_t*, int32_t*,  \
                                       int, int64_t*);
INST(0)
INST(2)
INST(3)
INST(4)
INST(5)
INST(10)
INST(20)
#undef INST
