// mgx_pgs.hip — S2 of the staged soccer step (k_pgs_groups, mgx_staged.h) in its own translation
// unit. It is compiled without SLP vectorization (native.py): the SLP pass packs the solver's
// v += B'dl FMA chains into v_pk_fma with register-repacking moves, and the extra register
// traffic made the prefetch ring wait on its own loads (measured: 188 -> 139 instructions per
// 4-row block, no vmcnt(0) inside the sweep).
#include "mgx_internal.h"

namespace mgx {

template <typename T>
void launch_pgs(const Pipe& P, int slots, int lds, hipStream_t st, int maxit, T tol, T scale, int big) {
  static const int spw = getenv("MGX_PGS_SPW") ? atoi(getenv("MGX_PGS_SPW")) : MGX_PGS_SPW;  // debug: slots per wave
  int grid = (slots + (spw < 0 ? -spw : spw) - 1) / (spw < 0 ? -spw : spw);
  switch ((P.dpl + MGX_PGS_LPS / 8 - 1) / (MGX_PGS_LPS / 8)) {  // register entries per lane
#define MGX_PGS_CASE(E) \
    case E: hipLaunchKernelGGL((k_pgs_groups<T, E>), dim3(grid), dim3(64), lds, st, P, maxit, tol, scale, spw, big); break;
    MGX_PGS_CASE(1) MGX_PGS_CASE(2) MGX_PGS_CASE(3) MGX_PGS_CASE(4) MGX_PGS_CASE(5) MGX_PGS_CASE(6) MGX_PGS_CASE(7)
    default: hipLaunchKernelGGL((k_pgs_groups<T, 8>), dim3(grid), dim3(64), lds, st, P, maxit, tol, scale, spw, big); break;
#undef MGX_PGS_CASE
  }
}
template void launch_pgs<float>(const Pipe&, int, int, hipStream_t, int, float, float, int);
template void launch_pgs<double>(const Pipe&, int, int, hipStream_t, int, double, double, int);

int pgs_configure_lds(int precision, int pl) {
  if (precision == MGX_F32)
    return mgx_set_lds(k_pgs_groups<float, 1>, pl) | mgx_set_lds(k_pgs_groups<float, 2>, pl) |
           mgx_set_lds(k_pgs_groups<float, 3>, pl) | mgx_set_lds(k_pgs_groups<float, 4>, pl) |
           mgx_set_lds(k_pgs_groups<float, 5>, pl) | mgx_set_lds(k_pgs_groups<float, 6>, pl) |
           mgx_set_lds(k_pgs_groups<float, 7>, pl) | mgx_set_lds(k_pgs_groups<float, 8>, pl);
  return mgx_set_lds(k_pgs_groups<double, 1>, pl) | mgx_set_lds(k_pgs_groups<double, 2>, pl) |
         mgx_set_lds(k_pgs_groups<double, 3>, pl) | mgx_set_lds(k_pgs_groups<double, 4>, pl) |
         mgx_set_lds(k_pgs_groups<double, 5>, pl) | mgx_set_lds(k_pgs_groups<double, 6>, pl) |
         mgx_set_lds(k_pgs_groups<double, 7>, pl) | mgx_set_lds(k_pgs_groups<double, 8>, pl);
}

}  // namespace mgx

MGX_PROF_SETTER(mgx_prof_set_buffer_pgs)
