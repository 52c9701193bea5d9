// mgx_pgs.hip — S2 of the staged soccer step (k_pgs_groups, mgx_staged.h) in its own translation
// unit. It is compiled without SLP vectorization (native.py): the SLP pass packs the solver's
// v += B'dl FMA chains into v_pk_fma with register-repacking moves, and the extra register
// traffic made the prefetch ring wait on its own loads (measured: 188 -> 139 instructions per
// 4-row block, no vmcnt(0) inside the sweep).
#include "mgx_internal.h"

namespace mgx {

// lanes per slot of the solver kernels: MGX_PGS_LPS (compile-time default) or the MGX_PGS_LPS
// environment variable (16 or 64), read per call like the other solver hooks, for A/B runs
int pgs_lanes() {
  const char* v = getenv("MGX_PGS_LPS");
  const int x = v ? atoi(v) : MGX_PGS_LPS;
  return x == 64 ? 64 : 16;
}
// main launch with B in an LDS arena (1) or read from global memory (0): MGX_PGS_LDS_B
// (compile-time default) or the environment variable of that name, read per call
int pgs_lds_b() {
  const char* e = getenv("MGX_PGS_LDS_B");
  return e ? (atoi(e) != 0) : MGX_PGS_LDS_B;
}

template <typename T, int LPS, bool BLDS>
static void launch_lps(const Pipe& P, int slots, int lds, hipStream_t st, int maxit, T tol, T scale, int big) {
  static const int spw_env = getenv("MGX_PGS_SPW") ? atoi(getenv("MGX_PGS_SPW")) : 0;  // debug: slots per wave
  const int spw = spw_env ? spw_env : 64 / LPS;
  int grid = (slots + (spw < 0 ? -spw : spw) - 1) / (spw < 0 ? -spw : spw);
  switch ((P.dpl + LPS / 8 - 1) / (LPS / 8)) {  // register entries per lane
#define MGX_PGS_CASE(E)                                                                                          \
    case E:                                                                                                     \
      hipLaunchKernelGGL((k_pgs_groups<T, E, LPS, BLDS>), dim3(grid), dim3(64), lds, st, P, maxit, tol, scale, spw, big); \
      break;
    MGX_PGS_CASE(1)
    default:
      if constexpr (LPS == 16) {
        switch ((P.dpl + 1) / 2) { MGX_PGS_CASE(2) MGX_PGS_CASE(3) MGX_PGS_CASE(4) default: break; }
      }
      break;  // nv <= 64
#undef MGX_PGS_CASE
  }
}

template <typename T>
void launch_pgs(const Pipe& P, int slots, int lds, hipStream_t st, int maxit, T tol, T scale, int big) {
  const bool blds = !big && pgs_lds_b();
  if (pgs_lanes() == 64) {
    if (blds) launch_lps<T, 64, true>(P, slots, lds, st, maxit, tol, scale, big);
    else launch_lps<T, 64, false>(P, slots, lds, st, maxit, tol, scale, big);
  } else {
    if (blds) launch_lps<T, 16, true>(P, slots, lds, st, maxit, tol, scale, big);
    else launch_lps<T, 16, false>(P, slots, lds, st, maxit, tol, scale, big);
  }
}
template void launch_pgs<float>(const Pipe&, int, int, hipStream_t, int, float, float, int);
template void launch_pgs<double>(const Pipe&, int, int, hipStream_t, int, double, double, int);

int pgs_configure_lds(int precision, int pl) {
  int rc = 0;
#define MGX_PGS_SET(T, E, L) rc |= mgx_set_lds(k_pgs_groups<T, E, L, true>, pl) | mgx_set_lds(k_pgs_groups<T, E, L, false>, pl);
#define MGX_PGS_SET_ALL(T) \
  MGX_PGS_SET(T, 1, 16) MGX_PGS_SET(T, 2, 16) MGX_PGS_SET(T, 3, 16) MGX_PGS_SET(T, 4, 16) MGX_PGS_SET(T, 1, 64)
  if (precision == MGX_F32) { MGX_PGS_SET_ALL(float) } else { MGX_PGS_SET_ALL(double) }
#undef MGX_PGS_SET_ALL
#undef MGX_PGS_SET
  return rc;
}

}  // namespace mgx

MGX_PROF_SETTER(mgx_prof_set_buffer_pgs)
