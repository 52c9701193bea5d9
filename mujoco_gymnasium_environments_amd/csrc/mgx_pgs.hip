// mgx_pgs.hip — the kernels of the staged soccer step (mgx_staged.h) in one translation unit:
// S1 k_soccer_rows, S2 k_pgs_groups, S3 k_soccer_finish, and k_soccer_settle, which runs the same
// three stages in one wave for reset() and for resets whose bank was not ready. One TU and one
// set of flags for all of them, so the settle and the pipeline share their machine arithmetic
// (a bank-installed reset is bit-identical to the fallback; tests/test_gpu_staged.py).
// Compiled without SLP vectorization (native.py): the SLP pass packs the solver's v += B'dl FMA
// chains into v_pk_fma with register-repacking moves, and the extra register traffic made the
// prefetch ring wait on its own loads (measured: 188 -> 139 instructions per 4-row block, no
// vmcnt(0) inside the sweep).
#include "mgx_internal.h"

namespace mgx {

// lanes per slot of the solver kernels: MGX_PGS_LPS (compile-time default) or the MGX_PGS_LPS
// environment variable (16 or 64), for A/B runs. Read once per process: the settle and solver
// kernels' dynamic-LDS limits are set at model creation from this value, so it must not change
// between configure and launch.
int pgs_lanes() {
  static const int lanes = [] {
    const char* v = getenv("MGX_PGS_LPS");
    const int x = v ? atoi(v) : MGX_PGS_LPS;
    return x == 64 ? 64 : 16;
  }();
  return lanes;
}
template <typename T, int LPS, bool BLDS, bool SQG = false>
static void launch_lps(const Pipe& P, int slots, int lds, hipStream_t st, int maxit, T tol, T scale, int big,
                       int spw_hook, int spw_force = 0) {
  const int spw = spw_force ? spw_force : spw_hook ? spw_hook : 64 / LPS;  // spw_hook: MGX_PGS_SPW (debug)
  int grid = (slots + (spw < 0 ? -spw : spw) - 1) / (spw < 0 ? -spw : spw);
  switch ((P.dpl + LPS / 8 - 1) / (LPS / 8)) {  // register entries per lane
#define MGX_PGS_CASE(E)                                                                                          \
    case E:                                                                                                     \
      hipLaunchKernelGGL((k_pgs_groups<T, E, LPS, BLDS, SQG>), dim3(grid), dim3(64), lds, st, P, maxit, tol, scale, spw, \
                         big);                                                                                  \
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
void launch_pgs(const Pipe& P, int slots, int lds, hipStream_t st, int maxit, T tol, T scale, int big, const Hooks& h) {
  if (big && P.warena > 0 && pgs_lanes() == 16) {
    // the wide launch with LDS-resident B: one slot per wave (all four lane groups on it), a
    // small grid striding over the few slots past the main launch's rows
    launch_lps<T, 16, true>(P, MGX_PGS_WIDE_LDS_GRID, P.warena + 64, st, maxit, tol, scale, big, h.pgs_spw, 1);
    return;
  }
  const bool blds = !big && h.pgs_lds_b;  // the main launch with B in an LDS arena (MGX_PGS_LDS_B)
  const int sp = h.pgs_spw;
  if (pgs_lanes() == 64) {
    if (blds) launch_lps<T, 64, true>(P, slots, lds, st, maxit, tol, scale, big, sp);
    else launch_lps<T, 64, false>(P, slots, lds, st, maxit, tol, scale, big, sp);
  } else {
    if (blds) launch_lps<T, 16, true>(P, slots, lds, st, maxit, tol, scale, big, sp);
    else if (P.sqg && !big) launch_lps<T, 16, false, true>(P, slots, lds, st, maxit, tol, scale, big, sp);
    else launch_lps<T, 16, false>(P, slots, lds, st, maxit, tol, scale, big, sp);
  }
}
template void launch_pgs<float>(const Pipe&, int, int, hipStream_t, int, float, float, int, const Hooks&);
template void launch_pgs<double>(const Pipe&, int, int, hipStream_t, int, double, double, int, const Hooks&);

// ---- S1 / S3 (the row builder and the finisher)
template <typename T>
__global__ void __launch_bounds__(64) k_soccer_rows(DevModel<T> m, SoccerIds<T> ids, mgx_state s, mgx_soccer_env ev,
                                                    const float* action, int n_env, const uint8_t* mask, Pipe P,
                                                    int banks) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int b = blockIdx.x;
  int slot;
  Env<T> e;
  if (b < n_env) {
    if (mask && !mask[b]) return;
    env_bind(m, e, smem);
    bind_carry_tail(m, e, P, b);
    load_state(m, e, (T*)s.qpos, (T*)s.qvel, (T*)s.qacc_warmstart, (T*)s.ctrl, (T*)s.qfrc_applied, (T*)s.xfrc_applied,
               (T*)s.time, b);
    soccer_pre(m, e, ids, SoccerAct(action, ev.action_f64, b, m.nu), (T*)ev.prev_ball_pos + 3 * (size_t)b,
               (T*)ev.wind + 3 * (size_t)b);
    slot = b;
  } else {
    int bi = b - n_env;
    if (!banks || bi >= n_env * P.R) return;
    int k = P.at<int>(P.o_bk)[bi];
    if (k < 0 || k >= 10) return;
    env_bind(m, e, smem);
    bind_carry_tail(m, e, P, b);
    bank_load_state(m, e, P, bi);
    slot = b;
  }
  int warn = 0;  // mj_checkPos / mj_checkVel
  if (any_bad(e.qpos, m.nq)) { reset_env(m, e); warn++; }
  if (any_bad(e.qvel, m.nv)) { reset_env(m, e); warn++; }
  stage_rows(m, e, P, slot, warn);
}

// The bank slots' settle steps (S3 of the extra slots), one wave per bank record, launched before
// the live finisher: a bank that completes its tenth step here is ready for a reset in this
// step's live finisher, as when one wave finished an env's banks and then the env.
template <typename T>
__global__ void __launch_bounds__(64) k_soccer_bank_finish(DevModel<T> m, SoccerIds<T> ids, int n_env, Pipe P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int bi = blockIdx.x;
  if (bi >= n_env * P.R) return;
  int k = P.at<int>(P.o_bk)[bi];
  if (k < 0 || k >= 10) return;
  Env<T> e;
  env_bind(m, e, smem);
  const int slot = n_env + bi;
  int warn = load_carry(m, e, P, slot);
  if (!finish_physics(m, e, P, slot)) {
    load_template(m, e, P);
    warn++;
  }
  bank_store_state(m, e, P, bi, warn);
  k++;
  if (k == 10) bank_finalize(m, e, ids, P, bi);
  if (lane_id() == 0) P.at<int>(P.o_bk)[bi] = k;
}

template <typename T>
__global__ void __launch_bounds__(64) k_soccer_finish(DevModel<T> m, SoccerIds<T> ids, mgx_state s, mgx_soccer_env ev,
                                                      const float* action, float* obs, double* reward,
                                                      uint8_t* terminated, uint8_t* truncated, float* final_obs,
                                                      int autoreset, uint64_t seed, int env_offset, int n_env,
                                                      const uint8_t* mask, Pipe P, int banks) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int env = blockIdx.x;
  if (env >= n_env) return;
  int l = lane_id();
  if (env == 0 && l == 0) {  // the solver lists are consumed; their sizes stay for diagnostics
    P.ctr()[3] = P.ctr()[1];
    P.ctr()[4] = P.ctr()[2];
    P.ctr()[1] = 0;
    P.ctr()[2] = 0;
  }
  if (env == 0)
    for (int b = lane_id(); b < P.nbk; b += 64) P.at<int>(P.o_hist)[b] = 0;
  Env<T> e;
  env_bind(m, e, smem);
  if (mask && !mask[env]) return;
  int warn = load_carry(m, e, P, env);
  if (!finish_physics(m, e, P, env)) {
    load_template(m, e, P);
    warn++;
  }
  store_state(m, e, (T*)s.qpos, (T*)s.qvel, (T*)s.qacc_warmstart, (T*)s.ctrl, (T*)s.qfrc_applied, (T*)s.xfrc_applied,
              (T*)s.time, env);
  if (l == 0 && s.warning) s.warning[env] += warn;
  if (l == 0 && s.overflow && e.overflow) s.overflow[env] += 1;
  const SoccerAct a(action, ev.action_f64, env, m.nu);
  float* o = obs + (size_t)env * 80;
  bool done = soccer_post(m, e, ids, a, ev.step + env, ev.goal_scored + env, (T*)ev.prev_ball_pos + 3 * (size_t)env,
                          (T*)ev.prev_robot_pos + 3 * (size_t)env, (T*)ev.stats + 5 * (size_t)env, o, reward + env,
                          terminated + env, truncated + env, ev.flags ? ev.flags + 2 * (size_t)env : nullptr);
  if (ev.rollout && l == 0) {
    double* ro = (double*)ev.rollout + 8 * (size_t)env;
    const double ne = e.nefc, it = e.nefc > 0 ? P.at<int>(P.o_niter)[env] : 0;
    ro[0] += reward[env];
    ro[1] += terminated[env];
    ro[2] += truncated[env];
    ro[3] += 1.0;
    ro[4] += ne;
    ro[5] += it;
    ro[6] += ne * ne;
    ro[7] += it * ne * ne;
  }
  if (done && autoreset) {
    if (final_obs)
      for (int i = l; i < 80; i += 64) final_obs[(size_t)env * 80 + i] = o[i];
    __threadfence();
    wsync();
    bool ok = banks && bank_install(m, e, ids, P, s, ev, obs, seed, env_offset, env);
    if (!ok && l == 0) {
      int i = atomicAdd(P.ctr(), 1);
      P.at<int>(P.o_fix)[i] = env * 4 + FIX_RESET;
    }
  }
}


template <typename T>
void launch_soccer_rows(const DevModel<T>& Ms, const SoccerIds<T>& ids, const mgx_state& s, const mgx_soccer_env& ev,
                        const float* action, int n_env, const uint8_t* mask, const Pipe& P, int banks, int slots, int lds,
                        hipStream_t st) {
  hipLaunchKernelGGL(k_soccer_rows<T>, dim3(slots), dim3(64), lds, st, Ms, ids, s, ev, action, n_env, mask, P, banks);
}
template <typename T>
void launch_soccer_finish(const DevModel<T>& Mf, const SoccerIds<T>& ids, const mgx_state& s, const mgx_soccer_env& ev,
                          const float* action, float* obs, double* reward, uint8_t* terminated, uint8_t* truncated,
                          float* final_obs, int autoreset, uint64_t seed, int env_offset, int n_env, const uint8_t* mask,
                          const Pipe& P, int banks, int lds, hipStream_t st) {
  if (banks && P.R > 0)
    hipLaunchKernelGGL(k_soccer_bank_finish<T>, dim3(n_env * P.R), dim3(64), lds, st, Mf, ids, n_env, P);
  hipLaunchKernelGGL(k_soccer_finish<T>, dim3(n_env), dim3(64), lds, st, Mf, ids, s, ev, action, obs, reward, terminated,
                     truncated, final_obs, autoreset, seed, env_offset, n_env, mask, P, banks);
}
// the settle kernel takes the main solver launch's lanes per slot and register entries per lane
// (launch_lps), so its PGS is the pipeline's
template <typename T>
void launch_soccer_settle(const DevModel<T>& Ms, const DevModel<T>& Mf, const SoccerIds<T>& ids, const mgx_state& s,
                          const mgx_soccer_env& ev, const T* draws, float* obs, uint64_t seed, int env_offset, int n_env,
                          const uint8_t* mask, const Pipe& P, int mode, int grid, int lds, hipStream_t st, int maxit, T tol,
                          T scale) {
#define MGX_SETTLE(E, L)                                                                                            \
  hipLaunchKernelGGL((k_soccer_settle<T, E, L>), dim3(grid), dim3(64), lds, st, Ms, Mf, ids, s, ev, draws, obs, seed, \
                     env_offset, n_env, mask, P, mode, maxit, tol, scale)
  if (pgs_lanes() == 64) {
    MGX_SETTLE(1, 64);
  } else {
    switch ((P.dpl + 1) / 2) {
      case 1: MGX_SETTLE(1, 16); break;
      case 2: MGX_SETTLE(2, 16); break;
      case 3: MGX_SETTLE(3, 16); break;
      default: MGX_SETTLE(4, 16); break;
    }
  }
#undef MGX_SETTLE
}
#define MGX_STAGED_INST(T)                                                                                              \
  template void launch_soccer_rows<T>(const DevModel<T>&, const SoccerIds<T>&, const mgx_state&, const mgx_soccer_env&, \
                                      const float*, int, const uint8_t*, const Pipe&, int, int, int, hipStream_t);      \
  template void launch_soccer_finish<T>(const DevModel<T>&, const SoccerIds<T>&, const mgx_state&,                      \
                                        const mgx_soccer_env&, const float*, float*, double*, uint8_t*, uint8_t*, float*, \
                                        int, uint64_t, int, int, const uint8_t*, const Pipe&, int, int, hipStream_t);     \
  template void launch_soccer_settle<T>(const DevModel<T>&, const DevModel<T>&, const SoccerIds<T>&, const mgx_state&, \
                                        const mgx_soccer_env&, const T*, float*, uint64_t, int, int, const uint8_t*,    \
                                        const Pipe&, int, int, int, hipStream_t, int, T, T);
MGX_STAGED_INST(float)
MGX_STAGED_INST(double)
#undef MGX_STAGED_INST

// dynamic-LDS attributes of the row builder, finisher and settle kernels
int staged_kernels_configure(int precision, int ls, int lf, int settle) {
  int rc = 0;
#define MGX_SETTLE_SET(T) \
  rc |= mgx_set_lds(k_soccer_settle<T, 1, 16>, settle) | mgx_set_lds(k_soccer_settle<T, 2, 16>, settle) | \
        mgx_set_lds(k_soccer_settle<T, 3, 16>, settle) | mgx_set_lds(k_soccer_settle<T, 4, 16>, settle) | \
        mgx_set_lds(k_soccer_settle<T, 1, 64>, settle);
  if (precision == MGX_F32) {
    rc |= mgx_set_lds(k_soccer_rows<float>, ls > 64 * 1024 ? ls : 64 * 1024) | mgx_set_lds(k_soccer_finish<float>, lf) |
          mgx_set_lds(k_soccer_bank_finish<float>, lf);
    MGX_SETTLE_SET(float)
  } else {
    rc |= mgx_set_lds(k_soccer_rows<double>, ls > 64 * 1024 ? ls : 64 * 1024) | mgx_set_lds(k_soccer_finish<double>, lf) |
          mgx_set_lds(k_soccer_bank_finish<double>, lf);
    MGX_SETTLE_SET(double)
  }
#undef MGX_SETTLE_SET
  return rc;
}

int pgs_configure_lds(int precision, int pl, int wl) {
  int rc = 0;
#define MGX_PGS_SET(T, E, L)                                                                            \
  rc |= mgx_set_lds(k_pgs_groups<T, E, L, true>, pl > wl ? pl : wl) | mgx_set_lds(k_pgs_groups<T, E, L, false>, pl) | \
        mgx_set_lds(k_pgs_groups<T, E, L, false, true>, pl);
#define MGX_PGS_SET_ALL(T) \
  MGX_PGS_SET(T, 1, 16) MGX_PGS_SET(T, 2, 16) MGX_PGS_SET(T, 3, 16) MGX_PGS_SET(T, 4, 16) MGX_PGS_SET(T, 1, 64)
  if (precision == MGX_F32) { MGX_PGS_SET_ALL(float) } else { MGX_PGS_SET_ALL(double) }
#undef MGX_PGS_SET_ALL
#undef MGX_PGS_SET
  return rc;
}

}  // namespace mgx

MGX_PROF_SETTER(mgx_prof_set_buffer_pgs)
