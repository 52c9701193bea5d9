// mgx_construction.hip — humanoid_construction kernels, the generic wide-model physics kernels
// and their C-ABI (include/mgx.h).
//
// humanoid_construction has nv = 99 (a free humanoid, a 3-dof crane, ten free blocks), beyond
// the one-dof-per-lane execution model of every other task. Its kernels run the wide physics of
// mgx_wide.h: still one 64-thread workgroup (= one wavefront) per environment, two dofs per
// lane. A construction env step is clip -> ctrl -> one RK4 mj_step (Newton) -> progress /
// reward / termination / observation, with same-step autoreset (mj_resetData + draws, no
// forward pass), all in one launch. The rows B live in per-env global scratch.
#define MGX_TEAM  // kernels with a Newton helper wave (lane_id, team_begin)
#include "mgx_internal.h"

using namespace mgx;

MGX_PROF_SETTER(mgx_prof_set_buffer_construction)

namespace {

int fail(int code, const std::string& msg) { return host_fail(code, msg); }

template <typename T>
__device__ __forceinline__ void bind(const DevModel<T>& m, WEnv<T>& w, char* smem, const mgx_state& s, int env) {
  wenv_bind<T>(m, w, smem, (T*)s.scratch + (size_t)env * m.L.gB_stride);
}

// MODE 0: one env step (+ same-step autoreset), four waves per env (wave 0 + the Newton helper
// waves, mgx_wide.h team_helper); MODE 1: reset (host draws or Philox), one wave
constexpr int kTeamThreads = 128;  // two waves: the kernel needs all 512 registers of a wave (one wave per SIMD)
template <typename T, int MODE>
__global__ void __launch_bounds__(MODE == 0 ? kTeamThreads : 64) k_construction(DevModel<T> m, ConstructionIds ids, mgx_state s,
                                                     mgx_construction_env ce, const float* action, const T* draws,
                                                     float* obs, double* reward, uint8_t* terminated,
                                                     uint8_t* truncated, float* final_obs, int autoreset,
                                                     uint64_t seed, int env_offset, int n_env, const uint8_t* mask) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int env = blockIdx.x;
  if (env >= n_env) return;
  if (mask && !mask[env]) return;
  WEnv<T> w;
  bind(m, w, smem, s, env);
  if constexpr (MODE == 0) {
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) != 0) {  // helper waves
      team_helper(m, w);
      return;
    }
  }
  team_init(w.e);
  Env<T>& e = w.e;
  const int l = lane_id();
  T* qpos = (T*)s.qpos; T* qvel = (T*)s.qvel; T* qacc = (T*)s.qacc_warmstart; T* ctrl = (T*)s.ctrl;
  T* qfrc = (T*)s.qfrc_applied; T* xfrc = (T*)s.xfrc_applied; T* tm = (T*)s.time;
  if (MODE == 1) {
    const T* dr = draws ? draws + 4 * (size_t)env : nullptr;
    if (!draws) {
      construction_philox_draws(seed, (uint32_t)(env_offset + env), (uint32_t)ce.episode[env], e.vec2);
      wsync();
      dr = e.vec2;
    }
    construction_reset_body(m, w, dr, ce, env, obs);
    wstore_state(m, w, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
    if (l == 0 && ce.episode) ce.episode[env] += 1;
    return;
  }
  wload_state(m, w, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
  const ActRow act(action, ce.action_f64, env, ids.n_act);
  construction_pre(m, e, ids, act);
  const int warn = wmj_step(m, w);
  const bool done = construction_post(m, e, ids, act, ce, env, obs, reward, terminated, truncated);
  if (ce.rollout && l == 0) {
    double* ro = ce.rollout + 4 * (size_t)env;
    ro[0] += reward[env];
    ro[1] += terminated[env];
    ro[2] += truncated[env];
    ro[3] += 1.0;
  }
  if (done && autoreset) {
    if (final_obs)
      for (int i = l; i < MGX_CONSTRUCTION_OBS; i += 64)
        final_obs[(size_t)env * MGX_CONSTRUCTION_OBS + i] = obs[(size_t)env * MGX_CONSTRUCTION_OBS + i];
    __threadfence();
    wsync();
    construction_philox_draws(seed, (uint32_t)(env_offset + env), (uint32_t)ce.episode[env], e.vec2);
    wsync();
    construction_reset_body(m, w, e.vec2, ce, env, obs);
    if (l == 0) ce.episode[env] += 1;
  }
  wstore_state(m, w, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
  if (l == 0) {
    if (s.warning) s.warning[env] += warn;
    if (s.overflow && e.overflow) s.overflow[env] += 1;
  }
  team_exit(w.e);
}

// env-logic-only test hook: state from the caller (golden vectors), no physics
template <typename T>
__global__ void __launch_bounds__(64) k_construction_logic(DevModel<T> m, ConstructionIds ids,
                                                           mgx_construction_logic_io io, mgx_construction_env ce,
                                                           int n_env) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int env = blockIdx.x;
  if (env >= n_env) return;
  Env<T> e;
  env_bind(m, e, smem);
  const int l = lane_id();
  for (int k = l; k < m.nq; k += 64) e.qpos[k] = ((const T*)io.qpos)[(size_t)env * m.nq + k];
  for (int k = l; k < m.nv; k += 64) e.qvel[k] = ((const T*)io.qvel)[(size_t)env * m.nv + k];
  for (int k = l; k < 3 * m.nbody; k += 64) e.xpos[k] = ((const T*)io.xpos)[(size_t)env * 3 * m.nbody + k];
  wsync();
  const ActRow act(io.action, ce.action_f64, env, ids.n_act);
  construction_pre(m, e, ids, act);
  construction_post(m, e, ids, act, ce, env, io.obs, io.reward, io.terminated, io.truncated);
  for (int k = l; k < m.nu; k += 64) ((T*)io.ctrl)[(size_t)env * m.nu + k] = e.ctrl[k];
}

// generic wide-model physics: nsub mj_steps (mgx_step for models with nv > 64)
template <typename T>
__global__ void __launch_bounds__(kTeamThreads) k_wide_step(DevModel<T> m, mgx_state s, mgx_frames fr, int n_env,
                                                            int nsub, const uint8_t* mask) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int env = blockIdx.x;
  if (env >= n_env) return;
  if (mask && !mask[env]) return;
  WEnv<T> w;
  bind(m, w, smem, s, env);
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) != 0) {
    team_helper(m, w);
    return;
  }
  team_init(w.e);
  Env<T>& e = w.e;
  T* qpos = (T*)s.qpos; T* qvel = (T*)s.qvel; T* qacc = (T*)s.qacc_warmstart; T* ctrl = (T*)s.ctrl;
  T* qfrc = (T*)s.qfrc_applied; T* xfrc = (T*)s.xfrc_applied; T* tm = (T*)s.time;
  wload_state(m, w, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
  int warn = 0;
#pragma clang loop unroll(disable)
  for (int k = 0; k < nsub; k++) warn += wmj_step(m, w);
  wstore_state(m, w, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
  const int l = lane_id();
  if (l == 0 && s.warning) s.warning[env] += warn;
  if (l == 0 && s.overflow && e.overflow) s.overflow[env] += 1;
  if (fr.xpos) for (int k = l; k < 3 * m.nbody; k += 64) ((T*)fr.xpos)[(size_t)env * 3 * m.nbody + k] = e.xpos[k];
  if (fr.xquat) for (int k = l; k < 4 * m.nbody; k += 64) ((T*)fr.xquat)[(size_t)env * 4 * m.nbody + k] = e.xquat[k];
  if (fr.subtree_com)
    for (int k = l; k < 3 * m.nbody; k += 64) ((T*)fr.subtree_com)[(size_t)env * 3 * m.nbody + k] = e.subtree_com[k];
  if (l == 0) {
    if (fr.ncon) fr.ncon[env] = e.ncon;
    if (fr.nefc) fr.nefc[env] = e.nefc;
    if (fr.niter) fr.niter[env] = e.niter;
  }
  team_exit(w.e);
}

// Debug dump of one wide forward pass (mgx_debug_forward's layout, DbgOff in mgx_internal.h)
template <typename T>
__global__ void __launch_bounds__(64) k_wide_debug(DevModel<T> m, mgx_state s, int n_env, T* dbg, DbgOff o) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int env = blockIdx.x;
  if (env >= n_env) return;
  WEnv<T> w;
  bind(m, w, smem, s, env);
  Env<T>& e = w.e;
  wload_state(m, w, (T*)s.qpos, (T*)s.qvel, (T*)s.qacc_warmstart, (T*)s.ctrl, (T*)s.qfrc_applied, (T*)s.xfrc_applied,
              (T*)s.time, env);
  T* D = dbg + (size_t)env * o.total;
  const int l = lane_id();
  kinematics(m, e);
  com_crb(m, e);
  for (int k = l; k < m.nM; k += 64) D[o.qM + k] = e.qLD[k];
  wsync();
  factor_ld<T, true>(m, e, e.qLD);
  for (int k = 0; k < 2; k++) {
    const int d = wdof(k);
    w.diaginv[k] = d < m.nv ? (T)1 / e.qLD[m.dof_Madr[d]] : (T)0;
  }
  for (int k = l; k < m.nM; k += 64) D[o.qLD + k] = e.qLD[k];
  velocity_bodies(m, e);
  for (int k = 0; k < 2; k++) {
    const int d = wdof(k);
    w.qfrc_smooth[k] = d < m.nv ? dof_force_applied(m, e, d, w.qfrc_applied[k]) : (T)0;
  }
  wsolve_M(m, w, e.qLD, w.qfrc_smooth, w.qacc_smooth);
  collision(m, e);
  wsync();
  for (int k = l; k < 3 * m.nbody; k += 64) D[o.xipos + k] = e.xipos[k];
  for (int k = l; k < 10 * m.nbody; k += 64) D[o.cinert + k] = e.cinert[k];
  for (int k = l; k < 6 * m.nv; k += 64) D[o.cdof_dot + k] = e.cdof_dot[k];
  for (int k = l; k < 6 * m.nbody; k += 64) D[o.cvel + k] = e.cvel[k];
  for (int k = l; k < 3 * m.ngeom; k += 64) D[o.geom_xpos + k] = e.geom_xpos[k];
  for (int k = l; k < 9 * m.ngeom; k += 64) D[o.geom_xmat + k] = e.geom_xmat[k];
  for (int c = l; c < e.ncon; c += 64) {
    D[o.con_dist + c] = e.con_dist[c];
    for (int k = 0; k < 3; k++) D[o.con_pos + 3 * c + k] = e.con_pos[3 * c + k];
    for (int k = 0; k < 9; k++) D[o.con_frame + 9 * c + k] = e.con_frame[9 * c + k];
    D[o.con_geom + 2 * c] = (T)e.con_geom[2 * c];
    D[o.con_geom + 2 * c + 1] = (T)e.con_geom[2 * c + 1];
  }
  wsync();
  make_constraint(m, e);
  for (int k = 0; k < 2; k++) {
    const int d = wdof(k);
    if (d < m.nv) e.vec0[d] = sqrt(w.diaginv[k]);
  }
  wsync();
  if (MGX_TRANSFORM_LANE_ROW) transform_rows<T, true>(m, e);
  else wtransform_rows(m, w, __builtin_amdgcn_readfirstlane(e.nefc), 0, 1);  // as wforward
  wsync();
  wsync();
  for (int r = l; r < e.nefc; r += 64)
    for (int k = 0; k < m.nv; k++) D[o.Bmat + r * m.nv + k] = e.Bm[r * e.Bs + k];
  wnewton(m, w);
  wsync();
  for (int k = l; k < 3 * m.nbody; k += 64) { D[o.xpos + k] = e.xpos[k]; D[o.subtree_com + k] = e.subtree_com[k]; }
  for (int k = l; k < 4 * m.nbody; k += 64) D[o.xquat + k] = e.xquat[k];
  for (int k = l; k < 6 * m.nv; k += 64) D[o.cdof + k] = e.cdof[k];
  if (l == 0) { D[o.ncon] = (T)e.ncon; D[o.nefc] = (T)e.nefc; D[o.niter] = (T)e.niter; }
  for (int r = l; r < e.nefc; r += 64) {
    D[o.efc_type + r] = (T)e.efc_type[r]; D[o.efc_id + r] = (T)e.efc_id[r]; D[o.efc_pos + r] = e.efc[8 * r + 7];
    D[o.efc_margin + r] = e.efc_margin[r]; D[o.efc_R + r] = e.efc[8 * r + 2]; D[o.efc_aref + r] = e.efc[8 * r + 5];
    D[o.efc_force + r] = e.efc[8 * r + 1];
  }
  for (int k = 0; k < 2; k++) {
    const int d = wdof(k);
    if (d < m.nv) {
      D[o.qfrc_smooth + d] = w.qfrc_smooth[k]; D[o.qacc_smooth + d] = w.qacc_smooth[k]; D[o.qacc + d] = w.qacc[k];
      D[o.qfrc_constraint + d] = w.qfrc_constraint[k];
    }
  }
}

bool construction_env_ok(const mgx_construction_env* e) { return e->scal && e->ints && e->total_reward; }

template <typename T>
int configure_lds(const mgx_model* m) {
  return mgx_set_lds(k_construction<T, 0>, m->L.bytes) | mgx_set_lds(k_construction<T, 1>, m->L.bytes) |
         mgx_set_lds(k_construction_logic<T>, m->L.bytes) | mgx_set_lds(k_wide_step<T>, m->L.bytes) |
         mgx_set_lds(k_wide_debug<T>, m->L.bytes);
}

template <typename T, int MODE>
void launch(const mgx_model* m, const DevModel<T>& M, const mgx_state* s, const mgx_construction_env* e,
            const float* action, const T* draws, float* obs, double* reward, uint8_t* term, uint8_t* trunc,
            float* final_obs, int autoreset, uint64_t seed, int env_offset, int n_env, const uint8_t* mask,
            hipStream_t st) {
  hipLaunchKernelGGL((k_construction<T, MODE>), dim3(n_env), dim3(MODE == 0 ? kTeamThreads : 64), m->L.bytes, st, M, m->cn, *s, *e, action, draws,
                     obs, reward, term, trunc, final_obs, autoreset, seed, env_offset, n_env, mask);
}

// a wide model's kernels: RK4 + Newton, rows in global scratch, nv <= 128
int wide_supported(const mgx_model* m) {
  const bool f32 = m->precision == MGX_F32;
  if (!m->wide) return fail(MGX_E_UNSUPPORTED, "the wide kernels are for models with 64 < nv <= 128");
  if ((f32 ? m->mf.integrator : m->md.integrator) != 1 || (f32 ? m->mf.solver : m->md.solver) != 2)
    return fail(MGX_E_UNSUPPORTED, "the wide kernels implement RK4 + Newton (construction_site.xml:10)");
  if (!m->L.gB) return fail(MGX_E_UNSUPPORTED, "the wide kernels keep the constraint rows in global scratch");
  return MGX_OK;
}

}  // namespace

namespace mgx {
// mgx_step / mgx_debug_forward for wide models (mgx_step.hip dispatches here)
int wide_step(const mgx_model* m, const mgx_state* s, const mgx_frames& fr, int n_env, int nsub, const uint8_t* mask,
              hipStream_t st) {
  int rc = wide_supported(m);
  if (rc) return rc;
  if (m->precision == MGX_F32)
    hipLaunchKernelGGL(k_wide_step<float>, dim3(n_env), dim3(kTeamThreads), m->L.bytes, st, m->mf, *s, fr, n_env, nsub, mask);
  else
    hipLaunchKernelGGL(k_wide_step<double>, dim3(n_env), dim3(kTeamThreads), m->L.bytes, st, m->md, *s, fr, n_env, nsub, mask);
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}
int wide_debug(const mgx_model* m, const mgx_state* s, int n_env, void* dbg, const DbgOff& o, hipStream_t st) {
  int rc = wide_supported(m);
  if (rc) return rc;
  if (m->precision == MGX_F32)
    hipLaunchKernelGGL(k_wide_debug<float>, dim3(n_env), dim3(64), m->L.bytes, st, m->mf, *s, n_env, (float*)dbg, o);
  else
    hipLaunchKernelGGL(k_wide_debug<double>, dim3(n_env), dim3(64), m->L.bytes, st, m->md, *s, n_env, (double*)dbg, o);
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}
int wide_kernels_configure(const mgx_model* m) {
  return m->precision == MGX_F32 ? configure_lds<float>(m) : configure_lds<double>(m);
}
}  // namespace mgx

extern "C" {

int mgx_construction_configure(mgx_model* m, const mgx_construction_ids* ids) {
  if (!m || !ids) return fail(MGX_E_ARG, "null argument");
  int rc = wide_supported(m);
  if (rc) return rc;
  const bool f32 = m->precision == MGX_F32;
  const int nv = f32 ? m->mf.nv : m->md.nv, nu = f32 ? m->mf.nu : m->md.nu, nb = f32 ? m->mf.nbody : m->md.nbody;
  const int nq = f32 ? m->mf.nq : m->md.nq;
  if (ids->max_episode_steps <= 0) return fail(MGX_E_ARG, "max_episode_steps must be > 0");
  if (ids->n_act != nu || nu > 64) return fail(MGX_E_ARG, "n_act must equal nu (<= 64): ctrl[:] = action");
  if (nq < 30 || nv < 30) return fail(MGX_E_ARG, "the observation reads qpos[:30] and qvel[:30]");
  if (ids->humanoid < 0 || ids->humanoid >= nb) return fail(MGX_E_ARG, "humanoid body id out of range");
  if (!(ids->action_limit > 0)) return fail(MGX_E_ARG, "action_limit must be > 0");
  ConstructionIds& o = m->cn;
  o.humanoid = ids->humanoid;
  o.n_act = ids->n_act;
  o.max_episode_steps = ids->max_episode_steps;
  o.action_limit = ids->action_limit;
  m->construction_ok = true;
  return MGX_OK;
}

int mgx_construction_step(const mgx_model* m, const mgx_state* s, const mgx_construction_env* e, const float* action,
                          float* obs, double* reward, uint8_t* terminated, uint8_t* truncated, float* final_obs,
                          int autoreset, uint64_t seed, int env_offset, int n_env, const uint8_t* mask, void* stream) {
  if (!m || !e || !action || !obs || !reward || !terminated || !truncated) return fail(MGX_E_ARG, "null argument");
  if (e->action_f64 != 0 && e->action_f64 != 1) return fail(MGX_E_ARG, "action_f64 must be 0 (float32) or 1 (float64)");
  if (!m->construction_ok) return fail(MGX_E_ARG, "mgx_construction_configure not called");
  if (!construction_env_ok(e)) return fail(MGX_E_ARG, "null construction env buffer");
  if (autoreset && !e->episode) return fail(MGX_E_ARG, "autoreset needs the episode counter buffer");
  const int rc = host_check_state(s);
  if (rc) return rc;
  if (!s->scratch) return fail(MGX_E_ARG, "this model needs mgx_state.scratch (scratch_bytes_per_env)");
  if (n_env <= 0) return MGX_OK;
  hipStream_t st = (hipStream_t)stream;
  if (m->precision == MGX_F32)
    launch<float, 0>(m, m->mf, s, e, action, nullptr, obs, reward, terminated, truncated, final_obs, autoreset, seed,
                     env_offset, n_env, mask, st);
  else
    launch<double, 0>(m, m->md, s, e, action, nullptr, obs, reward, terminated, truncated, final_obs, autoreset, seed,
                      env_offset, n_env, mask, st);
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}

int mgx_construction_reset(const mgx_model* m, const mgx_state* s, const mgx_construction_env* e, const void* draws,
                           float* obs, uint64_t seed, int env_offset, int n_env, const uint8_t* mask, void* stream) {
  if (!m || !e || !obs) return fail(MGX_E_ARG, "null argument");
  if (!m->construction_ok) return fail(MGX_E_ARG, "mgx_construction_configure not called");
  if (!construction_env_ok(e)) return fail(MGX_E_ARG, "null construction env buffer");
  if (!draws && !e->episode) return fail(MGX_E_ARG, "device draws need the episode counter buffer");
  const int rc = host_check_state(s);
  if (rc) return rc;
  if (!s->scratch) return fail(MGX_E_ARG, "this model needs mgx_state.scratch (scratch_bytes_per_env)");
  if (n_env <= 0) return MGX_OK;
  hipStream_t st = (hipStream_t)stream;
  if (m->precision == MGX_F32)
    launch<float, 1>(m, m->mf, s, e, nullptr, (const float*)draws, obs, nullptr, nullptr, nullptr, nullptr, 0, seed,
                     env_offset, n_env, mask, st);
  else
    launch<double, 1>(m, m->md, s, e, nullptr, (const double*)draws, obs, nullptr, nullptr, nullptr, nullptr, 0, seed,
                      env_offset, n_env, mask, st);
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}

int mgx_construction_logic_test(const mgx_model* m, const mgx_construction_logic_io* io, const mgx_construction_env* e,
                                int n_env, void* stream) {
  if (!m || !io || !e) return fail(MGX_E_ARG, "null argument");
  if (!m->construction_ok) return fail(MGX_E_ARG, "mgx_construction_configure not called");
  if (!construction_env_ok(e)) return fail(MGX_E_ARG, "null construction env buffer");
  if (n_env <= 0) return MGX_OK;
  hipStream_t st = (hipStream_t)stream;
  if (m->precision == MGX_F32)
    hipLaunchKernelGGL(k_construction_logic<float>, dim3(n_env), dim3(64), m->L.bytes, st, m->mf, m->cn, *io, *e, n_env);
  else
    hipLaunchKernelGGL(k_construction_logic<double>, dim3(n_env), dim3(64), m->L.bytes, st, m->md, m->cn, *io, *e,
                       n_env);
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}

}  // extern "C"
