// mgx_parkour.hip — quadruped_parkour kernels and their C-ABI (include/mgx.h).
//
// One 64-thread workgroup (= one wavefront) per environment, the same execution model and
// LDS layout as the monolithic soccer step (mgx_physics.h): a parkour env step is
// clip -> 10 x mj_step (dt 1 ms, PGS, Euler; plane contacts) -> obstacle motors ->
// observation / reward / termination, with same-step autoreset, all in one launch.
#include "mgx_internal.h"

using namespace mgx;

MGX_PROF_SETTER(mgx_prof_set_buffer_parkour)

namespace {

int fail(int code, const std::string& msg) { return host_fail(code, msg); }

// Philox-drawn reset of `env` for its current episode counter (the counter then advances);
// writes the state back to HBM.
template <typename T>
__device__ __forceinline__ void parkour_reset_philox(const DevModel<T>& m, Env<T>& e, const ParkourIds<T>& ids,
                                                     mgx_state s, mgx_parkour_env ev, float* obs, uint64_t seed,
                                                     int env_offset, int env) {
  int l = lane_id();
  int E = ev.episode[env];
  parkour_philox_draws(seed, (uint32_t)(env_offset + env), (uint32_t)E, e.vec1);
  wsync();
  T d0 = e.vec1[0], d1 = e.vec1[1];
  wsync();
  int warn = parkour_reset_body(m, e, ids, d0, d1, ev, env, obs);
  store_state(m, e, (T*)s.qpos, (T*)s.qvel, (T*)s.qacc_warmstart, (T*)s.ctrl, (T*)s.qfrc_applied, (T*)s.xfrc_applied,
              (T*)s.time, env);
  if (l == 0) {
    if (s.warning) s.warning[env] += warn;
    if (s.overflow && e.overflow) s.overflow[env] += 1;
    ev.episode[env] = E + 1;
  }
}

// MODE 0: one env step (+ same-step autoreset); MODE 1: reset (host draws or Philox)
template <typename T, int MODE, bool GB>
__global__ void __launch_bounds__(64) k_parkour(DevModel<T> m, ParkourIds<T> ids, mgx_state s, mgx_parkour_env ev,
                                                const float* action, const T* draws, float* obs, double* reward,
                                                uint8_t* terminated, uint8_t* truncated, float* final_obs, int autoreset,
                                                uint64_t seed, int env_offset, int n_env, const uint8_t* mask) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int env = blockIdx.x;
  if (env >= n_env) return;
  if (mask && !mask[env]) return;
  Env<T> e;
  env_bind<T, GB>(m, e, smem, GB ? (T*)s.scratch + (size_t)env * m.L.gB_stride : nullptr);
  int l = lane_id();
  T* qpos = (T*)s.qpos; T* qvel = (T*)s.qvel; T* qacc = (T*)s.qacc_warmstart; T* ctrl = (T*)s.ctrl;
  T* qfrc = (T*)s.qfrc_applied; T* xfrc = (T*)s.xfrc_applied; T* tm = (T*)s.time;
  if (MODE == 1) {
    if (!draws) {
      parkour_reset_philox(m, e, ids, s, ev, obs, seed, env_offset, env);
      return;
    }
    load_state(m, e, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
    int warn = parkour_reset_body(m, e, ids, draws[2 * (size_t)env], draws[2 * (size_t)env + 1], ev, env, obs);
    store_state(m, e, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
    if (l == 0) {
      if (s.warning) s.warning[env] += warn;
      if (s.overflow && e.overflow) s.overflow[env] += 1;
      if (ev.episode) ev.episode[env] += 1;
    }
    return;
  }
  load_state(m, e, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
  const ActRow a(action, ev.action_f64, env, ids.n_leg);
  parkour_pre(m, e, ids, a);
  int warn = 0;
  for (int k = 0; k < 10; k++) warn += mj_step_env(m, e);  // frame_skip (parkour_env.py:367-368)
  bool done = parkour_post(m, e, ids, a, ev, env, obs, reward, terminated, truncated);
  if (ev.rollout && l == 0) {
    T* ro = (T*)ev.rollout + 4 * (size_t)env;
    ro[0] += (T)reward[env];
    ro[1] += (T)terminated[env];
    ro[2] += (T)truncated[env];
    ro[3] += (T)1;
  }
  store_state(m, e, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
  if (l == 0 && s.warning) s.warning[env] += warn;
  if (l == 0 && s.overflow && e.overflow) s.overflow[env] += 1;
  if (done && autoreset) {
    if (final_obs)
      for (int i = l; i < 95; i += 64) final_obs[(size_t)env * 95 + i] = obs[(size_t)env * 95 + i];
    __threadfence();
    wsync();
    parkour_reset_philox(m, e, ids, s, ev, obs, seed, env_offset, env);
  }
}

// env-logic-only test hook: frames and contact lists from the caller (golden vectors)
template <typename T>
__global__ void __launch_bounds__(64) k_parkour_logic(DevModel<T> m, ParkourIds<T> ids, mgx_parkour_logic_io io,
                                                      mgx_parkour_env ev, int n_env) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int env = blockIdx.x;
  if (env >= n_env) return;
  Env<T> e;
  env_bind(m, e, smem);
  int l = lane_id();
  for (int k = l; k < m.nq; k += 64) e.qpos[k] = ((const T*)io.qpos)[(size_t)env * m.nq + k];
  for (int k = l; k < m.nv; k += 64) e.qvel[k] = ((const T*)io.qvel)[(size_t)env * m.nv + k];
  for (int k = l; k < m.nu; k += 64) e.ctrl[k] = ((const T*)io.ctrl)[(size_t)env * m.nu + k];
  for (int k = l; k < 3 * m.nbody; k += 64) e.xpos[k] = ((const T*)io.xpos)[(size_t)env * 3 * m.nbody + k];
  int nc = io.ncon[env];
  e.ncon = nc;
  for (int c = l; c < nc; c += 64) {
    e.con_geom[2 * c] = io.con_geom[((size_t)env * io.max_contacts + c) * 2];
    e.con_geom[2 * c + 1] = io.con_geom[((size_t)env * io.max_contacts + c) * 2 + 1];
  }
  wsync();
  const ActRow a(io.action, ev.action_f64, env, ids.n_leg);
  parkour_pre(m, e, ids, a);
  parkour_post(m, e, ids, a, ev, env, io.obs, io.reward, io.terminated, io.truncated);
  wsync();
  for (int k = l; k < m.nu; k += 64) ((T*)io.ctrl)[(size_t)env * m.nu + k] = e.ctrl[k];
}

template <typename T>
void fill_parkour_ids(ParkourIds<T>& o, const mgx_parkour_ids* ids) {
  o.torso = ids->torso;
  for (int i = 0; i < 4; i++) o.feet[i] = ids->feet[i];
  o.platform_qpos = ids->platform_qpos; o.pendulum_qpos = ids->pendulum_qpos;
  o.platform_act = ids->platform_act; o.pendulum_act = ids->pendulum_act;
  o.n_leg = ids->n_leg; o.max_episode_steps = ids->max_episode_steps;
  for (int i = 0; i < 16; i++) o.act_lim[i] = ids->act_lim[i];
}

bool parkour_env_ok(const mgx_parkour_env* e) {
  return e->last_position && e->max_progress && e->episode_reward && e->er_kind && e->reached && e->fall_count &&
         e->stuck && e->step;
}

}  // namespace

// rows in LDS or, with MGX_ROWS_IN_SCRATCH / an oversize model, in per-env global scratch
#define MGX_PK_LAUNCH(T, MODE, ...)                                  \
  do {                                                               \
    if (m->L.gB) hipLaunchKernelGGL((k_parkour<T, MODE, true>), __VA_ARGS__);  \
    else hipLaunchKernelGGL((k_parkour<T, MODE, false>), __VA_ARGS__);        \
  } while (0)

extern "C" {

int mgx_parkour_configure(mgx_model* m, const mgx_parkour_ids* ids) {
  if (!m || !ids) return fail(MGX_E_ARG, "null argument");
  if (m->wide) return fail(MGX_E_UNSUPPORTED, MGX_WIDE_MSG);
  int nq = m->precision == MGX_F32 ? m->mf.nq : m->md.nq;
  int nu = m->precision == MGX_F32 ? m->mf.nu : m->md.nu;
  int nb = m->precision == MGX_F32 ? m->mf.nbody : m->md.nbody;
  if (ids->max_episode_steps <= 0) return fail(MGX_E_ARG, "max_episode_steps must be > 0");
  if ((m->precision == MGX_F32 ? m->mf.integrator : m->md.integrator) != 0)
    return fail(MGX_E_UNSUPPORTED, "the parkour kernels need an Euler model whose rows fit LDS");
  if ((m->precision == MGX_F32 ? m->mf.solver : m->md.solver) != 0)
    return fail(MGX_E_UNSUPPORTED, "the parkour kernels solve with PGS (quadruped.xml:4)");
  if (ids->n_leg != 16 || nu < 16 || nq < 7) return fail(MGX_E_ARG, "parkour needs 16 leg actuators and a free root");
  if (ids->torso < 0 || ids->torso >= nb) return fail(MGX_E_ARG, "torso body id out of range");
  for (int i = 0; i < 4; i++)
    if (ids->feet[i] < 0 || ids->feet[i] >= nb) return fail(MGX_E_ARG, "foot body id out of range");
  if (ids->platform_qpos < 0 || ids->platform_qpos >= nq || ids->pendulum_qpos < 0 || ids->pendulum_qpos >= nq)
    return fail(MGX_E_ARG, "obstacle qpos index out of range");
  if (ids->platform_act >= nu || ids->pendulum_act >= nu) return fail(MGX_E_ARG, "obstacle actuator id out of range");
  int rc;
  if (m->precision == MGX_F32) {
    fill_parkour_ids(m->pkf, ids);
    rc = mgx_set_lds(k_parkour<float, 0, false>, m->L.bytes) | mgx_set_lds(k_parkour<float, 1, false>, m->L.bytes) |
         mgx_set_lds(k_parkour<float, 0, true>, m->L.bytes) | mgx_set_lds(k_parkour<float, 1, true>, m->L.bytes) |
         mgx_set_lds(k_parkour_logic<float>, m->L.bytes);
  } else {
    fill_parkour_ids(m->pkd, ids);
    rc = mgx_set_lds(k_parkour<double, 0, false>, m->L.bytes) | mgx_set_lds(k_parkour<double, 1, false>, m->L.bytes) |
         mgx_set_lds(k_parkour<double, 0, true>, m->L.bytes) | mgx_set_lds(k_parkour<double, 1, true>, m->L.bytes) |
         mgx_set_lds(k_parkour_logic<double>, m->L.bytes);
  }
  if (rc != MGX_OK) return rc;
  rc = parkour_staged_configure(m);
  if (rc != MGX_OK) return rc;
  m->parkour_ok = true;
  return MGX_OK;
}

int mgx_parkour_step(const mgx_model* m, const mgx_state* s, const mgx_parkour_env* e, const float* action, float* obs,
                     double* reward, uint8_t* terminated, uint8_t* truncated, float* final_obs, int autoreset,
                     uint64_t seed, int env_offset, int n_env, const uint8_t* mask, void* stream) {
  if (!m || !e || !action || !obs || !reward || !terminated || !truncated) return fail(MGX_E_ARG, "null argument");
  if (e->action_f64 != 0 && e->action_f64 != 1) return fail(MGX_E_ARG, "action_f64 must be 0 (float32) or 1 (float64)");
  if (!m->parkour_ok) return fail(MGX_E_ARG, "mgx_parkour_configure not called");
  if (!parkour_env_ok(e)) return fail(MGX_E_ARG, "null parkour env buffer");
  if (autoreset && !e->episode) return fail(MGX_E_ARG, "autoreset needs the episode counter buffer");
  int rc = host_check_state(s);
  if (rc) return rc;
  if (n_env <= 0) return MGX_OK;
  hipStream_t st = (hipStream_t)stream;
  if (e->workspace)  // the staged step (mgx_pk_staged.hip)
    return parkour_step_staged(m, s, e, action, obs, reward, terminated, truncated, final_obs, autoreset, seed,
                               env_offset, n_env, mask, st);
  if (m->L.gB && !s->scratch) return fail(MGX_E_ARG, "this model needs mgx_state.scratch (scratch_bytes_per_env)");
  if (m->precision == MGX_F32)
    MGX_PK_LAUNCH(float, 0, dim3(n_env), dim3(64), m->L.bytes, st, m->mf, m->pkf, *s, *e, action,
                       (const float*)nullptr, obs, reward, terminated, truncated, final_obs, autoreset, seed,
                       env_offset, n_env, mask);
  else
    MGX_PK_LAUNCH(double, 0, dim3(n_env), dim3(64), m->L.bytes, st, m->md, m->pkd, *s, *e, action,
                       (const double*)nullptr, obs, reward, terminated, truncated, final_obs, autoreset, seed,
                       env_offset, n_env, mask);
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}

int mgx_parkour_reset(const mgx_model* m, const mgx_state* s, const mgx_parkour_env* e, const void* draws, float* obs,
                      uint64_t seed, int env_offset, int n_env, const uint8_t* mask, void* stream) {
  if (!m || !e || !obs) return fail(MGX_E_ARG, "null argument");
  if (!m->parkour_ok) return fail(MGX_E_ARG, "mgx_parkour_configure not called");
  if (!parkour_env_ok(e)) return fail(MGX_E_ARG, "null parkour env buffer");
  if (!draws && !e->episode) return fail(MGX_E_ARG, "device draws need the episode counter buffer");
  int rc = host_check_state(s);
  if (rc) return rc;
  if (n_env <= 0) return MGX_OK;
  hipStream_t st = (hipStream_t)stream;
  if (e->workspace)  // every reset of a staged batch settles through the staged stages
    return parkour_reset_staged(m, s, e, draws, obs, seed, env_offset, n_env, mask, st);
  if (m->L.gB && !s->scratch) return fail(MGX_E_ARG, "this model needs mgx_state.scratch (scratch_bytes_per_env)");
  if (m->precision == MGX_F32)
    MGX_PK_LAUNCH(float, 1, dim3(n_env), dim3(64), m->L.bytes, st, m->mf, m->pkf, *s, *e,
                       (const float*)nullptr, (const float*)draws, obs, (double*)nullptr, (uint8_t*)nullptr,
                       (uint8_t*)nullptr, (float*)nullptr, 0, seed, env_offset, n_env, mask);
  else
    MGX_PK_LAUNCH(double, 1, dim3(n_env), dim3(64), m->L.bytes, st, m->md, m->pkd, *s, *e,
                       (const float*)nullptr, (const double*)draws, obs, (double*)nullptr, (uint8_t*)nullptr,
                       (uint8_t*)nullptr, (float*)nullptr, 0, seed, env_offset, n_env, mask);
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}

int64_t mgx_parkour_workspace_bytes(const mgx_model* m, int n_env, int banks) {
  return parkour_workspace_bytes(m, n_env, banks);
}
int mgx_parkour_workspace_init(const mgx_model* m, void* workspace, uint64_t bytes, int n_env, int banks, void* stream) {
  return parkour_workspace_init(m, workspace, bytes, n_env, banks, (hipStream_t)stream);
}

int mgx_parkour_logic_test(const mgx_model* m, const mgx_parkour_logic_io* io, const mgx_parkour_env* e, int n_env,
                           void* stream) {
  if (!m || !io || !e) return fail(MGX_E_ARG, "null argument");
  if (!m->parkour_ok) return fail(MGX_E_ARG, "mgx_parkour_configure not called");
  if (!parkour_env_ok(e)) return fail(MGX_E_ARG, "null parkour env buffer");
  if (io->max_contacts > m->L.max_ncon) return fail(MGX_E_CAPACITY, "max_contacts exceeds the contact capacity");
  if (n_env <= 0) return MGX_OK;
  hipStream_t st = (hipStream_t)stream;
  if (m->precision == MGX_F32)
    hipLaunchKernelGGL(k_parkour_logic<float>, dim3(n_env), dim3(64), m->L.bytes, st, m->mf, m->pkf, *io, *e, n_env);
  else
    hipLaunchKernelGGL(k_parkour_logic<double>, dim3(n_env), dim3(64), m->L.bytes, st, m->md, m->pkd, *io, *e, n_env);
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}

}  // extern "C"
