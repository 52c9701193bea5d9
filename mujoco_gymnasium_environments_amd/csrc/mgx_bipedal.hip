// mgx_bipedal.hip — bipedal_rescue kernels and their C-ABI (include/mgx.h).
//
// One 64-thread workgroup (= one wavefront) per environment, as the generic step kernel
// (mgx_step.hip): a bipedal env step is clip + float32 energy -> one RK4 mj_step (four
// forward passes; constraint rows in per-env global scratch when the model's ~500 rows do not
// fit LDS) -> victim interactions -> observation / reward / termination / stats, with
// same-step autoreset (10 settle steps), all in one launch.
#include "mgx_internal.h"

using namespace mgx;

MGX_PROF_SETTER(mgx_prof_set_buffer_bipedal)

namespace {

int fail(int code, const std::string& msg) { return host_fail(code, msg); }

template <typename T, bool GB>
__device__ __forceinline__ void bind(const DevModel<T>& m, Env<T>& e, char* smem, const mgx_state& s, int env) {
  env_bind<T, GB>(m, e, smem, GB ? (T*)s.scratch + (size_t)env * m.L.gB_stride : nullptr);
}

// One launch = one env step (MODE 0; ended envs then reset in the same launch when autoreset)
// or one reset (MODE 1; host draws, or Philox keyed by (seed, env_offset + env, episode)). ONE
// physics call site: the step's RK4 mj_step and a reset's 10 settle steps share the loop below,
// so the forward pass (four stages per RK4 step) is inlined once.
template <typename T, int MODE, bool GB>
__global__ void __launch_bounds__(64) k_bipedal(DevModel<T> m, BipedalIds ids, mgx_state s, mgx_bipedal_env be,
                                                const float* action, const T* draws, float* obs, double* reward,
                                                uint8_t* terminated, uint8_t* truncated, float* final_obs, int autoreset,
                                                uint64_t seed, int env_offset, int n_env, const uint8_t* mask) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int env = blockIdx.x;
  if (env >= n_env) return;
  if (mask && !mask[env]) return;
  Env<T> e;
  bind<T, GB>(m, e, smem, s, env);
  int l = lane_id();
  T* qpos = (T*)s.qpos; T* qvel = (T*)s.qvel; T* qacc = (T*)s.qacc_warmstart; T* ctrl = (T*)s.ctrl;
  T* qfrc = (T*)s.qfrc_applied; T* xfrc = (T*)s.xfrc_applied; T* tm = (T*)s.time;
  load_state(m, e, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
  bool resetting = MODE == 1;
  if (MODE == 1) {
    const T* dr = draws ? draws + 12 * (size_t)env : nullptr;
    if (!draws) {
      bipedal_philox_draws(seed, (uint32_t)(env_offset + env), (uint32_t)be.episode[env], e.vec3);
      wsync();
      dr = e.vec3;
    }
    bipedal_reset_prologue(m, e, ids, dr, be, env);
  } else {
    bipedal_pre(m, e, ids, ActRow(action, be.action_f64, env, ids.n_act), be, env);
  }
  int warn = 0;
  for (;;) {
    const int nsteps = resetting ? 10 : 1;  // rescue_env.py:390-391 settle steps / one mj_step
#pragma clang loop unroll(disable)
    for (int k = 0; k < nsteps; k++) warn += mj_step_env<T, true>(m, e);
    if (resetting) {
      bipedal_reset_epilogue(m, e, ids, be, env, obs);
      if (l == 0 && be.episode) be.episode[env] += 1;
      break;
    }
    const bool done =
        bipedal_post(m, e, ids, ActRow(action, be.action_f64, env, ids.n_act), be, env, obs, reward, terminated, truncated);
    if (be.rollout && l == 0) {
      T* ro = (T*)be.rollout + 4 * (size_t)env;
      ro[0] += (T)reward[env];
      ro[1] += (T)terminated[env];
      ro[2] += (T)truncated[env];
      ro[3] += (T)1;
    }
    if (!(done && autoreset)) break;
    if (final_obs)
      for (int i = l; i < 102; i += 64) final_obs[(size_t)env * 102 + i] = obs[(size_t)env * 102 + i];
    __threadfence();
    wsync();
    bipedal_philox_draws(seed, (uint32_t)(env_offset + env), (uint32_t)be.episode[env], e.vec3);
    wsync();
    bipedal_reset_prologue(m, e, ids, e.vec3, be, env);
    resetting = true;
  }
  store_state(m, e, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
  if (l == 0) {
    if (s.warning) s.warning[env] += warn;
    if (s.overflow && e.overflow) s.overflow[env] += 1;
  }
}

// env-logic-only test hook: frames and contact distances from the caller (golden vectors)
template <typename T>
__global__ void __launch_bounds__(64) k_bipedal_logic(DevModel<T> m, BipedalIds ids, mgx_bipedal_logic_io io,
                                                      mgx_bipedal_env be, int n_env) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int env = blockIdx.x;
  if (env >= n_env) return;
  Env<T> e;
  env_bind(m, e, smem);
  int l = lane_id();
  for (int k = l; k < m.nq; k += 64) e.qpos[k] = ((const T*)io.qpos)[(size_t)env * m.nq + k];
  for (int k = l; k < m.nv; k += 64) e.qvel[k] = ((const T*)io.qvel)[(size_t)env * m.nv + k];
  for (int k = l; k < m.nu; k += 64) e.ctrl[k] = 0;
  for (int k = l; k < 3 * m.nbody; k += 64) e.xpos[k] = ((const T*)io.xpos)[(size_t)env * 3 * m.nbody + k];
  for (int k = l; k < 4 * m.nbody; k += 64) e.xquat[k] = ((const T*)io.xquat)[(size_t)env * 4 * m.nbody + k];
  int nc = io.ncon[env];
  e.ncon = nc;
  for (int c = l; c < nc; c += 64) e.con_dist[c] = ((const T*)io.con_dist)[(size_t)env * io.max_contacts + c];
  wsync();
  const ActRow a(io.action, be.action_f64, env, ids.n_act);
  bipedal_pre(m, e, ids, a, be, env);
  bipedal_post(m, e, ids, a, be, env, io.obs, io.reward, io.terminated, io.truncated, io.upright);
  wsync();
  for (int k = l; k < m.nu; k += 64) ((T*)io.ctrl)[(size_t)env * m.nu + k] = e.ctrl[k];
}

bool bipedal_env_ok(const mgx_bipedal_env* e) {
  return e->step && e->energy && e->energy_used && e->rescued && e->carried && e->carrying && e->closest &&
         e->prev_rescued && e->prev_carried && e->prev_sz && e->fall_timer && e->victims_rescued && e->distance &&
         e->ttfr && e->falls && e->collisions && e->prev_robot_pos;
}

template <typename T>
int configure_lds(const mgx_model* m) {
  return mgx_set_lds(k_bipedal<T, 0, true>, m->L.bytes) | mgx_set_lds(k_bipedal<T, 1, true>, m->L.bytes) |
         mgx_set_lds(k_bipedal<T, 0, false>, m->L.bytes) | mgx_set_lds(k_bipedal<T, 1, false>, m->L.bytes) |
         mgx_set_lds(k_bipedal_logic<T>, m->L.bytes);
}

template <typename T, int MODE>
void launch(const mgx_model* m, const DevModel<T>& M, const mgx_state* s, const mgx_bipedal_env* e, const float* action,
            const T* draws, float* obs, double* reward, uint8_t* term, uint8_t* trunc, float* final_obs, int autoreset,
            uint64_t seed, int env_offset, int n_env, const uint8_t* mask, hipStream_t st) {
  if (m->L.gB)
    hipLaunchKernelGGL((k_bipedal<T, MODE, true>), dim3(n_env), dim3(64), m->L.bytes, st, M, m->bp, *s, *e, action,
                       draws, obs, reward, term, trunc, final_obs, autoreset, seed, env_offset, n_env, mask);
  else
    hipLaunchKernelGGL((k_bipedal<T, MODE, false>), dim3(n_env), dim3(64), m->L.bytes, st, M, m->bp, *s, *e, action,
                       draws, obs, reward, term, trunc, final_obs, autoreset, seed, env_offset, n_env, mask);
}

}  // namespace

extern "C" {

int mgx_bipedal_configure(mgx_model* m, const mgx_bipedal_ids* ids) {
  if (!m || !ids) return fail(MGX_E_ARG, "null argument");
  if (m->wide) return fail(MGX_E_UNSUPPORTED, MGX_WIDE_MSG);
  bool f32 = m->precision == MGX_F32;
  int nq = f32 ? m->mf.nq : m->md.nq, nv = f32 ? m->mf.nv : m->md.nv, nu = f32 ? m->mf.nu : m->md.nu;
  int nb = f32 ? m->mf.nbody : m->md.nbody;
  if ((f32 ? m->mf.integrator : m->md.integrator) != 1)
    return fail(MGX_E_UNSUPPORTED, "the bipedal kernels integrate with RK4 (rescue_env.py:148)");
  if ((f32 ? m->mf.solver : m->md.solver) != 0)
    return fail(MGX_E_UNSUPPORTED, "the bipedal kernels solve with PGS (rescue_env.py:146)");
  if (ids->max_episode_steps <= 0) return fail(MGX_E_ARG, "max_episode_steps must be > 0");
  if (ids->n_act != 26 || nu < 26) return fail(MGX_E_ARG, "bipedal needs 26 actuators written from the action");
  if (ids->torso < 0 || ids->torso >= nb) return fail(MGX_E_ARG, "torso body id out of range");
  for (int i = 0; i < 5; i++) {
    if (ids->victims[i] < 0 || ids->victims[i] >= nb) return fail(MGX_E_ARG, "victim body id out of range");
    if (ids->victim_x[i] < 0 || ids->victim_x[i] >= nq || ids->victim_y[i] < 0 || ids->victim_y[i] >= nq)
      return fail(MGX_E_ARG, "victim qpos address out of range");
  }
  for (int i = 0; i < 26; i++)
    if (ids->obs_qposadr[i] < 0 || ids->obs_qposadr[i] >= nq || ids->obs_dofadr[i] < 0 || ids->obs_dofadr[i] >= nv)
      return fail(MGX_E_ARG, "observed joint address out of range");
  if (ids->root_x < 0 || ids->root_x >= nq || ids->root_y < 0 || ids->root_y >= nq || ids->root_z < 0 ||
      ids->root_z >= nq || ids->root_dof < 0 || ids->root_dof + 6 > nv)
    return fail(MGX_E_ARG, "root joint address out of range");
  int rc = f32 ? configure_lds<float>(m) : configure_lds<double>(m);
  if (rc != MGX_OK) return rc;
  rc = bipedal_staged_configure(m);
  if (rc != MGX_OK) return rc;
  BipedalIds& o = m->bp;
  o.torso = ids->torso;
  for (int i = 0; i < 5; i++) {
    o.victims[i] = ids->victims[i];
    o.victim_x[i] = ids->victim_x[i];
    o.victim_y[i] = ids->victim_y[i];
  }
  for (int i = 0; i < 26; i++) { o.obs_qposadr[i] = ids->obs_qposadr[i]; o.obs_dofadr[i] = ids->obs_dofadr[i]; }
  o.root_x = ids->root_x; o.root_y = ids->root_y; o.root_z = ids->root_z; o.root_dof = ids->root_dof;
  o.n_act = ids->n_act;
  o.max_episode_steps = ids->max_episode_steps;
  m->bipedal_ok = true;
  return MGX_OK;
}

int mgx_bipedal_step(const mgx_model* m, const mgx_state* s, const mgx_bipedal_env* e, const float* action, float* obs,
                     double* reward, uint8_t* terminated, uint8_t* truncated, float* final_obs, int autoreset,
                     uint64_t seed, int env_offset, int n_env, const uint8_t* mask, void* stream) {
  if (!m || !e || !action || !obs || !reward || !terminated || !truncated) return fail(MGX_E_ARG, "null argument");
  if (e->action_f64 != 0 && e->action_f64 != 1) return fail(MGX_E_ARG, "action_f64 must be 0 (float32) or 1 (float64)");
  if (!m->bipedal_ok) return fail(MGX_E_ARG, "mgx_bipedal_configure not called");
  if (!bipedal_env_ok(e)) return fail(MGX_E_ARG, "null bipedal env buffer");
  if (autoreset && !e->episode) return fail(MGX_E_ARG, "autoreset needs the episode counter buffer");
  int rc = host_check_state(s);
  if (rc) return rc;
  if (n_env <= 0) return MGX_OK;
  hipStream_t st = (hipStream_t)stream;
  if (e->workspace)  // the staged RK4 step (mgx_rk_staged.hip)
    return bipedal_step_staged(m, s, e, action, obs, reward, terminated, truncated, final_obs, autoreset, seed,
                               env_offset, n_env, mask, st);
  if (m->L.gB && !s->scratch) return fail(MGX_E_ARG, "this model needs mgx_state.scratch (scratch_bytes_per_env)");
  if (m->precision == MGX_F32)
    launch<float, 0>(m, m->mf, s, e, action, nullptr, obs, reward, terminated, truncated, final_obs, autoreset, seed,
                     env_offset, n_env, mask, st);
  else
    launch<double, 0>(m, m->md, s, e, action, nullptr, obs, reward, terminated, truncated, final_obs, autoreset, seed,
                      env_offset, n_env, mask, st);
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}

int mgx_bipedal_reset(const mgx_model* m, const mgx_state* s, const mgx_bipedal_env* e, const void* draws, float* obs,
                      uint64_t seed, int env_offset, int n_env, const uint8_t* mask, void* stream) {
  if (!m || !e || !obs) return fail(MGX_E_ARG, "null argument");
  if (!m->bipedal_ok) return fail(MGX_E_ARG, "mgx_bipedal_configure not called");
  if (!bipedal_env_ok(e)) return fail(MGX_E_ARG, "null bipedal env buffer");
  if (!draws && !e->episode) return fail(MGX_E_ARG, "device draws need the episode counter buffer");
  int rc = host_check_state(s);
  if (rc) return rc;
  if (n_env <= 0) return MGX_OK;
  hipStream_t st = (hipStream_t)stream;
  if (e->workspace)
    return bipedal_reset_staged(m, s, e, draws, obs, seed, env_offset, n_env, mask, st);
  if (m->L.gB && !s->scratch) return fail(MGX_E_ARG, "this model needs mgx_state.scratch (scratch_bytes_per_env)");
  if (m->precision == MGX_F32)
    launch<float, 1>(m, m->mf, s, e, nullptr, (const float*)draws, obs, nullptr, nullptr, nullptr, nullptr, 0, seed,
                     env_offset, n_env, mask, st);
  else
    launch<double, 1>(m, m->md, s, e, nullptr, (const double*)draws, obs, nullptr, nullptr, nullptr, nullptr, 0, seed,
                      env_offset, n_env, mask, st);
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}

int mgx_bipedal_logic_test(const mgx_model* m, const mgx_bipedal_logic_io* io, const mgx_bipedal_env* e, int n_env,
                           void* stream) {
  if (!m || !io || !e) return fail(MGX_E_ARG, "null argument");
  if (!m->bipedal_ok) return fail(MGX_E_ARG, "mgx_bipedal_configure not called");
  if (!bipedal_env_ok(e)) return fail(MGX_E_ARG, "null bipedal env buffer");
  if (io->max_contacts > m->L.max_ncon) return fail(MGX_E_CAPACITY, "max_contacts exceeds the contact capacity");
  if (n_env <= 0) return MGX_OK;
  hipStream_t st = (hipStream_t)stream;
  if (m->precision == MGX_F32)
    hipLaunchKernelGGL(k_bipedal_logic<float>, dim3(n_env), dim3(64), m->L.bytes, st, m->mf, m->bp, *io, *e, n_env);
  else
    hipLaunchKernelGGL(k_bipedal_logic<double>, dim3(n_env), dim3(64), m->L.bytes, st, m->md, m->bp, *io, *e, n_env);
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}

}  // extern "C"
