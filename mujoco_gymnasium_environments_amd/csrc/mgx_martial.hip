// mgx_martial.hip — humanoid_martial_arts kernels and their C-ABI (include/mgx.h).
//
// One 64-thread workgroup (= one wavefront) per environment, the execution model and LDS layout
// of the monolithic step (mgx_physics.h): a martial-arts env step is clip -> ctrl -> one mj_step
// (Euler, Newton: the Hessian and its Cholesky factor in the env's LDS) -> observation / reward /
// termination / statistics, with same-step autoreset (mj_forward, no settle steps), all in one
// launch.
#include "mgx_internal.h"

using namespace mgx;

MGX_PROF_SETTER(mgx_prof_set_buffer_martial)

namespace {

int fail(int code, const std::string& msg) { return host_fail(code, msg); }

template <typename T>
__device__ __forceinline__ void martial_reset_philox(const DevModel<T>& m, Env<T>& e, const MartialIds& ids, mgx_state s,
                                                     mgx_martial_env me, float* obs, uint64_t seed, int env_offset,
                                                     int env) {
  const int l = lane_id();
  const int E = me.episode[env];
  martial_philox_draws(seed, (uint32_t)(env_offset + env), (uint32_t)E, e.vec1);
  wsync();
  const T d0 = e.vec1[0], d1 = e.vec1[1];
  wsync();
  martial_reset_body(m, e, ids, d0, d1, me, env, obs);
  store_state(m, e, (T*)s.qpos, (T*)s.qvel, (T*)s.qacc_warmstart, (T*)s.ctrl, (T*)s.qfrc_applied, (T*)s.xfrc_applied,
              (T*)s.time, env);
  if (l == 0) {
    if (s.overflow && e.overflow) s.overflow[env] += 1;
    me.episode[env] = E + 1;
  }
}

// MODE 0: one env step (+ same-step autoreset); MODE 1: reset (host draws or Philox)
template <typename T, int MODE, bool GB>
__global__ void __launch_bounds__(64) k_martial(DevModel<T> m, MartialIds ids, mgx_state s, mgx_martial_env me,
                                                const float* action, const T* draws, float* obs, double* reward,
                                                uint8_t* terminated, uint8_t* truncated, float* final_obs, int autoreset,
                                                uint64_t seed, int env_offset, int n_env, const uint8_t* mask) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int env = blockIdx.x;
  if (env >= n_env) return;
  if (mask && !mask[env]) return;
  Env<T> e;
  env_bind<T, GB>(m, e, smem, GB ? (T*)s.scratch + (size_t)env * m.L.gB_stride : nullptr);
  const int l = lane_id();
  T* qpos = (T*)s.qpos; T* qvel = (T*)s.qvel; T* qacc = (T*)s.qacc_warmstart; T* ctrl = (T*)s.ctrl;
  T* qfrc = (T*)s.qfrc_applied; T* xfrc = (T*)s.xfrc_applied; T* tm = (T*)s.time;
  if (MODE == 1) {
    if (!draws) {
      martial_reset_philox(m, e, ids, s, me, obs, seed, env_offset, env);
      return;
    }
    load_state(m, e, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
    martial_reset_body(m, e, ids, draws[2 * (size_t)env], draws[2 * (size_t)env + 1], me, env, obs);
    store_state(m, e, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
    if (l == 0) {
      if (s.overflow && e.overflow) s.overflow[env] += 1;
      if (me.episode) me.episode[env] += 1;
    }
    return;
  }
  load_state(m, e, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
  const ActRow act(action, me.action_f64, env, ids.n_act);
  martial_pre(m, e, ids, act);
  const int warn = mj_step_env<T, false, true>(m, e);
  const bool done = martial_post(m, e, ids, act, me, env, obs, reward, terminated, truncated);
  if (me.rollout && l == 0) {
    double* ro = me.rollout + 4 * (size_t)env;
    ro[0] += reward[env];
    ro[1] += terminated[env];
    ro[2] += truncated[env];
    ro[3] += 1.0;
  }
  store_state(m, e, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
  if (l == 0 && s.warning) s.warning[env] += warn;
  if (l == 0 && s.overflow && e.overflow) s.overflow[env] += 1;
  if (done && autoreset) {
    if (final_obs)
      for (int i = l; i < MGX_MARTIAL_OBS; i += 64)
        final_obs[(size_t)env * MGX_MARTIAL_OBS + i] = obs[(size_t)env * MGX_MARTIAL_OBS + i];
    __threadfence();
    wsync();
    martial_reset_philox(m, e, ids, s, me, obs, seed, env_offset, env);
  }
}

// env-logic-only test hook: frames from the caller (golden vectors), no physics
template <typename T>
__global__ void __launch_bounds__(64) k_martial_logic(DevModel<T> m, MartialIds ids, mgx_martial_logic_io io,
                                                      mgx_martial_env me, int n_env) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int env = blockIdx.x;
  if (env >= n_env) return;
  Env<T> e;
  env_bind(m, e, smem);
  const int l = lane_id();
  for (int k = l; k < m.nq; k += 64) e.qpos[k] = ((const T*)io.qpos)[(size_t)env * m.nq + k];
  for (int k = l; k < m.nv; k += 64) e.qvel[k] = ((const T*)io.qvel)[(size_t)env * m.nv + k];
  for (int k = l; k < 3 * m.nbody; k += 64) e.xpos[k] = ((const T*)io.xpos)[(size_t)env * 3 * m.nbody + k];
  for (int k = l; k < 4 * m.nbody; k += 64) e.xquat[k] = ((const T*)io.xquat)[(size_t)env * 4 * m.nbody + k];
  for (int k = l; k < 6 * m.nbody; k += 64) e.cvel[k] = ((const T*)io.cvel)[(size_t)env * 6 * m.nbody + k];
  wsync();
  const ActRow act(io.action, me.action_f64, env, ids.n_act);
  martial_pre(m, e, ids, act);
  martial_post(m, e, ids, act, me, env, io.obs, io.reward, io.terminated, io.truncated);
  for (int k = l; k < m.nu; k += 64) ((T*)io.ctrl)[(size_t)env * m.nu + k] = e.ctrl[k];
}

bool martial_env_ok(const mgx_martial_env* e) { return e->scal && e->ints; }

template <typename T, int MODE>
void launch(const mgx_model* m, const DevModel<T>& M, const mgx_state* s, const mgx_martial_env* e, const float* action,
            const T* draws, float* obs, double* reward, uint8_t* term, uint8_t* trunc, float* final_obs, int autoreset,
            uint64_t seed, int env_offset, int n_env, const uint8_t* mask, hipStream_t st) {
  if (m->L.gB)
    hipLaunchKernelGGL((k_martial<T, MODE, true>), dim3(n_env), dim3(64), m->L.bytes, st, M, m->ma, *s, *e, action, draws,
                       obs, reward, term, trunc, final_obs, autoreset, seed, env_offset, n_env, mask);
  else
    hipLaunchKernelGGL((k_martial<T, MODE, false>), dim3(n_env), dim3(64), m->L.bytes, st, M, m->ma, *s, *e, action, draws,
                       obs, reward, term, trunc, final_obs, autoreset, seed, env_offset, n_env, mask);
}

}  // namespace

extern "C" {

int mgx_martial_configure(mgx_model* m, const mgx_martial_ids* ids) {
  if (!m || !ids) return fail(MGX_E_ARG, "null argument");
  if (m->wide) return fail(MGX_E_UNSUPPORTED, MGX_WIDE_MSG);
  const bool f32 = m->precision == MGX_F32;
  const int nq = f32 ? m->mf.nq : m->md.nq, nv = f32 ? m->mf.nv : m->md.nv, nu = f32 ? m->mf.nu : m->md.nu;
  const int nb = f32 ? m->mf.nbody : m->md.nbody;
  if ((f32 ? m->mf.integrator : m->md.integrator) != 0)
    return fail(MGX_E_UNSUPPORTED, "the martial-arts kernels need an Euler model");
  if ((f32 ? m->mf.solver : m->md.solver) != 2)
    return fail(MGX_E_UNSUPPORTED, "the martial-arts kernels solve with Newton (martial_arts_scene.xml:163)");
  if (ids->max_episode_steps <= 0) return fail(MGX_E_ARG, "max_episode_steps must be > 0");
  if (ids->n_act != nu || nu > 32) return fail(MGX_E_ARG, "n_act must equal nu (<= 32): ctrl[:] = action * ctrlrange");
  if (29 + (nq - 7) + (nv - 6) != MGX_MARTIAL_OBS) return fail(MGX_E_ARG, "the observation needs nq - 7 + nv - 6 == 84");
  const int b[7] = {ids->torso, ids->right_hand, ids->left_hand, ids->right_foot, ids->left_foot, ids->dummy1, ids->dummy2};
  for (int k = 0; k < 7; k++)
    if (b[k] < 0 || b[k] >= nb) return fail(MGX_E_ARG, "body id out of range");
  MartialIds& o = m->ma;
  o.torso = ids->torso; o.right_hand = ids->right_hand; o.left_hand = ids->left_hand;
  o.right_foot = ids->right_foot; o.left_foot = ids->left_foot; o.dummy1 = ids->dummy1; o.dummy2 = ids->dummy2;
  o.n_act = ids->n_act;
  o.max_episode_steps = ids->max_episode_steps;
  for (int k = 0; k < 32; k++) o.ctrl_scale[k] = ids->ctrl_scale[k];
  const int rc =
      f32 ? (mgx_set_lds(k_martial<float, 0, false>, m->L.bytes) | mgx_set_lds(k_martial<float, 1, false>, m->L.bytes) |
             mgx_set_lds(k_martial<float, 0, true>, m->L.bytes) | mgx_set_lds(k_martial<float, 1, true>, m->L.bytes) |
             mgx_set_lds(k_martial_logic<float>, m->L.bytes))
          : (mgx_set_lds(k_martial<double, 0, false>, m->L.bytes) | mgx_set_lds(k_martial<double, 1, false>, m->L.bytes) |
             mgx_set_lds(k_martial<double, 0, true>, m->L.bytes) | mgx_set_lds(k_martial<double, 1, true>, m->L.bytes) |
             mgx_set_lds(k_martial_logic<double>, m->L.bytes));
  if (rc != MGX_OK) return rc;
  m->martial_ok = true;
  return MGX_OK;
}

int mgx_martial_step(const mgx_model* m, const mgx_state* s, const mgx_martial_env* e, const float* action, float* obs,
                     double* reward, uint8_t* terminated, uint8_t* truncated, float* final_obs, int autoreset,
                     uint64_t seed, int env_offset, int n_env, const uint8_t* mask, void* stream) {
  if (!m || !e || !action || !obs || !reward || !terminated || !truncated) return fail(MGX_E_ARG, "null argument");
  if (e->action_f64 != 0 && e->action_f64 != 1) return fail(MGX_E_ARG, "action_f64 must be 0 (float32) or 1 (float64)");
  if (!m->martial_ok) return fail(MGX_E_ARG, "mgx_martial_configure not called");
  if (!martial_env_ok(e)) return fail(MGX_E_ARG, "null martial-arts env buffer");
  if (autoreset && !e->episode) return fail(MGX_E_ARG, "autoreset needs the episode counter buffer");
  const int rc = host_check_state(s);
  if (rc) return rc;
  if (m->L.gB && !s->scratch) return fail(MGX_E_ARG, "this model needs mgx_state.scratch (scratch_bytes_per_env)");
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

int mgx_martial_reset(const mgx_model* m, const mgx_state* s, const mgx_martial_env* e, const void* draws, float* obs,
                      uint64_t seed, int env_offset, int n_env, const uint8_t* mask, void* stream) {
  if (!m || !e || !obs) return fail(MGX_E_ARG, "null argument");
  if (!m->martial_ok) return fail(MGX_E_ARG, "mgx_martial_configure not called");
  if (!martial_env_ok(e)) return fail(MGX_E_ARG, "null martial-arts env buffer");
  if (!draws && !e->episode) return fail(MGX_E_ARG, "device draws need the episode counter buffer");
  const int rc = host_check_state(s);
  if (rc) return rc;
  if (m->L.gB && !s->scratch) return fail(MGX_E_ARG, "this model needs mgx_state.scratch (scratch_bytes_per_env)");
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

int mgx_martial_logic_test(const mgx_model* m, const mgx_martial_logic_io* io, const mgx_martial_env* e, int n_env,
                           void* stream) {
  if (!m || !io || !e) return fail(MGX_E_ARG, "null argument");
  if (!m->martial_ok) return fail(MGX_E_ARG, "mgx_martial_configure not called");
  if (!martial_env_ok(e)) return fail(MGX_E_ARG, "null martial-arts env buffer");
  if (n_env <= 0) return MGX_OK;
  hipStream_t st = (hipStream_t)stream;
  if (m->precision == MGX_F32)
    hipLaunchKernelGGL(k_martial_logic<float>, dim3(n_env), dim3(64), m->L.bytes, st, m->mf, m->ma, *io, *e, n_env);
  else
    hipLaunchKernelGGL(k_martial_logic<double>, dim3(n_env), dim3(64), m->L.bytes, st, m->md, m->ma, *io, *e, n_env);
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}

}  // extern "C"
