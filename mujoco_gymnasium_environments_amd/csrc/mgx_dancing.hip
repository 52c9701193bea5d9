// mgx_dancing.hip — humanoid_dancing kernels and their C-ABI (include/mgx.h).
//
// One 64-thread workgroup (= one wavefront) per environment, as the generic step kernel
// (mgx_step.hip): a dancing env step is clip + rhythm + spotlight -> one RK4 mj_step (four
// forward passes, rows in LDS) -> observation / reward / termination / stats / crowd / move
// transition, with same-step autoreset (10 settle steps), all in one launch.
#include "mgx_internal.h"

using namespace mgx;

MGX_PROF_SETTER(mgx_prof_set_buffer_dancing)

namespace {

int fail(int code, const std::string& msg) { return host_fail(code, msg); }

template <typename T, bool GB>
__device__ __forceinline__ void bind(const DevModel<T>& m, Env<T>& e, char* smem, const mgx_state& s, int env) {
  env_bind<T, GB>(m, e, smem, GB ? (T*)s.scratch + (size_t)env * m.L.gB_stride : nullptr);
}

// One launch = one env step (MODE 0; ended envs then reset in the same launch when autoreset)
// or one reset (MODE 1; host draws, or Philox keyed by (seed, env_offset + env, episode)).
// The kernel has ONE physics call site: the step's single RK4 mj_step and a reset's 10 settle
// steps run through the same loop, so the ~1.6k-instruction forward pass is inlined once (the
// earlier three-site form carried ~1.5k SGPR spills per kernel).
template <typename T, int MODE, bool GB>
__global__ void __launch_bounds__(64) k_dancing(DevModel<T> m, DancingIds ids, mgx_state s, mgx_dancing_env de,
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
    const T* dr = draws ? draws + 2 * MGX_DANCE_SEQ * (size_t)env : nullptr;
    if (!draws) {
      dancing_philox_draws(seed, (uint32_t)(env_offset + env), (uint32_t)de.episode[env], e.vec3);
      wsync();
      dr = e.vec3;
    }
    dancing_reset_prologue(m, e, dr, de, env);
  } else {
    dancing_pre(m, e, ids, ActRow(action, de.action_f64, env, ids.n_act), de, env);
  }
  int warn = 0;
  for (;;) {
    const int nsteps = resetting ? 10 : 1;  // dancing_env.py:809-810 settle steps / one mj_step
#pragma clang loop unroll(disable)
    for (int k = 0; k < nsteps; k++) warn += mj_step_env<T, true>(m, e);
    if (resetting) {
      dancing_reset_epilogue(m, e, ids, de, env, obs);
      if (l == 0 && de.episode) de.episode[env] += 1;
      break;
    }
    const bool done =
        dancing_post(m, e, ids, ActRow(action, de.action_f64, env, ids.n_act), de, env, obs, reward, terminated, truncated);
    if (de.rollout && l == 0) {
      T* ro = (T*)de.rollout + 4 * (size_t)env;
      ro[0] += (T)reward[env];
      ro[1] += (T)terminated[env];
      ro[2] += (T)truncated[env];
      ro[3] += (T)1;
    }
    if (!(done && autoreset)) break;
    if (final_obs)
      for (int i = l; i < MGX_DANCE_OBS; i += 64) final_obs[(size_t)env * MGX_DANCE_OBS + i] = obs[(size_t)env * MGX_DANCE_OBS + i];
    __threadfence();
    wsync();
    dancing_philox_draws(seed, (uint32_t)(env_offset + env), (uint32_t)de.episode[env], e.vec3);
    wsync();
    dancing_reset_prologue(m, e, e.vec3, de, env);
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
__global__ void __launch_bounds__(64) k_dancing_logic(DevModel<T> m, DancingIds ids, mgx_dancing_logic_io io,
                                                      mgx_dancing_env de, int n_env) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int env = blockIdx.x;
  if (env >= n_env) return;
  Env<T> e;
  env_bind(m, e, smem);
  int l = lane_id();
  for (int k = l; k < m.nq; k += 64) e.qpos[k] = ((const T*)io.qpos)[(size_t)env * m.nq + k];
  for (int k = l; k < m.nv; k += 64) e.qvel[k] = ((const T*)io.qvel)[(size_t)env * m.nv + k];
  for (int k = l; k < m.nu; k += 64) e.ctrl[k] = 0;
  for (int k = l; k < 3 * m.nbody; k += 64) {
    e.xpos[k] = ((const T*)io.xpos)[(size_t)env * 3 * m.nbody + k];
    e.subtree_com[k] = ((const T*)io.subtree_com)[(size_t)env * 3 * m.nbody + k];
  }
  for (int k = l; k < 4 * m.nbody; k += 64) e.xquat[k] = ((const T*)io.xquat)[(size_t)env * 4 * m.nbody + k];
  int nc = io.ncon[env];
  e.ncon = nc;
  for (int c = l; c < nc; c += 64) {
    e.con_geom[2 * c] = io.con_geom[((size_t)env * io.max_contacts + c) * 2];
    e.con_geom[2 * c + 1] = io.con_geom[((size_t)env * io.max_contacts + c) * 2 + 1];
  }
  wsync();
  const ActRow a(io.action, de.action_f64, env, ids.n_act);
  dancing_pre(m, e, ids, a, de, env);
  dancing_post(m, e, ids, a, de, env, io.obs, io.reward, io.terminated, io.truncated);
  wsync();
  for (int k = l; k < m.nu; k += 64) ((T*)io.ctrl)[(size_t)env * m.nu + k] = e.ctrl[k];
}

bool dancing_env_ok(const mgx_dancing_env* e) {
  return e->scal && e->ints && e->hist && e->moves && e->durations && e->prev_jvel;
}

template <typename T>
int configure_lds(const mgx_model* m) {
  return mgx_set_lds(k_dancing<T, 0, true>, m->L.bytes) | mgx_set_lds(k_dancing<T, 1, true>, m->L.bytes) |
         mgx_set_lds(k_dancing<T, 0, false>, m->L.bytes) | mgx_set_lds(k_dancing<T, 1, false>, m->L.bytes) |
         mgx_set_lds(k_dancing_logic<T>, m->L.bytes);
}

template <typename T, int MODE>
void launch(const mgx_model* m, const DevModel<T>& M, const mgx_state* s, const mgx_dancing_env* e, const float* action,
            const T* draws, float* obs, double* reward, uint8_t* term, uint8_t* trunc, float* final_obs, int autoreset,
            uint64_t seed, int env_offset, int n_env, const uint8_t* mask, hipStream_t st) {
  if (m->L.gB)
    hipLaunchKernelGGL((k_dancing<T, MODE, true>), dim3(n_env), dim3(64), m->L.bytes, st, M, m->dn, *s, *e, action,
                       draws, obs, reward, term, trunc, final_obs, autoreset, seed, env_offset, n_env, mask);
  else
    hipLaunchKernelGGL((k_dancing<T, MODE, false>), dim3(n_env), dim3(64), m->L.bytes, st, M, m->dn, *s, *e, action,
                       draws, obs, reward, term, trunc, final_obs, autoreset, seed, env_offset, n_env, mask);
}

}  // namespace

extern "C" {

int mgx_dancing_configure(mgx_model* m, const mgx_dancing_ids* ids) {
  if (!m || !ids) return fail(MGX_E_ARG, "null argument");
  if (m->wide) return fail(MGX_E_UNSUPPORTED, MGX_WIDE_MSG);
  bool f32 = m->precision == MGX_F32;
  int nq = f32 ? m->mf.nq : m->md.nq, nv = f32 ? m->mf.nv : m->md.nv, nu = f32 ? m->mf.nu : m->md.nu;
  int nb = f32 ? m->mf.nbody : m->md.nbody;
  if ((f32 ? m->mf.integrator : m->md.integrator) != 1)
    return fail(MGX_E_UNSUPPORTED, "the dancing kernels integrate with RK4 (dancing_env.py:179)");
  if ((f32 ? m->mf.solver : m->md.solver) != 0)
    return fail(MGX_E_UNSUPPORTED, "the dancing kernels solve with PGS (dancing_env.py:177)");
  if (ids->max_episode_steps <= 0) return fail(MGX_E_ARG, "max_episode_steps must be > 0");
  if (ids->n_act != 29 || nu < 29) return fail(MGX_E_ARG, "dancing needs 29 actuators written from the action");
  if (nv < 6 || nv > 64) return fail(MGX_E_ARG, "dancing observes qvel[6:] (6 < nv <= 64)");
  if (ids->torso < 0 || ids->torso >= nb) return fail(MGX_E_ARG, "torso body id out of range");
  if (ids->n_range < 0 || ids->n_range > 32) return fail(MGX_E_ARG, "n_range must be in [0, 32]");
  (void)nq;
  int rc = f32 ? configure_lds<float>(m) : configure_lds<double>(m);
  if (rc != MGX_OK) return rc;
  DancingIds& o = m->dn;
  o.torso = ids->torso;
  o.right_foot = ids->right_foot; o.left_foot = ids->left_foot; o.floor = ids->floor; o.stage = ids->stage;
  o.n_act = ids->n_act;
  o.max_episode_steps = ids->max_episode_steps;
  o.n_range = ids->n_range;
  for (int i = 0; i < 32; i++) { o.jnt_lo[i] = ids->jnt_lo[i]; o.jnt_hi[i] = ids->jnt_hi[i]; }
  m->dancing_ok = true;
  return MGX_OK;
}

int mgx_dancing_step(const mgx_model* m, const mgx_state* s, const mgx_dancing_env* e, const float* action, float* obs,
                     double* reward, uint8_t* terminated, uint8_t* truncated, float* final_obs, int autoreset,
                     uint64_t seed, int env_offset, int n_env, const uint8_t* mask, void* stream) {
  if (!m || !e || !action || !obs || !reward || !terminated || !truncated) return fail(MGX_E_ARG, "null argument");
  if (e->action_f64 != 0 && e->action_f64 != 1) return fail(MGX_E_ARG, "action_f64 must be 0 (float32) or 1 (float64)");
  if (!m->dancing_ok) return fail(MGX_E_ARG, "mgx_dancing_configure not called");
  if (!dancing_env_ok(e)) return fail(MGX_E_ARG, "null dancing env buffer");
  if (autoreset && !e->episode) return fail(MGX_E_ARG, "autoreset needs the episode counter buffer");
  int rc = host_check_state(s);
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

int mgx_dancing_reset(const mgx_model* m, const mgx_state* s, const mgx_dancing_env* e, const void* draws, float* obs,
                      uint64_t seed, int env_offset, int n_env, const uint8_t* mask, void* stream) {
  if (!m || !e || !obs) return fail(MGX_E_ARG, "null argument");
  if (!m->dancing_ok) return fail(MGX_E_ARG, "mgx_dancing_configure not called");
  if (!dancing_env_ok(e)) return fail(MGX_E_ARG, "null dancing env buffer");
  if (!draws && !e->episode) return fail(MGX_E_ARG, "device draws need the episode counter buffer");
  int rc = host_check_state(s);
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

int mgx_dancing_logic_test(const mgx_model* m, const mgx_dancing_logic_io* io, const mgx_dancing_env* e, int n_env,
                           void* stream) {
  if (!m || !io || !e) return fail(MGX_E_ARG, "null argument");
  if (!m->dancing_ok) return fail(MGX_E_ARG, "mgx_dancing_configure not called");
  if (!dancing_env_ok(e)) return fail(MGX_E_ARG, "null dancing env buffer");
  if (io->max_contacts > m->L.max_ncon) return fail(MGX_E_CAPACITY, "max_contacts exceeds the contact capacity");
  if (n_env <= 0) return MGX_OK;
  hipStream_t st = (hipStream_t)stream;
  if (m->precision == MGX_F32)
    hipLaunchKernelGGL(k_dancing_logic<float>, dim3(n_env), dim3(64), m->L.bytes, st, m->mf, m->dn, *io, *e, n_env);
  else
    hipLaunchKernelGGL(k_dancing_logic<double>, dim3(n_env), dim3(64), m->L.bytes, st, m->md, m->dn, *io, *e, n_env);
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}

}  // extern "C"
