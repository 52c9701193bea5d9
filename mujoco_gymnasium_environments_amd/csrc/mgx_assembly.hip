// mgx_assembly.hip — robotic_arm_assembly kernels and their C-ABI (include/mgx.h).
//
// One 128-thread workgroup per environment: wave 0 runs the step as the generic step kernel
// (mgx_step.hip) does, wave 1 takes every other row batch of the Newton solver's passes (setup,
// gradient, J p, forces), tile row 3 of its MFMA Hessian and half of the Cholesky trailing tiles
// (mgx_physics.h team_helper_n; the kernel uses all 512 registers of a wave, so two envs per CU
// put one wave on each SIMD). An assembly env step is clip -> ctrl -> 10 mj_steps (Euler, Newton: the
// nv x nv Hessian and its Cholesky factor in the env's LDS; constraint rows in LDS or, when the
// scene's ~300 rows do not fit next to the rest, in per-env global scratch) -> gripper-contact
// task state / reward / termination / observation, with same-step autoreset (10 settle steps),
// all in one launch.
#define MGX_TEAM  // kernels with a Newton helper wave (lane_id, team_begin)
#include "mgx_internal.h"
#include "mgx_assembly.h"

using namespace mgx;

MGX_PROF_SETTER(mgx_prof_set_buffer_assembly)

namespace {

int fail(int code, const std::string& msg) { return host_fail(code, msg); }

template <typename T, bool GB>
__device__ __forceinline__ void bind(const DevModel<T>& m, Env<T>& e, char* smem, const mgx_state& s, int env) {
  env_bind<T, GB>(m, e, smem, GB ? (T*)s.scratch + (size_t)env * m.L.gB_stride : nullptr);
}

// MODE 0: one env step (10 substeps; ended envs then reset in the same launch when autoreset);
// MODE 1: reset. ONE physics call site: the step's substeps and a reset's settle steps share
// the loop below, so the Newton forward pass is inlined once.
constexpr int kTeamThreads = 128;  // wave 0 + the Newton helper wave (mgx_physics.h team_helper_n)
template <typename T, int MODE, bool GB>
__global__ void __launch_bounds__(kTeamThreads) k_assembly(DevModel<T> m, mgx_assembly_ids ids, mgx_state s, mgx_assembly_env ae,
                                                 const float* action, float* obs, double* reward, uint8_t* terminated,
                                                 uint8_t* truncated, float* final_obs, int autoreset, int n_env,
                                                 const uint8_t* mask) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int env = blockIdx.x;
  if (env >= n_env) return;
  if (mask && !mask[env]) return;
  Env<T> e;
  bind<T, GB>(m, e, smem, s, env);
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) != 0) {  // the helper wave
    team_helper_n(m, e);
    return;
  }
  team_init(e);
  const int l = lane_id();
  T* qpos = (T*)s.qpos; T* qvel = (T*)s.qvel; T* qacc = (T*)s.qacc_warmstart; T* ctrl = (T*)s.ctrl;
  T* qfrc = (T*)s.qfrc_applied; T* xfrc = (T*)s.xfrc_applied; T* tm = (T*)s.time;
  load_state(m, e, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
  bool resetting = MODE == 1;
  if (MODE == 1) assembly_reset_prologue(m, e, ae, env);
  else assembly_pre(m, e, ids, ActRow(action, ae.action_f64, env, 9));
  int warn = 0;
  for (;;) {
    const int nsteps = resetting ? ids.settle_steps : ids.substeps;  // assembly_env.py:186 / :228-229
#pragma clang loop unroll(disable)
    for (int k = 0; k < nsteps; k++) warn += mj_step_env<T, false, true>(m, e);
    if (resetting) {
      assembly_reset_epilogue(m, e, ids, env, obs);
      if (l == 0 && ae.episode) ae.episode[env] += 1;
      break;
    }
    const bool done = assembly_post(m, e, ids, ae, env, obs, reward, terminated, truncated);
    if (ae.rollout && l == 0) {
      double* ro = ae.rollout + 4 * (size_t)env;
      ro[0] += reward[env];
      ro[1] += terminated[env];
      ro[2] += truncated[env];
      ro[3] += 1.0;
    }
    if (!(done && autoreset)) break;
    if (final_obs)
      for (int i = l; i < MGX_ASSEMBLY_OBS; i += 64)
        final_obs[(size_t)env * MGX_ASSEMBLY_OBS + i] = obs[(size_t)env * MGX_ASSEMBLY_OBS + i];
    __threadfence();
    wsync();
    assembly_reset_prologue(m, e, ae, env);
    resetting = true;
  }
  store_state(m, e, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
  if (l == 0) {
    if (s.warning) s.warning[env] += warn;
    if (s.overflow && e.overflow) s.overflow[env] += 1;
  }
  team_exit(e);
}

// env-logic-only test hook: frames and contact lists from the caller (golden vectors)
template <typename T>
__global__ void __launch_bounds__(64) k_assembly_logic(DevModel<T> m, mgx_assembly_ids ids, mgx_assembly_logic_io io,
                                                       mgx_assembly_env ae, int n_env) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int env = blockIdx.x;
  if (env >= n_env) return;
  Env<T> e;
  env_bind(m, e, smem);
  const int l = lane_id();
  for (int k = l; k < m.nq; k += 64) e.qpos[k] = ((const T*)io.qpos)[(size_t)env * m.nq + k];
  for (int k = l; k < m.nv; k += 64) e.qvel[k] = ((const T*)io.qvel)[(size_t)env * m.nv + k];
  for (int k = l; k < m.nu; k += 64) e.ctrl[k] = 0;
  for (int k = l; k < 3 * m.nbody; k += 64) e.xpos[k] = ((const T*)io.xpos)[(size_t)env * 3 * m.nbody + k];
  for (int k = l; k < 4 * m.nbody; k += 64) e.xquat[k] = ((const T*)io.xquat)[(size_t)env * 4 * m.nbody + k];
  const int nc = io.ncon[env];
  e.ncon = nc;
  for (int c = l; c < nc; c += 64) {
    e.con_dist[c] = ((const T*)io.con_dist)[(size_t)env * io.max_contacts + c];
    e.con_geom[2 * c] = io.con_geom[((size_t)env * io.max_contacts + c) * 2];
    e.con_geom[2 * c + 1] = io.con_geom[((size_t)env * io.max_contacts + c) * 2 + 1];
  }
  wsync();
  assembly_pre(m, e, ids, ActRow(io.action, ae.action_f64, env, 9));
  assembly_post(m, e, ids, ae, env, io.obs, io.reward, io.terminated, io.truncated);
  for (int k = l; k < m.nu; k += 64) ((T*)io.ctrl)[(size_t)env * m.nu + k] = e.ctrl[k];
}

bool assembly_env_ok(const mgx_assembly_env* e) { return e->ints && e->cumulative && e->reset_qpos; }

template <typename T>
int configure_lds(const mgx_model* m) {
  return mgx_set_lds(k_assembly<T, 0, true>, m->L.bytes) | mgx_set_lds(k_assembly<T, 1, true>, m->L.bytes) |
         mgx_set_lds(k_assembly<T, 0, false>, m->L.bytes) | mgx_set_lds(k_assembly<T, 1, false>, m->L.bytes) |
         mgx_set_lds(k_assembly_logic<T>, m->L.bytes);
}

template <typename T, int MODE>
void launch(const mgx_model* m, const DevModel<T>& M, const mgx_state* s, const mgx_assembly_env* e, const float* action,
            float* obs, double* reward, uint8_t* term, uint8_t* trunc, float* final_obs, int autoreset, int n_env,
            const uint8_t* mask, hipStream_t st) {
  if (m->L.gB)
    hipLaunchKernelGGL((k_assembly<T, MODE, true>), dim3(n_env), dim3(kTeamThreads), m->L.bytes, st, M, m->as, *s, *e, action,
                       obs, reward, term, trunc, final_obs, autoreset, n_env, mask);
  else
    hipLaunchKernelGGL((k_assembly<T, MODE, false>), dim3(n_env), dim3(kTeamThreads), m->L.bytes, st, M, m->as, *s, *e, action,
                       obs, reward, term, trunc, final_obs, autoreset, n_env, mask);
}

int check_common(const mgx_model* m, const mgx_state* s, const mgx_assembly_env* e) {
  if (!m->assembly_ok) return fail(MGX_E_ARG, "mgx_assembly_configure not called");
  if (!assembly_env_ok(e)) return fail(MGX_E_ARG, "null assembly env buffer");
  if (s) {
    const int rc = host_check_state(s);
    if (rc) return rc;
    if (m->L.gB && !s->scratch) return fail(MGX_E_ARG, "this model needs mgx_state.scratch (scratch_bytes_per_env)");
  }
  return MGX_OK;
}

}  // namespace

extern "C" {

int mgx_assembly_configure(mgx_model* m, const mgx_assembly_ids* ids) {
  if (!m || !ids) return fail(MGX_E_ARG, "null argument");
  if (m->wide) return fail(MGX_E_UNSUPPORTED, MGX_WIDE_MSG);
  const bool f32 = m->precision == MGX_F32;
  const int nq = f32 ? m->mf.nq : m->md.nq, nu = f32 ? m->mf.nu : m->md.nu;
  const int nb = f32 ? m->mf.nbody : m->md.nbody, ng = f32 ? m->mf.ngeom : m->md.ngeom;
  if ((f32 ? m->mf.integrator : m->md.integrator) != 0)
    return fail(MGX_E_UNSUPPORTED, "the assembly kernels integrate with Euler (complete_model.xml:4)");
  if ((f32 ? m->mf.solver : m->md.solver) != 2)
    return fail(MGX_E_UNSUPPORTED, "the assembly kernels solve with Newton (complete_model.xml:4)");
  if (ids->max_episode_steps <= 0) return fail(MGX_E_ARG, "max_episode_steps must be > 0");
  if (ids->substeps < 1 || ids->settle_steps < 0) return fail(MGX_E_ARG, "substeps must be >= 1, settle_steps >= 0");
  if (nu != 9 || nq < 9) return fail(MGX_E_ARG, "assembly needs 9 actuators (7 motors, 2 finger servos) and nq >= 9");
  if (ids->n_geom != ng || ng > MGX_ASSEMBLY_MAX_GEOM) return fail(MGX_E_ARG, "n_geom must equal ngeom (<= 128)");
  if (ids->ee_body < 0 || ids->ee_body >= nb) return fail(MGX_E_ARG, "ee_site body id out of range");
  for (int c = 0; c < MGX_ASSEMBLY_NCOMP; c++)
    if (ids->comp_body[c] < 0 || ids->comp_body[c] >= nb) return fail(MGX_E_ARG, "component body id out of range");
  for (int g = 0; g < ng; g++)
    if (ids->geom_comp[g] < -1 || ids->geom_comp[g] >= MGX_ASSEMBLY_NCOMP) return fail(MGX_E_ARG, "geom_comp out of range");
  const int rc = f32 ? configure_lds<float>(m) : configure_lds<double>(m);
  if (rc != MGX_OK) return rc;
  m->as = *ids;
  m->assembly_ok = true;
  return MGX_OK;
}

int mgx_assembly_step(const mgx_model* m, const mgx_state* s, const mgx_assembly_env* e, const float* action, float* obs,
                      double* reward, uint8_t* terminated, uint8_t* truncated, float* final_obs, int autoreset,
                      int n_env, const uint8_t* mask, void* stream) {
  if (!m || !s || !e || !action || !obs || !reward || !terminated || !truncated) return fail(MGX_E_ARG, "null argument");
  if (e->action_f64 != 0 && e->action_f64 != 1) return fail(MGX_E_ARG, "action_f64 must be 0 (float32) or 1 (float64)");
  const int rc = check_common(m, s, e);
  if (rc) return rc;
  if (n_env <= 0) return MGX_OK;
  hipStream_t st = (hipStream_t)stream;
  if (m->precision == MGX_F32)
    launch<float, 0>(m, m->mf, s, e, action, obs, reward, terminated, truncated, final_obs, autoreset, n_env, mask, st);
  else
    launch<double, 0>(m, m->md, s, e, action, obs, reward, terminated, truncated, final_obs, autoreset, n_env, mask, st);
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}

int mgx_assembly_reset(const mgx_model* m, const mgx_state* s, const mgx_assembly_env* e, float* obs, int n_env,
                       const uint8_t* mask, void* stream) {
  if (!m || !s || !e || !obs) return fail(MGX_E_ARG, "null argument");
  const int rc = check_common(m, s, e);
  if (rc) return rc;
  if (n_env <= 0) return MGX_OK;
  hipStream_t st = (hipStream_t)stream;
  if (m->precision == MGX_F32)
    launch<float, 1>(m, m->mf, s, e, nullptr, obs, nullptr, nullptr, nullptr, nullptr, 0, n_env, mask, st);
  else
    launch<double, 1>(m, m->md, s, e, nullptr, obs, nullptr, nullptr, nullptr, nullptr, 0, n_env, mask, st);
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}

int mgx_assembly_logic_test(const mgx_model* m, const mgx_assembly_logic_io* io, const mgx_assembly_env* e, int n_env,
                            void* stream) {
  if (!m || !io || !e) return fail(MGX_E_ARG, "null argument");
  const int rc = check_common(m, nullptr, e);
  if (rc) return rc;
  if (io->max_contacts > m->L.max_ncon) return fail(MGX_E_CAPACITY, "max_contacts exceeds the contact capacity");
  if (n_env <= 0) return MGX_OK;
  hipStream_t st = (hipStream_t)stream;
  if (m->precision == MGX_F32)
    hipLaunchKernelGGL(k_assembly_logic<float>, dim3(n_env), dim3(64), m->L.bytes, st, m->mf, m->as, *io, *e, n_env);
  else
    hipLaunchKernelGGL(k_assembly_logic<double>, dim3(n_env), dim3(64), m->L.bytes, st, m->md, m->as, *io, *e, n_env);
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}

}  // extern "C"
