// mgx_step.hip — the generic physics kernels (mujoco.mj_step for any compiled model) and their
// C-ABI: mgx_step, mgx_reset_data, mgx_debug_forward / mgx_debug_layout (include/mgx.h).
//
// One 64-thread workgroup (= one wavefront) per environment. Variants are compile-time:
//   GB  the constraint rows B live in per-env global scratch (mgx_state.scratch) instead of
//       LDS, for models whose rows exceed the LDS budget (Layout.gB, e.g. bipedal_rescue);
//   RK  the model integrates with RK4 (mj_RungeKutta) instead of semi-implicit Euler.
#include "mgx_internal.h"

using namespace mgx;

MGX_PROF_SETTER(mgx_prof_set_buffer_step)

namespace {
int fail(int code, const std::string& msg) { return host_fail(code, msg); }
#define HIPCHK(x) MGX_HIPCHK(x)
int check_state(const mgx_state* s) { return host_check_state(s); }

// GB: B rows in global scratch (Layout.gB); RK: RK4 integrator
template <typename T, bool GB, bool RK, bool NT>
__global__ void __launch_bounds__(64) k_step(DevModel<T> m, mgx_state s, mgx_frames fr, int n_env, int nsub,
                                             const uint8_t* mask) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int env = blockIdx.x;
  if (env >= n_env) return;
  if (mask && !mask[env]) return;
  Env<T> e;
  env_bind<T, GB>(m, e, smem, GB ? (T*)s.scratch + (size_t)env * m.L.gB_stride : nullptr);
  T* qpos = (T*)s.qpos; T* qvel = (T*)s.qvel; T* qacc = (T*)s.qacc_warmstart; T* ctrl = (T*)s.ctrl;
  T* qfrc = (T*)s.qfrc_applied; T* xfrc = (T*)s.xfrc_applied; T* tm = (T*)s.time;
  load_state(m, e, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
  int warn = 0;
  for (int k = 0; k < nsub; k++) warn += mj_step_env<T, RK, NT>(m, e);
  store_state(m, e, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
  int l = lane_id();
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
}

template <typename T>
__global__ void k_reset(DevModel<T> m, mgx_state s, int n_env, const uint8_t* mask) {
  int env = blockIdx.x;
  if (env >= n_env || (mask && !mask[env])) return;
  int l = threadIdx.x;
  for (int k = l; k < m.nq; k += 64) ((T*)s.qpos)[(size_t)env * m.nq + k] = m.qpos0[k];
  for (int k = l; k < m.nv; k += 64) {
    ((T*)s.qvel)[(size_t)env * m.nv + k] = 0;
    ((T*)s.qacc_warmstart)[(size_t)env * m.nv + k] = 0;
    ((T*)s.qfrc_applied)[(size_t)env * m.nv + k] = 0;
  }
  for (int k = l; k < m.nu; k += 64) ((T*)s.ctrl)[(size_t)env * m.nu + k] = 0;
  for (int k = l; k < 6 * m.nbody; k += 64) ((T*)s.xfrc_applied)[(size_t)env * 6 * m.nbody + k] = 0;
  if (l == 0) ((T*)s.time)[env] = 0;
}

template <typename T, bool GB, bool NT>
__global__ void __launch_bounds__(64) k_debug_forward(DevModel<T> m, mgx_state s, int n_env, T* dbg, DbgOff o) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int env = blockIdx.x;
  if (env >= n_env) return;
  Env<T> e;
  env_bind<T, GB>(m, e, smem, GB ? (T*)s.scratch + (size_t)env * m.L.gB_stride : nullptr);
  load_state(m, e, (T*)s.qpos, (T*)s.qvel, (T*)s.qacc_warmstart, (T*)s.ctrl, (T*)s.qfrc_applied,
             (T*)s.xfrc_applied, (T*)s.time, env);
  T* D = dbg + (size_t)env * o.total;
  int l = lane_id();
  kinematics(m, e);
  com_crb(m, e);
  for (int k = l; k < m.nM; k += 64) D[o.qM + k] = e.qLD[k];
  wsync();
  e.diaginv = factor_ld(m, e, e.qLD);
  for (int k = l; k < m.nM; k += 64) D[o.qLD + k] = e.qLD[k];
  velocity(m, e);
  e.qacc_smooth = solve_M(m, e, e.qLD, e.diaginv, e.qfrc_smooth);
  // the phase-A arrays before collision: with rows in global scratch the contact arrays overlay
  // them from collision on (make_layout, mono_overlay)
  wsync();
  for (int k = l; k < 3 * m.nbody; k += 64) D[o.xipos + k] = e.xipos[k];
  for (int k = l; k < 10 * m.nbody; k += 64) D[o.cinert + k] = e.cinert[k];
  for (int k = l; k < 6 * m.nv; k += 64) D[o.cdof_dot + k] = e.cdof_dot[k];
  for (int k = l; k < 6 * m.nbody; k += 64) D[o.cvel + k] = e.cvel[k];
  wsync();
  collision(m, e);
  wsync();
  for (int k = l; k < 3 * m.ngeom; k += 64) D[o.geom_xpos + k] = e.geom_xpos[k];
  for (int k = l; k < 9 * m.ngeom; k += 64) D[o.geom_xmat + k] = e.geom_xmat[k];
  // contacts before the solve: with a Newton model in gB mode their frames share LDS with the
  // Hessian (make_layout)
  for (int c = l; c < e.ncon; c += 64) {
    D[o.con_dist + c] = e.con_dist[c];
    for (int k = 0; k < 3; k++) D[o.con_pos + 3 * c + k] = e.con_pos[3 * c + k];
    for (int k = 0; k < 9; k++) D[o.con_frame + 9 * c + k] = e.con_frame[9 * c + k];
    D[o.con_geom + 2 * c] = (T)e.con_geom[2 * c];
    D[o.con_geom + 2 * c + 1] = (T)e.con_geom[2 * c + 1];
  }
  wsync();
  make_constraint(m, e);
  if (l < m.nv) e.vec0[l] = sqrt(e.diaginv);
  wsync();
  transform_rows(m, e);
  wsync();
  for (int r = l; r < e.nefc; r += 64)
    for (int k = 0; k < m.nv; k++) D[o.Bmat + r * m.nv + k] = e.Bm[r * e.Bs + k];
  if constexpr (NT) newton(m, e);
  else pgs(m, e);
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
  if (l < m.nv) {
    D[o.qfrc_smooth + l] = e.qfrc_smooth; D[o.qacc_smooth + l] = e.qacc_smooth; D[o.qacc + l] = e.qacc;
    D[o.qfrc_constraint + l] = e.qfrc_constraint;
  }
}


template <typename T, bool GB, bool RK>
int set_step_lds(const mgx_model* m) {
  return mgx_set_lds(k_step<T, GB, RK, false>, m->L.bytes) | mgx_set_lds(k_step<T, GB, RK, true>, m->L.bytes);
}

// NT (Newton solver) is chosen from the model at launch
template <typename T, bool GB, bool RK>
void launch_step_v(const mgx_model* m, const DevModel<T>& M, const mgx_state* s, const mgx_frames& fr, int n_env,
                   int nsub, const uint8_t* mask, hipStream_t st) {
  if (M.solver == 2)
    hipLaunchKernelGGL((k_step<T, GB, RK, true>), dim3(n_env), dim3(64), m->L.bytes, st, M, *s, fr, n_env, nsub, mask);
  else
    hipLaunchKernelGGL((k_step<T, GB, RK, false>), dim3(n_env), dim3(64), m->L.bytes, st, M, *s, fr, n_env, nsub, mask);
}

template <typename T>
int launch_step(const mgx_model* m, const DevModel<T>& M, const mgx_state* s, const mgx_frames& fr, int n_env, int nsub,
                const uint8_t* mask, hipStream_t st) {
  bool rk = M.integrator == 1;
  if (m->L.gB && rk) launch_step_v<T, true, true>(m, M, s, fr, n_env, nsub, mask, st);
  else if (m->L.gB) launch_step_v<T, true, false>(m, M, s, fr, n_env, nsub, mask, st);
  else if (rk) launch_step_v<T, false, true>(m, M, s, fr, n_env, nsub, mask, st);
  else launch_step_v<T, false, false>(m, M, s, fr, n_env, nsub, mask, st);
  return MGX_OK;
}

template <typename T, bool GB>
void launch_debug_v(const mgx_model* m, const DevModel<T>& M, const mgx_state* s, int n_env, T* dbg, DbgOff o,
                    hipStream_t st) {
  if (M.solver == 2)
    hipLaunchKernelGGL((k_debug_forward<T, GB, true>), dim3(n_env), dim3(64), m->L.bytes, st, M, *s, n_env, dbg, o);
  else
    hipLaunchKernelGGL((k_debug_forward<T, GB, false>), dim3(n_env), dim3(64), m->L.bytes, st, M, *s, n_env, dbg, o);
}

}  // namespace

namespace mgx {
// dynamic-LDS attributes of the generic kernels (called by mgx_model_create)
int step_kernels_configure(const mgx_model* m) {
  if (m->precision == MGX_F32)
    return set_step_lds<float, false, false>(m) | set_step_lds<float, false, true>(m) |
           set_step_lds<float, true, false>(m) | set_step_lds<float, true, true>(m) |
           mgx_set_lds(k_debug_forward<float, false, false>, m->L.bytes) | mgx_set_lds(k_debug_forward<float, true, false>, m->L.bytes) |
           mgx_set_lds(k_debug_forward<float, false, true>, m->L.bytes) | mgx_set_lds(k_debug_forward<float, true, true>, m->L.bytes);
  return set_step_lds<double, false, false>(m) | set_step_lds<double, false, true>(m) |
         set_step_lds<double, true, false>(m) | set_step_lds<double, true, true>(m) |
         mgx_set_lds(k_debug_forward<double, false, false>, m->L.bytes) | mgx_set_lds(k_debug_forward<double, true, false>, m->L.bytes) |
         mgx_set_lds(k_debug_forward<double, false, true>, m->L.bytes) | mgx_set_lds(k_debug_forward<double, true, true>, m->L.bytes);
}
}  // namespace mgx

extern "C" {

int mgx_step(const mgx_model* m, const mgx_state* s, mgx_frames* frames, int n_env, int nsub, const uint8_t* mask,
             void* stream) {
  if (!m || n_env < 0 || nsub < 0) return fail(MGX_E_ARG, "bad argument");
  int rc = check_state(s);
  if (rc) return rc;
  if (n_env == 0 || nsub == 0) return MGX_OK;
  mgx_frames fr{};
  if (frames) fr = *frames;
  if (m->L.gB && !s->scratch) return fail(MGX_E_ARG, "this model needs mgx_state.scratch (scratch_bytes_per_env)");
  hipStream_t st = (hipStream_t)stream;
  if (m->wide) return wide_step(m, s, fr, n_env, nsub, mask, st);
  if (m->precision == MGX_F32) launch_step<float>(m, m->mf, s, fr, n_env, nsub, mask, st);
  else launch_step<double>(m, m->md, s, fr, n_env, nsub, mask, st);
  HIPCHK(hipGetLastError());
  return MGX_OK;
}

int mgx_reset_data(const mgx_model* m, const mgx_state* s, int n_env, const uint8_t* mask, void* stream) {
  if (!m || n_env < 0) return fail(MGX_E_ARG, "bad argument");
  int rc = check_state(s);
  if (rc) return rc;
  if (n_env == 0) return MGX_OK;
  hipStream_t st = (hipStream_t)stream;
  if (m->precision == MGX_F32) hipLaunchKernelGGL(k_reset<float>, dim3(n_env), dim3(64), 0, st, m->mf, *s, n_env, mask);
  else hipLaunchKernelGGL(k_reset<double>, dim3(n_env), dim3(64), 0, st, m->md, *s, n_env, mask);
  HIPCHK(hipGetLastError());
  return MGX_OK;
}

int mgx_debug_layout(const mgx_model* m, int32_t* offsets, int32_t n) {
  if (!m || !offsets) return fail(MGX_E_ARG, "null argument");
  int nb = m->precision == MGX_F32 ? m->mf.nbody : m->md.nbody;
  int nv = m->precision == MGX_F32 ? m->mf.nv : m->md.nv;
  int nM = m->precision == MGX_F32 ? m->mf.nM : m->md.nM;
  int ng = m->precision == MGX_F32 ? m->mf.ngeom : m->md.ngeom;
  DbgOff o = dbg_offsets(nb, nv, nM, ng, m->L.max_ncon, m->L.max_nefc);
  const int* src = (const int*)&o;
  int cnt = (int)(sizeof(DbgOff) / sizeof(int));
  for (int i = 0; i < n && i < cnt; i++) offsets[i] = src[i];
  return cnt;
}

int mgx_debug_forward(const mgx_model* m, const mgx_state* s, int n_env, void* dbg, void* stream) {
  if (!m || !dbg) return fail(MGX_E_ARG, "null argument");
  int rc = check_state(s);
  if (rc) return rc;
  if (n_env <= 0) return MGX_OK;
  if (m->L.gB && !s->scratch) return fail(MGX_E_ARG, "this model needs mgx_state.scratch (scratch_bytes_per_env)");
  hipStream_t st = (hipStream_t)stream;
  if (m->wide) {
    DbgOff o = m->precision == MGX_F32
                   ? dbg_offsets(m->mf.nbody, m->mf.nv, m->mf.nM, m->mf.ngeom, m->L.max_ncon, m->L.max_nefc)
                   : dbg_offsets(m->md.nbody, m->md.nv, m->md.nM, m->md.ngeom, m->L.max_ncon, m->L.max_nefc);
    return wide_debug(m, s, n_env, dbg, o, st);
  }
  if (m->precision == MGX_F32) {
    DbgOff o = dbg_offsets(m->mf.nbody, m->mf.nv, m->mf.nM, m->mf.ngeom, m->L.max_ncon, m->L.max_nefc);
    if (m->L.gB) launch_debug_v<float, true>(m, m->mf, s, n_env, (float*)dbg, o, st);
    else launch_debug_v<float, false>(m, m->mf, s, n_env, (float*)dbg, o, st);
  } else {
    DbgOff o = dbg_offsets(m->md.nbody, m->md.nv, m->md.nM, m->md.ngeom, m->L.max_ncon, m->L.max_nefc);
    if (m->L.gB) launch_debug_v<double, true>(m, m->md, s, n_env, (double*)dbg, o, st);
    else launch_debug_v<double, false>(m, m->md, s, n_env, (double*)dbg, o, st);
  }
  HIPCHK(hipGetLastError());
  return MGX_OK;
}

}  // extern "C"
