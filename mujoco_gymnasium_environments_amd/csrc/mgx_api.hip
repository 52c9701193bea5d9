// mgx_api.hip — kernels and the C-ABI of libmgx.so (declared in include/mgx.h).
//
// Launch geometry: one 64-thread workgroup (= one wavefront) per environment, dynamic LDS
// sized from the model (Layout). Kernels never allocate; all state is caller-owned.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "mgx_internal.h"

using namespace mgx;

MGX_PROF_SETTER(mgx_prof_set_buffer)

namespace {
thread_local std::string g_err;
int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(x) MGX_HIPCHK(x)
}  // namespace

namespace mgx {
int host_fail(int code, const std::string& msg) { return fail(code, msg); }
}  // namespace mgx

// ------------------------------------------------------------------------- kernels
// soccer reset body shared by the explicit-reset and autoreset paths: draws (36 values in
// reference order, from the host or from Philox) -> randomised qpos, 10 settle mj_steps, obs.
template <typename T>
__device__ __forceinline__ int soccer_reset_body(const DevModel<T>& m, Env<T>& e, const SoccerIds<T>& ids, const T* draws, T* wind,
                                 T* prev_ball, T* prev_robot, T* stats, int* step, uint8_t* goal, float* obs) {
  soccer_apply_reset(m, e, ids, draws, wind);
  int warn = 0;
  for (int k = 0; k < 10; k++) warn += mj_step_env(m, e);  // soccer_env.py:378-379
  soccer_obs(m, e, ids, 0, obs);
  wsync();
  int l = lane_id();
  if (l < 3) { prev_ball[l] = e.xpos[3 * ids.ball + l]; prev_robot[l] = e.xpos[3 * ids.torso + l]; }
  if (l < 5) stats[l] = 0;
  if (l == 0) { *step = 0; *goal = 0; }
  return warn;
}

// Philox-drawn reset of `env` for its current episode counter, then the counter advances;
// with banks, the bank of the consumed episode restarts for episode + R. Writes the state.
template <typename T>
__device__ __forceinline__ void soccer_reset_philox(const DevModel<T>& m, Env<T>& e, const SoccerIds<T>& ids, mgx_state s,
                                                    mgx_soccer_env ev, float* obs, uint64_t seed, int env_offset, int env,
                                                    const Pipe* P) {
  int l = lane_id();
  int E = ev.episode[env];
  soccer_philox_draws(seed, (uint32_t)(env_offset + env), (uint32_t)E, ids.n_noise, e.vec1);
  wsync();
  int warn = soccer_reset_body(m, e, ids, e.vec1, (T*)ev.wind + 3 * (size_t)env, (T*)ev.prev_ball_pos + 3 * (size_t)env,
                               (T*)ev.prev_robot_pos + 3 * (size_t)env, (T*)ev.stats + 5 * (size_t)env, ev.step + env,
                               ev.goal_scored + env, obs + (size_t)env * 80);
  store_state(m, e, (T*)s.qpos, (T*)s.qvel, (T*)s.qacc_warmstart, (T*)s.ctrl, (T*)s.qfrc_applied, (T*)s.xfrc_applied,
              (T*)s.time, env);
  if (l == 0) {
    if (s.warning) s.warning[env] += warn;
    if (s.overflow && e.overflow) s.overflow[env] += 1;
    ev.episode[env] = E + 1;
  }
  wsync();
  if (P) bank_init(m, e, ids, *P, env, E % P->R, E + P->R, seed, env_offset);
}

// One full soccer step of `env` in one wave (pre, mj_step, post, same-step autoreset).
template <typename T>
__device__ __forceinline__ void soccer_step_mono(const DevModel<T>& m, Env<T>& e, const SoccerIds<T>& ids, mgx_state s,
                                                 mgx_soccer_env ev, const float* action, float* obs, double* reward,
                                                 uint8_t* terminated, uint8_t* truncated, float* final_obs, int autoreset,
                                                 uint64_t seed, int env_offset, int env, const Pipe* P) {
  T* qpos = (T*)s.qpos; T* qvel = (T*)s.qvel; T* qacc = (T*)s.qacc_warmstart; T* ctrl = (T*)s.ctrl;
  T* qfrc = (T*)s.qfrc_applied; T* xfrc = (T*)s.xfrc_applied; T* tm = (T*)s.time;
  load_state(m, e, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
  T* prev_ball = (T*)ev.prev_ball_pos + 3 * (size_t)env;
  float* o = obs + (size_t)env * 80;
  int l = lane_id();
  const SoccerAct a(action, ev.action_f64, env, m.nu);
  soccer_pre(m, e, ids, a, prev_ball, (T*)ev.wind + 3 * (size_t)env);
  int warn = mj_step_env(m, e);
  bool done = soccer_post(m, e, ids, a, ev.step + env, ev.goal_scored + env, prev_ball,
                          (T*)ev.prev_robot_pos + 3 * (size_t)env, (T*)ev.stats + 5 * (size_t)env, o, reward + env,
                          terminated + env, truncated + env, ev.flags ? ev.flags + 2 * (size_t)env : nullptr);
  if (ev.rollout && l == 0) {
    double* ro = (double*)ev.rollout + 8 * (size_t)env;
    const double ne = e.nefc, it = e.niter;
    ro[0] += reward[env];
    ro[1] += terminated[env];
    ro[2] += truncated[env];
    ro[3] += 1.0;
    ro[4] += ne;
    ro[5] += it;
    ro[6] += ne * ne;
    ro[7] += it * ne * ne;
  }
  store_state(m, e, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
  if (l == 0 && s.warning) s.warning[env] += warn;
  if (l == 0 && s.overflow && e.overflow) s.overflow[env] += 1;
  if (done && autoreset) {
    if (final_obs)
      for (int i = l; i < 80; i += 64) final_obs[(size_t)env * 80 + i] = o[i];
    __threadfence();
    wsync();
    if (!(P && bank_install(m, e, ids, *P, s, ev, obs, seed, env_offset, env)))
      soccer_reset_philox(m, e, ids, s, ev, obs, seed, env_offset, env, P);
  }
}

// soccer, monolithic (one wave per env): MODE 0 = step (+ optional same-step autoreset), MODE 1 =
// reset. A staged batch (workspace) resets through k_soccer_settle instead (mgx_staged.h).
template <typename T, int MODE>
__global__ void __launch_bounds__(64) k_soccer(DevModel<T> m, SoccerIds<T> ids, mgx_state s, mgx_soccer_env ev,
                                               const float* action, const T* draws, float* obs, double* reward,
                                               uint8_t* terminated, uint8_t* truncated, float* final_obs,
                                               int autoreset, uint64_t seed, int env_offset, int n_env,
                                               const uint8_t* mask, Pipe pipe, int use_pipe) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int env = blockIdx.x;
  if (env >= n_env) return;
  if (mask && !mask[env]) return;
  Env<T> e;
  env_bind(m, e, smem);
  const Pipe* P = use_pipe ? &pipe : nullptr;
  if (MODE == 0) {
    soccer_step_mono(m, e, ids, s, ev, action, obs, reward, terminated, truncated, final_obs, autoreset, seed,
                     env_offset, env, P);
    return;
  }
  if (!draws) {
    soccer_reset_philox(m, e, ids, s, ev, obs, seed, env_offset, env, nullptr);
    return;
  }
  T* qpos = (T*)s.qpos; T* qvel = (T*)s.qvel; T* qacc = (T*)s.qacc_warmstart; T* ctrl = (T*)s.ctrl;
  T* qfrc = (T*)s.qfrc_applied; T* xfrc = (T*)s.xfrc_applied; T* tm = (T*)s.time;
  load_state(m, e, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
  int warn = soccer_reset_body(m, e, ids, draws + (size_t)env * 36, (T*)ev.wind + 3 * (size_t)env,
                               (T*)ev.prev_ball_pos + 3 * (size_t)env, (T*)ev.prev_robot_pos + 3 * (size_t)env,
                               (T*)ev.stats + 5 * (size_t)env, ev.step + env, ev.goal_scored + env,
                               obs + (size_t)env * 80);
  if (ev.episode && lane_id() == 0) ev.episode[env] += 1;
  store_state(m, e, qpos, qvel, qacc, ctrl, qfrc, xfrc, tm, env);
  if (lane_id() == 0 && s.warning) s.warning[env] += warn;
  if (lane_id() == 0 && s.overflow && e.overflow) s.overflow[env] += 1;
}

// mj_step from mj_resetData'd state (the checkAcc template, see load_template)
template <typename T>
__global__ void __launch_bounds__(64) k_soccer_template(DevModel<T> m, Pipe P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Env<T> e;
  env_bind(m, e, smem);
  int l = lane_id();
  reset_env(m, e);
  forward(m, e);
  e.qacc_ws = e.qacc;
  euler(m, e);
  for (int k = l; k < m.nq; k += 64) P.at<T>(P.o_tq)[k] = e.qpos[k];
  for (int k = l; k < m.nv; k += 64) { P.at<T>(P.o_tv)[k] = e.qvel[k]; }
  if (l < m.nv) P.at<T>(P.o_ta)[l] = e.qacc_ws;
  for (int k = l; k < 3 * m.nbody; k += 64) { P.at<T>(P.o_tx)[k] = e.xpos[k]; P.at<T>(P.o_tsc)[k] = e.subtree_com[k]; }
  for (int k = l; k < 4 * m.nbody; k += 64) P.at<T>(P.o_txq)[k] = e.xquat[k];
  int nc = e.ncon < P.maxC ? e.ncon : P.maxC;
  for (int k = l; k < nc; k += 64) {
    P.at<int>(P.o_tcg)[2 * k] = e.con_geom[2 * k];
    P.at<int>(P.o_tcg)[2 * k + 1] = e.con_geom[2 * k + 1];
    P.at<T>(P.o_tcd)[k] = e.con_dist[k];
    P.at<T>(P.o_tcm)[k] = e.con_mu[k];
  }
  if (l == 0) { P.at<int>(P.o_tn)[0] = nc; P.at<T>(P.o_tt)[0] = e.time; }
}

// Env-logic-only test hook: frames/contacts come from the caller (golden vectors generated
// from the reference's own Python), no physics is run.
template <typename T>
__global__ void __launch_bounds__(64) k_soccer_logic(DevModel<T> m, SoccerIds<T> ids, mgx_soccer_logic_io io,
                                                     int n_env) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int env = blockIdx.x;
  if (env >= n_env) return;
  Env<T> e;
  env_bind(m, e, smem);
  int l = lane_id();
  const T* qpos = (const T*)io.qpos + (size_t)env * m.nq;
  const T* qvel = (const T*)io.qvel + (size_t)env * m.nv;
  for (int k = l; k < m.nq; k += 64) e.qpos[k] = qpos[k];
  for (int k = l; k < m.nv; k += 64) e.qvel[k] = qvel[k];
  for (int k = l; k < 3 * m.nbody; k += 64) {
    e.xpos[k] = ((const T*)io.xpos)[(size_t)env * 3 * m.nbody + k];
    e.subtree_com[k] = ((const T*)io.subtree_com)[(size_t)env * 3 * m.nbody + k];
  }
  for (int k = l; k < 4 * m.nbody; k += 64) e.xquat[k] = ((const T*)io.xquat)[(size_t)env * 4 * m.nbody + k];
  for (int k = l; k < 6 * m.nbody; k += 64) e.xfrc[k] = ((T*)io.xfrc_applied)[(size_t)env * 6 * m.nbody + k];
  e.qfrc_applied = l < m.nv ? ((T*)io.qfrc_applied)[(size_t)env * m.nv + l] : (T)0;
  int nc = io.ncon[env];
  e.ncon = nc;
  for (int c = l; c < nc; c += 64) {
    e.con_geom[2 * c] = io.con_geom[((size_t)env * io.max_contacts + c) * 2];
    e.con_geom[2 * c + 1] = io.con_geom[((size_t)env * io.max_contacts + c) * 2 + 1];
    e.con_dist[c] = ((const T*)io.con_dist)[(size_t)env * io.max_contacts + c];
    e.con_mu[c] = ((const T*)io.con_mu)[(size_t)env * io.max_contacts + c];
  }
  wsync();
  const T* stale = (const T*)io.xpos + (size_t)env * 3 * m.nbody + 3 * ids.ball;
  const SoccerAct a(io.action, 0, env, m.nu);
  soccer_pre(m, e, ids, a, stale, (const T*)io.wind + 3 * (size_t)env);
  soccer_post(m, e, ids, a, io.step + env, io.goal_scored + env, (T*)io.prev_ball_pos + 3 * (size_t)env,
              (T*)io.prev_robot_pos + 3 * (size_t)env, (T*)io.stats + 5 * (size_t)env, io.obs + (size_t)env * 80,
              io.reward + env, io.terminated + env, io.truncated + env, io.flags + 2 * (size_t)env);
  wsync();
  if (l < m.nv) ((T*)io.qfrc_applied)[(size_t)env * m.nv + l] = e.qfrc_applied;
  for (int k = l; k < 6 * m.nbody; k += 64) ((T*)io.xfrc_applied)[(size_t)env * 6 * m.nbody + k] = e.xfrc[k];
}

// ------------------------------------------------------------------------- host side
namespace {

int align_up(int x, int a) { return (x + a - 1) / a * a; }

Layout make_layout(const mgx_model_desc* d, int real_bytes, int max_ncon, int max_nefc, int max_active,
                   bool gB = false) {
  Layout L{};
  int p = 0;
  int al = 16 / real_bytes;  // 16-byte alignment in elements
  auto take = [&](int n) { int r = p; p = align_up(p + (n > 0 ? n : 1), al); return r; };
  int nb = d->nbody, nv = d->nv, nj = d->njnt, ng = d->ngeom;
  L.max_ncon = max_ncon; L.max_nefc = max_nefc; L.max_active = max_active;
  // carry: state + frames read by env logic + factors + contacts (the finisher's inputs)
  L.qpos = take(d->nq); L.qvel = take(nv); L.ctrl = take(d->nu); L.xfrc = take(6 * nb);
  L.xpos = take(3 * nb); L.xquat = take(4 * nb); L.subtree_com = take(3 * nb);
  L.qLD = take(d->nM); L.qMH = take(d->nM); L.con_dist = take(max_ncon); L.con_mu = take(max_ncon);
  L.carry_reals = p;
  L.carry_lds = p;
  L.cfs = 9;
  const int nvw = nv > 64 ? 128 : 64;  // dof-indexed scratch vectors: one or two dofs per lane
  L.vec0 = take(nvw); L.vec1 = take(nvw); L.vec2 = take(nvw); L.vec3 = take(nvw);
  int vec_end = p;
  L.rk = d->integrator == 1 ? take(((d->nq + 3) & ~3) + nvw) : 0;
  // persistent for the rest of the forward pass
  // Newton with rows in global scratch (gB): the Hessian / its factor overlay the phase-A union,
  // dead from the row transform on (newton() is its only user; no env logic reads a union array
  // after the solve), and the contact frames sit in the Hessian's tail beyond the phase-A arrays
  // (live from collision to make_constraint only). The PGS block table is not allocated.
  // Assembly (fp64, 384 rows, 96 contacts): 113 -> 80 KiB per env, two envs per CU.
  const bool hess_union = gB && d->solver == 2;
  L.cdof = take(6 * nv);
  const int cf9 = align_up(9 * max_ncon, al), cp3 = align_up(3 * max_ncon, al);
  const int union_dead = align_up(9 * nb, al) + align_up(3 * nb, al) + align_up(9 * nb, al) + align_up(10 * nb, al) +
                         align_up(10 * nb, al) + align_up(6 * nb, al) + align_up(6 * nv, al) + 2 * align_up(3 * nj, al);
  // monolithic PGS models with rows in global scratch: the contact points / frames, the row
  // margins (make_constraint only) and the broadphase survivor list (collision only) overlay
  // xmat .. xanchor of the union, dead once the velocity stage is done (bipedal: 62.4 -> 51.4 KiB,
  // three envs per CU instead of two)
  const int cvel_sz = align_up(6 * nb, al);
  const int act_r = align_up((max_active * 4 + real_bytes - 1) / real_bytes, al);
  const bool mono_overlay = gB && !hess_union && !(d->layout_flags & MGX_KEEP_CVEL) &&
                            cp3 + cf9 + align_up(max_nefc, al) + act_r <= union_dead + cvel_sz;
  if (!hess_union && !mono_overlay) { L.con_pos = take(3 * max_ncon); L.con_frame = take(9 * max_ncon); }
  // wide Newton models: efc / efc_margin in global scratch (gb_efc_off), the Hessian packed lower
  const bool efcg = gB && nv > 64 && d->solver == 2;
  L.efc = take(efcg ? 1 : 8 * max_nefc); L.efc_margin = take(mono_overlay || efcg ? 1 : max_nefc);
  L.efc_blk = take(hess_union ? 1 : 2 * max_nefc);
  L.hess = (d->solver == 2 && !hess_union) ? take(nv * nv) : 0;
  // env logic that reads cvel after the step (martial arts, martial_arts_env.py:536-589) keeps
  // it out of the union the constraint rows overwrite
  const bool keep_cvel = (d->layout_flags & MGX_KEEP_CVEL) != 0;
  if (keep_cvel) L.cvel = take(6 * nb);
  // union: phase A (kinematics .. collision) arrays, then B rows on top
  int u0 = p;
  L.xmat = take(9 * nb); L.xipos = take(3 * nb); L.ximat = take(9 * nb); L.cinert = take(10 * nb);
  L.crb = take(10 * nb);
  if (!keep_cvel) L.cvel = take(6 * nb);
  L.cfrc = take(6 * nb); L.cdof_dot = take(6 * nv);
  L.xaxis = take(3 * nj); L.xanchor = take(3 * nj); L.geom_xpos = take(3 * ng); L.geom_xmat = take(9 * ng);
  L.act_force = take(d->nu);
  int endA = p;
  L.act_union = 0;
  if (mono_overlay) {
    int o = u0;
    L.con_pos = o; o += cp3;
    L.con_frame = o; o += cf9;
    L.efc_margin = o; o += align_up(max_nefc, al);
    L.act_union = o;
  }
  L.rowc = 0;
  L.Bstride = nv | 1;  // odd stride: lane-per-row access is bank-conflict free
  L.Bmat = u0;
  L.chunk_rows = max_nefc;
  if (gB) {  // rows in per-env global scratch
    L.gB = 1;
    L.gB_stride = align_up(max_nefc * L.Bstride, al);
    L.chunk_rows = 0;
    if (efcg) {  // then efc, efc_margin (the device derives the same offsets)
      L.gB_stride = gb_efm_off(L, real_bytes) + align_up(max_nefc, al);
      if (gb_efc_off(L, real_bytes) != align_up(max_nefc * L.Bstride, al)) abort();
    }
  }
  // gB: the row transform stages up to 64 rows at a time in the phase-A union (dead by then)
  L.tchunk = L.gB ? std::min(64, (endA - u0) / L.Bstride) : 0;
  if (hess_union) {
    L.hess = u0;
    L.con_pos = endA;
    L.con_frame = align_up(L.con_pos + 3 * max_ncon, al);
    endA = std::max(align_up(L.con_frame + 9 * max_ncon, al), align_up(u0 + (efcg ? nv * (nv + 1) / 2 : nv * nv), al));
  }
  int endB = align_up(u0 + L.chunk_rows * L.Bstride, al);
  L.reals = endA > endB ? endA : endB;
  int q = 0;
  auto takei = [&](int n) { int r = q; q = align_up(q + (n > 0 ? n : 1), 4); return r; };
  L.con_geom = takei(2 * max_ncon);
  L.carry_ints = q;
  L.con_pair = takei(max_ncon);
  L.act_list = takei(max_active);
  L.efc_type = takei(max_nefc); L.efc_id = takei(max_nefc);
  L.con_efcadr = takei(1);
  if (d->solver == 2 && takei(4) != team_off(L)) abort();  // Newton models: the helper-wave command words
  L.ints = q;
  L.bytes = L.reals * real_bytes + L.ints * 4;
  (void)vec_end;
  return L;
}

// The staged row builder (k_soccer_rows, k_rk_rows, the row stage of the settle kernels): the
// per-slot working set by liveness, so more row-builder waves share a CU (LDS-bound: 160 KiB / CU).
//   carry: the finisher's inputs; xfrc_applied and qMH (written once, read by the finisher or
//          once per step) sit in the slot's pipe carry in global memory, not in LDS (carry_lds);
//   cvel:  velocity stage -> row blocks;
//   region R, three lives: phase A (kinematics .. velocity) xipos / cinert / crb live throughout,
//          xmat / ximat / xaxis / xanchor until com_crb, then cdof_dot / cfrc / act_force and an
//          LDS copy of xfrc_applied over them; phase C (collision): the geom poses (computed from xquat just before collision,
//          geom_poses) + contact normals / points + the broadphase list (later efc_id);
//          phase D (row blocks): cacc over the geom poses.
// fp64 soccer, default capacity (64 contacts, 192 rows): 31.7 -> 19.7 KB per row-builder wave,
// eight waves per CU instead of five (the VGPR limit of the row builder is also eight).
Layout make_staged_layout(const mgx_model_desc* d, int real_bytes, int max_ncon, int max_nefc, int max_active,
                          int gcon) {
  Layout L{};
  int p = 0;
  const int al = 16 / real_bytes;
  auto a = [&](int n) { return align_up(n > 0 ? n : 1, al); };
  auto take = [&](int n) { int r = p; p += a(n); return r; };
  const int nb = d->nbody, nv = d->nv, nj = d->njnt, ng = d->ngeom;
  L.max_ncon = max_ncon; L.max_nefc = max_nefc; L.max_active = max_active;
  L.staged = 1;
  L.late_geom = 1;
  L.cfs = 3;
  L.qpos = take(d->nq); L.qvel = take(nv); L.ctrl = take(d->nu);
  L.xpos = take(3 * nb); L.xquat = take(4 * nb); L.subtree_com = take(3 * nb);
  L.qLD = take(d->nM); L.con_dist = take(max_ncon);
  L.carry_lds = p;
  L.con_mu = take(max_ncon); L.xfrc = take(6 * nb); L.qMH = take(d->nM);
  L.carry_reals = p;
  p = L.carry_lds;  // the row builder's LDS continues after the LDS part of the carry
  const int nvw = nv > 64 ? 128 : 64;
  L.vec0 = take(nvw); L.vec1 = take(nvw); L.vec2 = take(nvw); L.vec3 = take(nvw);
  L.cdof = take(6 * nv);
  L.efc = take(1); L.efc_margin = take(1); L.efc_blk = take(1);
  L.cvel = take(6 * nb);
  const int R = p;
  // phase A
  L.xipos = R; L.cinert = L.xipos + a(3 * nb); L.crb = L.cinert + a(10 * nb);
  const int dead = L.crb + a(10 * nb);
  L.xmat = dead; L.ximat = L.xmat + a(9 * nb); L.xaxis = L.ximat + a(9 * nb); L.xanchor = L.xaxis + a(3 * nj);
  const int endA1 = L.xanchor + a(3 * nj);
  L.cdof_dot = dead; L.cfrc = L.cdof_dot + a(6 * nv); L.act_force = L.cfrc + a(6 * nb);
  L.xfrc_lds = L.act_force + a(d->nu);
  const int endA2 = L.xfrc_lds + a(6 * nb);
  // phase C
  const int ecap = std::min(max_nefc, align_up(2 * nj, 4));  // efc_id: the joint-limit rows only
  const int nlist = std::max(max_active, ecap);
  L.geom_xpos = R; L.geom_xmat = L.geom_xpos + a(3 * ng);
  L.con_frame = L.geom_xmat + a(9 * ng);
  // the contact points live in the pipe (Pipe.o_cpos) unless gcon = 0 (MGX_GCON=0, A/B: in phase
  // C's LDS)
  L.gcon = gcon;
  L.con_pos = gcon ? 0 : L.con_frame + a(3 * max_ncon);
  L.act_union = L.con_frame + a(3 * max_ncon) + (gcon ? 0 : a(3 * max_ncon));
  const int endC = L.act_union + a((nlist * 4 + real_bytes - 1) / real_bytes);
  // phase D: cacc (12 per body) over the geom poses when they cover it, else after phase C
  L.cacc = a(12 * nb) <= L.con_frame - R ? R : endC;
  const int endD = L.cacc + a(12 * nb);
  L.reals = std::max(std::max(endA1, endA2), std::max(endC, endD));
  L.rowc = 0; L.rk = 0; L.hess = 0;
  L.Bstride = nv | 1; L.Bmat = R; L.chunk_rows = 0; L.gB = 0; L.gB_stride = 0; L.tchunk = 0;
  int q = 0;
  auto takei = [&](int n) { int r = q; q = align_up(q + (n > 0 ? n : 1), 4); return r; };
  L.con_geom = takei(2 * max_ncon);
  L.carry_ints = q;
  L.con_pair = takei(max_ncon);
  L.act_list = 0; L.efc_id = 0;  // both at act_union (env_bind)
  L.efc_type = takei(1);
  L.con_efcadr = takei(1);
  L.ints = q;
  L.bytes = L.reals * real_bytes + L.ints * 4;
  return L;
}

// The finisher binds the staged carry (all of it in LDS) and the four scratch vectors after it.
Layout finisher_layout(const Layout& S, int real_bytes) {
  Layout L = S;
  const int nvw = S.vec1 - S.vec0;
  L.vec0 = S.carry_reals; L.vec1 = L.vec0 + nvw; L.vec2 = L.vec1 + nvw; L.vec3 = L.vec2 + nvw;
  L.carry_lds = S.carry_reals;
  L.reals = L.vec3 + nvw;
  L.ints = S.carry_ints;
  L.bytes = L.reals * real_bytes + L.ints * 4;
  return L;
}

template <typename T>
struct Builder {
  std::vector<char> host;
  std::vector<std::pair<size_t, const void**>> fix;  // (offset, pointer slot)
  size_t add(const void* src, size_t bytes, const void** slot) {
    size_t off = (host.size() + 15) / 16 * 16;
    host.resize(off + (bytes ? bytes : 16));
    if (bytes) memcpy(host.data() + off, src, bytes);
    fix.push_back({off, slot});
    return off;
  }
  template <typename S>
  void ints(const S* src, size_t n, const int** slot) {
    std::vector<int> v(n ? n : 1, 0);
    for (size_t i = 0; i < n; i++) v[i] = (int)src[i];
    add(v.data(), v.size() * 4, (const void**)slot);
  }
  void reals(const double* src, size_t n, const T** slot) {
    std::vector<T> v(n ? n : 1, (T)0);
    for (size_t i = 0; i < n; i++) v[i] = (T)src[i];
    add(v.data(), v.size() * sizeof(T), (const void**)slot);
  }
};

template <typename T>
int build_model(const mgx_model_desc* d, int device, mgx_model* out, DevModel<T>& M) {
  Builder<T> B;
  int nb = d->nbody, nv = d->nv, nj = d->njnt, ng = d->ngeom, np = d->npair, nu = d->nu;
  M.nq = d->nq; M.nv = nv; M.nu = nu; M.nbody = nb; M.njnt = nj; M.ngeom = ng; M.npair = np; M.nM = d->nM;
  M.nmaskword = d->nmaskword; M.solver = d->solver; M.integrator = d->integrator; M.cone = d->cone;
  M.iterations = d->iterations;
  M.timestep = (T)d->timestep; M.tolerance = (T)d->tolerance; M.impratio = (T)d->impratio;
  M.meaninertia = (T)d->meaninertia;
  for (int k = 0; k < 3; k++) M.gravity[k] = (T)d->gravity[k];
  // derived tables: body chains, dof ancestors
  std::vector<int> chain(nb * MGX_MAX_DEPTH, 0), depth(nb, 0);
  for (int b = 1; b < nb; b++) {
    std::vector<int> path;
    for (int i = b; i > 0; i = d->body_parentid[i]) path.push_back(i);
    if ((int)path.size() > MGX_MAX_DEPTH) return fail(MGX_E_CAPACITY, "body tree deeper than MGX_MAX_DEPTH");
    depth[b] = (int)path.size();
    for (int c = 0; c < depth[b]; c++) chain[b * MGX_MAX_DEPTH + c] = path[depth[b] - 1 - c];
  }
  std::vector<int> chainlen(nv), anc(nv * MGX_MAX_DEPTH, -1), ancadr(nv * MGX_MAX_DEPTH, 0);
  std::vector<uint64_t> ancmask(nv, 0), ancmask_hi(nv, 0);
  for (int k = 0; k < nv; k++) {
    int t = 0;
    for (int j = k; j >= 0; j = d->dof_parentid[j], t++) {
      if (t >= MGX_MAX_DEPTH) return fail(MGX_E_CAPACITY, "dof chain longer than MGX_MAX_DEPTH");
      anc[k * MGX_MAX_DEPTH + t] = j;
      ancadr[k * MGX_MAX_DEPTH + t] = d->dof_Madr[j];
      if (j != k) {
        if (j < 64) ancmask[k] |= 1ull << j;
        else ancmask_hi[k] |= 1ull << (j - 64);
      }
    }
    chainlen[k] = t;
  }
  B.ints(d->body_parentid, nb, &M.body_parentid); B.ints(d->body_rootid, nb, &M.body_rootid);
  B.ints(d->body_jntnum, nb, &M.body_jntnum); B.ints(d->body_jntadr, nb, &M.body_jntadr);
  B.ints(d->body_dofnum, nb, &M.body_dofnum); B.ints(d->body_dofadr, nb, &M.body_dofadr);
  B.ints(d->body_subtree_end, nb, &M.body_subtree_end); B.ints(chain.data(), chain.size(), &M.body_chain);
  B.ints(depth.data(), nb, &M.body_depth);
  B.add(d->body_dofmask, sizeof(uint32_t) * nb * d->nmaskword, (const void**)&M.body_dofmask);
  B.reals(d->body_pos, 3 * nb, &M.body_pos); B.reals(d->body_quat, 4 * nb, &M.body_quat);
  B.reals(d->body_ipos, 3 * nb, &M.body_ipos); B.reals(d->body_iquat, 4 * nb, &M.body_iquat);
  B.reals(d->body_mass, nb, &M.body_mass); B.reals(d->body_inertia, 3 * nb, &M.body_inertia);
  B.reals(d->body_invweight0, 2 * nb, &M.body_invweight0);
  B.ints(d->jnt_type, nj, &M.jnt_type); B.ints(d->jnt_bodyid, nj, &M.jnt_bodyid);
  B.ints(d->jnt_qposadr, nj, &M.jnt_qposadr); B.ints(d->jnt_dofadr, nj, &M.jnt_dofadr);
  B.ints(d->jnt_limited, nj, &M.jnt_limited);
  B.reals(d->jnt_pos, 3 * nj, &M.jnt_pos); B.reals(d->jnt_axis, 3 * nj, &M.jnt_axis);
  B.reals(d->jnt_range, 2 * nj, &M.jnt_range); B.reals(d->jnt_stiffness, nj, &M.jnt_stiffness);
  B.reals(d->jnt_margin, nj, &M.jnt_margin); B.reals(d->jnt_solref, 2 * nj, &M.jnt_solref);
  B.reals(d->jnt_solimp, 5 * nj, &M.jnt_solimp);
  B.ints(d->dof_bodyid, nv, &M.dof_bodyid); B.ints(d->dof_jntid, nv, &M.dof_jntid);
  B.ints(d->dof_parentid, nv, &M.dof_parentid); B.ints(d->dof_Madr, nv, &M.dof_Madr);
  B.ints(chainlen.data(), nv, &M.dof_chainlen); B.ints(anc.data(), anc.size(), &M.dof_anc);
  B.add(ancmask.data(), 8 * ancmask.size(), (const void**)&M.dof_ancmask);
  B.add(ancmask_hi.data(), 8 * ancmask_hi.size(), (const void**)&M.dof_ancmask_hi);
  B.ints(ancadr.data(), ancadr.size(), &M.dof_ancadr);
  B.reals(d->dof_armature, nv, &M.dof_armature); B.reals(d->dof_damping, nv, &M.dof_damping);
  B.reals(d->dof_invweight0, nv, &M.dof_invweight0);
  B.ints(d->geom_type, ng, &M.geom_type); B.ints(d->geom_bodyid, ng, &M.geom_bodyid);
  B.reals(d->geom_size, 3 * ng, &M.geom_size); B.reals(d->geom_pos, 3 * ng, &M.geom_pos);
  B.reals(d->geom_quat, 4 * ng, &M.geom_quat); B.reals(d->geom_rbound, ng, &M.geom_rbound);
  B.ints(d->pair_geom, 2 * np, &M.pair_geom); B.ints(d->pair_condim, np, &M.pair_condim);
  B.reals(d->pair_friction, 5 * np, &M.pair_friction); B.reals(d->pair_margin, np, &M.pair_margin);
  {
    std::vector<int> bpi(4 * (size_t)np, 0);
    std::vector<double> bpr(4 * (size_t)np, 0.0);
    for (int p = 0; p < np; p++) {
      const int g1 = d->pair_geom[2 * p], g2 = d->pair_geom[2 * p + 1];
      const int t1 = d->geom_type[g1], t2 = d->geom_type[g2];
      const double mg = d->pair_margin[p];
      auto boxed = [](int t) { return t == GBOX || t == GCAPSULE || t == GCYLINDER; };
      int kind = 0;
      if (t1 == GPLANE) kind = 1;
      else if (boxed(t1) && boxed(t2)) kind = 2;
      else if (t1 == GSPHERE && boxed(t2)) kind = 4;
      else if (t2 == GSPHERE && boxed(t1)) kind = 8;
      bpi[4 * p] = g1; bpi[4 * p + 1] = g2; bpi[4 * p + 2] = kind;
      bpr[4 * p] = t1 == GPLANE ? d->geom_rbound[g2] + mg : d->geom_rbound[g1] + d->geom_rbound[g2] + mg;
      bpr[4 * p + 1] = mg;
      bpr[4 * p + 2] = kind == 4 ? d->geom_rbound[g1] : (kind == 8 ? d->geom_rbound[g2] : 0.0);
    }
    B.ints(bpi.data(), bpi.size(), &M.pair_bpi);
    B.reals(bpr.data(), bpr.size(), &M.pair_bpr);
    std::vector<double> obb(3 * (size_t)ng, 0.0);
    for (int g = 0; g < ng; g++) {
      const double* sz = d->geom_size + 3 * g;
      const int t = d->geom_type[g];
      if (t == GBOX) { obb[3 * g] = sz[0]; obb[3 * g + 1] = sz[1]; obb[3 * g + 2] = sz[2]; }
      if (t == GCAPSULE) { obb[3 * g] = sz[0]; obb[3 * g + 1] = sz[0]; obb[3 * g + 2] = sz[1] + sz[0]; }
      if (t == GCYLINDER) { obb[3 * g] = sz[0]; obb[3 * g + 1] = sz[0]; obb[3 * g + 2] = sz[1]; }
    }
    B.reals(obb.data(), obb.size(), &M.geom_obb);
  }
  B.reals(d->pair_gap, np, &M.pair_gap); B.reals(d->pair_solref, 2 * np, &M.pair_solref);
  B.reals(d->pair_solimp, 5 * np, &M.pair_solimp);
  B.ints(d->actuator_trnid, nu, &M.actuator_trnid); B.ints(d->actuator_ctrllimited, nu, &M.actuator_ctrllimited);
  B.ints(d->actuator_forcelimited, nu, &M.actuator_forcelimited);
  B.reals(d->actuator_gear, nu, &M.actuator_gear); B.reals(d->actuator_ctrlrange, 2 * nu, &M.actuator_ctrlrange);
  B.reals(d->actuator_forcerange, 2 * nu, &M.actuator_forcerange);
  B.reals(d->actuator_gainprm, 3 * nu, &M.actuator_gainprm); B.reals(d->actuator_biasprm, 3 * nu, &M.actuator_biasprm);
  B.reals(d->qpos0, d->nq, &M.qpos0); B.reals(d->qpos_spring, d->nq, &M.qpos_spring);
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipMalloc(&out->dbuf, B.host.size()));
  HIPCHK(hipMemcpy(out->dbuf, B.host.data(), B.host.size(), hipMemcpyHostToDevice));
  out->dbytes = B.host.size();
  for (auto& f : B.fix) *f.second = (char*)out->dbuf + f.first;
  return MGX_OK;
}

template <typename KernelT>
int set_lds(KernelT k, int bytes) { return mgx_set_lds(k, bytes); }

int check_state(const mgx_state* s) { return mgx::host_check_state(s); }

}  // namespace

namespace mgx {
int host_check_state(const mgx_state* s) {
  if (!s || !s->qpos || !s->qvel || !s->qacc_warmstart || !s->ctrl || !s->qfrc_applied || !s->xfrc_applied || !s->time)
    return fail(MGX_E_ARG, "null state buffer");
  return MGX_OK;
}
}  // namespace mgx

// LDS bytes of one main-launch solver wave: its slots' row scalars, block tables and compressed B
// (tools/pgs_census.py measures what the slots need at bench conditions); 16 lanes per slot =
// 4 slots per wave, 64 lanes = 1
static int pgs_arena_bytes(int precision) {
  const int a = precision == MGX_F32 ? MGX_PGS_ARENA_F32 : MGX_PGS_ARENA_F64;
  return pgs_lanes() == 64 ? a / 2 : a;
}

// LDS bytes of the soccer wide launch's one-slot waves with B in LDS (pgs_group BLDS sizes: whole
// ring turns of blocks plus the look-ahead, 16-byte rounded B) for the model's largest slot, or 0
// when that exceeds 160 KiB or MGX_PGS_WIDE_LDS=0 (B from global memory, the A/B alternative)
static int wide_arena_bytes(const mgx_model* m) {
  const int wide_lds = m->hooks.pgs_wide_lds;
  const int rb = m->precision == MGX_F32 ? 4 : 8;
  const int nv = m->precision == MGX_F32 ? m->mf.nv : m->md.nv;
  const int maxE = m->Ls.max_nefc;
  const int nbRun = (maxE / 4 + MGX_PGS_RING_LDS - 1) / MGX_PGS_RING_LDS * MGX_PGS_RING_LDS;
  const int nbA = nbRun + MGX_PGS_RING_LDS - 1;
  const int bcap = 32 + (maxE / 4) * (8 + 32 * ((nv + 7) / 8));
  const int worst = nbA * (4 * MGX_SCAL * rb + 4 * mgx_twl(false)) + ((bcap + 3) & ~3) * rb;
  return wide_lds && pgs_lanes() == 16 && worst + 64 <= 160 * 1024 ? (worst + 15) & ~15 : 0;
}

// Staged-step workspace layout for (model, n_env, banks); offsets in bytes, 256-aligned. rk: the
// RK4 staged step's extra arrays (stage carry, template scratch); nobs: floats per bank observation.
size_t mgx::make_staged_pipe(const mgx_model* m, void* ws, int n_env, int banks, Pipe* P, bool rk, int nobs) {
  int rb = m->precision == MGX_F32 ? 4 : 8;
  int nq = m->precision == MGX_F32 ? m->mf.nq : m->md.nq;
  int nv = m->precision == MGX_F32 ? m->mf.nv : m->md.nv;
  Pipe p{};
  p.base = (char*)ws;
  p.N = n_env; p.R = banks; p.S = n_env * (1 + banks);
  p.maxE = m->Ls.max_nefc; p.nv = nv; p.dpl = (nv + 7) / 8;  // solver: support entries per lane
  // test hook: MGX_PGS_LDS_ROWS (Hooks.pgs_lds_rows, read at model creation) lowers the main
  // launch's LDS rows, so ordinary states exercise the wide-LDS launch (tests/test_gpu_capacity.py)
  const Hooks& H = m->hooks;
  const bool cap_env = H.pgs_lds_rows > 0;
  int capE = cap_env ? (H.pgs_lds_rows + 3) / 4 * 4 : MGX_PGS_LDS_ROWS;
  if (capE < 4 || capE > p.maxE) capE = MGX_PGS_LDS_ROWS;
  if (rk) {
    // the RK4 pipeline's rows (bipedal: ~150 per forward, up to 512): MGX_RK_LDS_ROWS, default 256
    capE = H.rk_lds_rows > 0 ? (H.rk_lds_rows + 3) / 4 * 4 : 256;
    if (capE < 4) capE = 256;
  }
  p.capE = p.maxE < capE ? p.maxE : capE;
  // soccer at full capacity (more rows than MGX_PGS_LDS_ROWS): the main launch keeps as many rows
  // of LDS row scalars per slot as four waves per CU allow (fp64: 224), the wide launch beside it
  // solves the rare slot beyond that with its B in LDS (measured, one box: 1.554M env-steps/s
  // against 1.460M for one main launch over every slot with its row scalars read from the pipe at
  // six waves per CU, 1.534M for that launch held to four; reduced capacity 1.647M).
  // MGX_PGS_SINGLE=1 selects the single main launch (A/B); the MGX_PGS_LDS_ROWS test hook sets the
  // main launch's rows directly.
  p.sqg = 0;
  if (!rk && !cap_env && !H.pgs_lds_b && p.maxE > MGX_PGS_LDS_ROWS) {
    if (H.pgs_single) {
      p.capE = p.maxE;
      p.sqg = 1;
    } else {
      // MGX_PGS_WPC (A/B): size the LDS rows for more waves per CU than four; the slots beyond
      // them run in the main launch with their scalars from the pipe (hmain), whose LDS then
      // sets the wave's allocation when it is the larger
      const int budget = 160 * 1024 / H.pgs_wpc;
      int r = H.pgs_wpc == 4 ? MGX_PGS_LDS_ROWS : 8;
      while (r + 8 <= p.maxE && staged_pgs_lds_bytes(m, r + 8, pgs_lanes(), 0, mgx_twl(false)) <= budget) r += 8;
      p.capE = r;
    }
  }
  // the wide launch (slots over capE rows: soccer in the split mode) copies its one slot's B, row
  // scalars and block table into LDS when the largest slot fits 160 KiB (MGX_PGS_WIDE_LDS=0: B
  // from global memory, the A/B alternative). Same sizes as pgs_group's BLDS path: whole ring
  // turns of blocks plus the look-ahead, 16-byte rounded B.
  p.warena = !rk && p.maxE > p.capE ? wide_arena_bytes(m) : 0;
  // LDS arena of one main-launch solver wave (scalars + block table + B of its slots); the
  // test / tuning hook MGX_PGS_ARENA overrides it (a small arena sends waves to the global-B launch)
  p.arena = pgs_arena_bytes(m->precision);
  if (H.pgs_arena > 0 && H.pgs_arena <= 96 * 1024) p.arena = H.pgs_arena;
  p.carry_stride = ((m->Ls.carry_reals + 63) & ~63) + 5 * 64;
  p.carryi_stride = m->Ls.carry_ints + 8;
  p.bcap = 32 + (p.maxE / 4) * (8 + 32 * ((nv + 7) / 8));
  p.tw = MGX_TW;  // block-table words (uint32) per 4-row block in the pipe, either B layout (mgx_staged.h)
  p.nobs = nobs;
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t r = off; off = (off + bytes + 255) / 256 * 256; return r; };
  size_t S = (size_t)p.S, NB = (size_t)n_env * (banks > 0 ? banks : 1);
  p.o_ctr = take(64);
  p.o_carry = take(S * p.carry_stride * rb);
  p.o_carryi = take(S * p.carryi_stride * 4);
  p.o_ne = take(S * 4); p.o_blen = take(S * 4); p.o_niter = take(S * 4); p.o_k2list = take(S * 4); p.o_k2big = take(S * 4); p.o_fix = take((size_t)n_env * 4);
  // the solver-list buckets are sized for the model's capacity, not the main launch's rows (a
  // per-call hook changes those), so the workspace layout never depends on MGX_PGS_LDS_ROWS
  // heavy slots in the main launch (hmain, the full-capacity soccer default): when the SQG layout of
  // maxE rows fits the LDS of a capE-row wave. The MGX_PGS_LDS_ROWS test hook keeps the wide launch.
  p.hmain = !rk && !cap_env && !p.sqg && !H.pgs_lds_b && p.capE < p.maxE &&
            staged_pgs_lds_bytes(m, p.maxE, pgs_lanes(), 1, mgx_twl(false)) <=
                (H.pgs_wpc == 4 ? staged_pgs_lds_bytes(m, p.capE, pgs_lanes(), 0, mgx_twl(false))
                                : 160 * 1024 / H.pgs_wpc);
  if (p.hmain) p.warena = 0;
  p.prio_rows = H.pgs_prio_rows > 0 ? H.pgs_prio_rows : p.capE;
  p.nbk = (p.hmain ? p.maxE : p.capE) / 4 + 1;
  p.o_hist = take((size_t)(p.maxE / 4 + 1) * 4);
  p.o_blist = take((size_t)(p.maxE / 4 + 1) * S * 4);
  p.o_scal = take(S * p.maxE * MGX_SCAL * rb);
  p.o_blk = take(S * (p.maxE / 4) * p.tw * 4);  // tw uint32 per 4-row block
  p.o_B = take(S * (size_t)p.bcap * rb);
  p.o_vout = take(S * 64 * rb);
  p.o_bq = take(NB * nq * rb); p.o_bv = take(NB * nv * rb); p.o_ba = take(NB * nv * rb); p.o_btime = take(NB * rb);
  p.o_bobs = take(NB * nobs * 4); p.o_bprev = take(NB * 6 * rb); p.o_bwind = take(NB * 3 * rb);
  p.o_bk = take(NB * 4); p.o_bep = take(NB * 4); p.o_bwarn = take(NB * 4); p.o_bseed = take(NB * 8);
  int nb = m->precision == MGX_F32 ? m->mf.nbody : m->md.nbody;
  p.maxC = m->Ls.max_ncon;
  p.o_cpos = take(S * 3 * (size_t)p.maxC * rb);
  p.o_tq = take(nq * rb); p.o_tv = take(nv * rb); p.o_ta = take(64 * rb); p.o_tt = take(rb);
  p.o_tx = take(3 * nb * rb); p.o_txq = take(4 * nb * rb); p.o_tsc = take(3 * nb * rb); p.o_tn = take(4);
  p.o_tcg = take(2 * p.maxC * 4); p.o_tcd = take(p.maxC * rb); p.o_tcm = take(p.maxC * rb);
  // per-slot ints: the RK4 step's warnings / overflow over its stages, parkour's overflow flag over
  // its substeps; the checkAcc template kernel's rows when the monolithic layout keeps them in
  // global memory
  p.o_rkw = take(S * 4);
  p.o_tscr = take(m->L.gB ? (size_t)m->L.gB_stride * rb : 64);
  if (rk) {
    const int nq4 = (nq + 3) & ~3;
    p.rk_stride = 2 * nq4 + 8 * 64 + 4;
    p.o_rk = take(S * p.rk_stride * rb);
    p.o_rks = take(S * 4);
  }
  if (P) *P = p;
  return off;
}
static size_t make_pipe(const mgx_model* m, void* ws, int n_env, int banks, Pipe* P) {
  return make_staged_pipe(m, ws, n_env, banks, P, false, 80);
}

// LDS of one solver wave holding `rows` rows per slot (main launch: min(max_nefc,
// MGX_PGS_LDS_ROWS); wide launch: max_nefc)
int mgx::staged_pgs_lds_bytes(const mgx_model* m, int rows, int lps, int sqg, int twl) {
  int rb = m->precision == MGX_F32 ? 4 : 8;
  int nb3 = (rows / 4 + MGX_PGS_RING - 1) / MGX_PGS_RING * MGX_PGS_RING;  // whole ring turns
  const int spw = 64 / lps;
  // the row scalars (or, SQG: the forces only; pgs_group) + the block table
  const int sq = sqg ? 4 : 4 * MGX_SCAL;
  return spw * (sq * nb3 + 4) * rb + spw * nb3 * 4 * twl + 64;
}
static int pgs_lds_bytes(const mgx_model* m, int rows, int sqg = 0) {
  return staged_pgs_lds_bytes(m, rows, pgs_lanes(), sqg, mgx_twl(false));
}

// Hooks (mgx_internal.h): the MGX_* A/B and test variables, read once per model
mgx::Hooks mgx::read_hooks() {
  Hooks h;
  auto get = [](const char* name, int dflt) {
    const char* v = getenv(name);
    return v && *v ? atoi(v) : dflt;
  };
  h.pgs_lds_rows = get("MGX_PGS_LDS_ROWS", 0);
  h.rk_lds_rows = get("MGX_RK_LDS_ROWS", 0);
  h.pgs_single = get("MGX_PGS_SINGLE", 0);
  h.pgs_lds_b = get("MGX_PGS_LDS_B", MGX_PGS_LDS_B) != 0;
  h.pgs_arena = get("MGX_PGS_ARENA", 0);
  h.pgs_lds_pad = get("MGX_PGS_LDS_PAD", 0);
  h.pgs_wide_lds = get("MGX_PGS_WIDE_LDS", 1);
  h.pgs_spw = get("MGX_PGS_SPW", 0);
  h.pgs_prio_rows = get("MGX_PGS_PRIO_ROWS", 0);
  h.tight_bp = get("MGX_TIGHT_BROADPHASE", -1);
  h.pgs_wpc = get("MGX_PGS_WPC", 4);
  if (h.pgs_wpc < 4 || h.pgs_wpc > 16) h.pgs_wpc = 4;
  // MGX_SIDE_STREAM=0 runs the wide solver launch after the main one on the caller's stream: with
  // more streams than hardware queues (several tasks on one GPU, each on its own stream) a side
  // stream can queue behind another task's long kernels
  h.side_stream = get("MGX_SIDE_STREAM", 1) != 0;
  h.gcon = get("MGX_GCON", 1);
  h.rows_lds = get("MGX_ROWS_LDS", 0);
  return h;
}

// A side stream and two events per caller stream (created once, kept for the process): the wide
// solver launch runs beside the main one. nullptr if the runtime refuses (then both run in order).
struct SideStream {
  hipStream_t s;
  hipEvent_t rows, big;
};
static SideStream* side_stream(hipStream_t st) {
  static std::mutex mu;
  static std::map<std::pair<hipStream_t, int>, SideStream*> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  auto key = std::make_pair(st, dev);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  SideStream* x = new SideStream{};
  if (hipStreamCreateWithFlags(&x->s, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&x->rows, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&x->big, hipEventDisableTiming) != hipSuccess) {
    delete x;
    x = nullptr;
  }
  cache[key] = x;
  return x;
}

// LDS of the one-wave settle: the row builder's layout, then one solver wave with maxE rows per
// slot, then the finisher's layout, in turn
static int settle_lds_bytes(const mgx_model* m, const Pipe& P) {
  int b = pgs_lds_bytes(m, P.maxE);
  if (m->Ls.bytes > b) b = m->Ls.bytes;
  if (m->Lf.bytes > b) b = m->Lf.bytes;
  return b;
}

template <typename T>
static int soccer_step_staged(const mgx_model* m, const DevModel<T>& M, const DevModel<T>& Ms, const DevModel<T>& Mf,
                              const SoccerIds<T>& ids, const mgx_state* s, const mgx_soccer_env* e, const float* action,
                              float* obs, double* reward, uint8_t* terminated, uint8_t* truncated, float* final_obs,
                              int autoreset, uint64_t seed, int env_offset, int n_env, const uint8_t* mask,
                              hipStream_t st) {
  Pipe P;
  int banks = autoreset ? e->banks : 0;
  size_t need = make_pipe(m, e->workspace, n_env, e->banks, &P);
  if (e->workspace_bytes < need) return fail(MGX_E_ARG, "workspace smaller than mgx_soccer_workspace_bytes");
  int slots = n_env * (1 + banks);
  const Hooks& H = m->hooks;
  // occupancy probe: MGX_ROWS_LDS pads the row builder's LDS (fewer waves per CU; up to 64 KiB)
  const int rlds = H.rows_lds > m->Ls.bytes && H.rows_lds <= 64 * 1024 ? H.rows_lds : m->Ls.bytes;
  launch_soccer_rows<T>(Ms, ids, *s, *e, action, n_env, mask, P, banks, slots, rlds, st);
  T scale = (T)1 / (M.meaninertia * (T)(M.nv > 1 ? M.nv : 1));
  // slots over the main launch's LDS rows (MuJoCo has no cap: the rows are kept, not dropped):
  // a small grid-stride global-B launch with maxE rows of LDS per slot, which exits at once when
  // the list is empty. It runs on a side stream beside the main launch (a slot of ~300 rows is
  // one wave's 50-sweep chain, which would otherwise trail the main launch). With the LDS-arena
  // main launch (MGX_PGS_LDS_B) it also takes the waves that did not fit their arena, so it
  // follows the main launch there.
  const int wgrid = 64 / pgs_lanes() * MGX_PGS_WIDE_GRID, wlds = pgs_lds_bytes(m, P.maxE);
  int mlds = H.pgs_lds_b ? P.arena : pgs_lds_bytes(m, P.capE, P.sqg);
  if (P.hmain) mlds = std::max(mlds, pgs_lds_bytes(m, P.maxE, 1));  // the heavy slots' SQG layout
  // occupancy probe: MGX_PGS_LDS_PAD pads the main solver launch's LDS (fewer waves per CU)
  if (H.pgs_lds_pad > mlds && H.pgs_lds_pad <= 96 * 1024) mlds = H.pgs_lds_pad;
  if (!H.pgs_lds_b && (P.maxE <= P.capE || P.hmain)) {
    // every slot fits the main launch (the default capacity): no wide launch at all
    launch_pgs<T>(P, slots, mlds, st, M.iterations, M.tolerance, scale, 0, H);
  } else if (SideStream* side = (!H.pgs_lds_b && H.side_stream) ? side_stream(st) : nullptr) {
    HIPCHK(hipEventRecord(side->rows, st));
    HIPCHK(hipStreamWaitEvent(side->s, side->rows, 0));
    launch_pgs<T>(P, wgrid, wlds, side->s, M.iterations, M.tolerance, scale, 1, H);
    HIPCHK(hipEventRecord(side->big, side->s));
    launch_pgs<T>(P, slots, mlds, st, M.iterations, M.tolerance, scale, 0, H);
    HIPCHK(hipStreamWaitEvent(st, side->big, 0));
  } else {
    launch_pgs<T>(P, slots, mlds, st, M.iterations, M.tolerance, scale, 0, H);
    launch_pgs<T>(P, wgrid, wlds, st, M.iterations, M.tolerance, scale, 1, H);
  }
  launch_soccer_finish<T>(Mf, ids, *s, *e, action, obs, reward, terminated, truncated, final_obs, autoreset, seed,
                          env_offset, n_env, mask, P, banks, m->Lf.bytes, st);
  // resets whose bank was not ready: settled in one wave each by the pipeline's own stages
  // (k_soccer_settle), a small grid-stride launch that exits at once when the list is empty
  int fgrid = n_env < 256 ? n_env : 256;
  launch_soccer_settle<T>(Ms, Mf, ids, *s, *e, (const T*)nullptr, obs, seed, env_offset, n_env, nullptr, P, SETTLE_FIXUP,
                          fgrid, settle_lds_bytes(m, P), st, M.iterations, M.tolerance, scale);
  HIPCHK(hipGetLastError());
  return MGX_OK;
}

// reset() of a staged batch: every env's reset (and, with Philox draws, its R banks) settled by
// the pipeline's stages in one wave (k_soccer_settle), so the staged batch has one arithmetic for
// every reset, whatever the bank count
template <typename T>
static int soccer_reset_staged(const mgx_model* m, const DevModel<T>& M, const DevModel<T>& Ms, const DevModel<T>& Mf,
                               const SoccerIds<T>& ids, const mgx_state* s, const mgx_soccer_env* e, const T* draws,
                               float* obs, uint64_t seed, int env_offset, int n_env, const uint8_t* mask, hipStream_t st) {
  Pipe P;
  size_t need = make_pipe(m, e->workspace, n_env, e->banks, &P);
  if (e->workspace_bytes < need) return fail(MGX_E_ARG, "workspace smaller than mgx_soccer_workspace_bytes");
  T scale = (T)1 / (M.meaninertia * (T)(M.nv > 1 ? M.nv : 1));
  launch_soccer_settle<T>(Ms, Mf, ids, *s, *e, draws, obs, seed, env_offset, n_env, mask, P, SETTLE_RESET, n_env,
                          settle_lds_bytes(m, P), st, M.iterations, M.tolerance, scale);
  HIPCHK(hipGetLastError());
  return MGX_OK;
}

template <typename T>
static void fill_ids(SoccerIds<T>& o, const mgx_soccer_ids* ids, const DevModel<T>& M, const mgx_model_desc* unused) {
  (void)unused;
  o.torso = ids->torso; o.ball = ids->ball; o.goalkeeper = ids->goalkeeper; o.ball_geom = ids->ball_geom;
  o.right_foot = ids->right_foot; o.left_foot = ids->left_foot; o.field_geom = ids->field_geom;
  o.ball_qposadr = ids->ball_qposadr; o.ball_dofadr = ids->ball_dofadr; o.gk_qposadr = ids->gk_qposadr;
  o.gk_qfrc_index = ids->gk_dofadr; o.max_episode_steps = ids->max_episode_steps;
  for (int i = 0; i < 25; i++) {
    o.obs_qposadr[i] = ids->obs_jnt_qposadr[i];
    o.obs_dofadr[i] = ids->obs_jnt_dofadr[i];
    o.obs_lo[i] = (T)ids->obs_jnt_range[2 * i];
    o.obs_hi[i] = (T)ids->obs_jnt_range[2 * i + 1];
  }
  o.robot_mask_lo = ids->robot_geom_mask_lo;
  o.robot_mask_hi = ids->robot_geom_mask_hi;
}

extern "C" {

const char* mgx_last_error(void) { return g_err.c_str(); }

int mgx_abi_version(void) { return MGX_ABI_VERSION; }

int mgx_model_create(const mgx_model_desc* d, int precision, int device, mgx_model** out) {
  if (!d || !out) return fail(MGX_E_ARG, "null argument");
  if (precision != MGX_F32 && precision != MGX_F64) return fail(MGX_E_ARG, "precision must be MGX_F32 or MGX_F64");
  // nv <= 64: one dof per lane (every task kernel); 64 < nv <= 128: the wide kernels only
  // (mgx_wide.h, two dofs per lane: humanoid_construction, nv 99), which every other configure
  // entry point refuses
  if (d->nv > MGX_MAX_NV_WIDE) return fail(MGX_E_CAPACITY, "nv > 128 not supported by the wave-per-env kernels");
  if (d->nbody > 4096 || (d->solver != 0 && d->solver != 2) || (d->integrator != 0 && d->integrator != 1))
    return fail(MGX_E_UNSUPPORTED, "this build implements PGS or Newton with Euler or RK4");
  bool condim13 = true;  // the staged row builder packs one contact per 4-row block
  for (int p = 0; p < d->npair; p++) {
    const int c = d->pair_condim[p];
    if (c != 1 && c != 3 && c != 4 && c != 6) return fail(MGX_E_UNSUPPORTED, "condim must be 1, 3, 4 or 6");
    condim13 = condim13 && (c == 1 || c == 3);
  }
  mgx_model* m = new mgx_model();
  m->hooks = read_hooks();
  m->precision = precision;
  m->device = device;
  m->npair = d->npair;
  m->wide = d->nv > MGX_MAX_NV;
  // capacities: the model's request (efc_capacity / con_capacity), else 192 rows / 64 contacts.
  // MGX_MAX_NEFC / MGX_MAX_NCON may raise them (read here, once); a value below the model's is
  // refused: it would drop rows MuJoCo keeps. A smaller capacity is a property of the model itself
  // (mgx_model_desc.efc_capacity / con_capacity), never of the environment.
  int max_nefc = d->efc_capacity > 0 ? d->efc_capacity : 192;
  int max_ncon = d->con_capacity > 0 ? d->con_capacity : 64;
  if (const char* v = getenv("MGX_MAX_NEFC")) {
    if (atoi(v) < max_nefc) { delete m; return fail(MGX_E_ARG, "MGX_MAX_NEFC below the model's row capacity"); }
    max_nefc = atoi(v);
  }
  if (const char* v = getenv("MGX_MAX_NCON")) {
    if (atoi(v) < max_ncon) { delete m; return fail(MGX_E_ARG, "MGX_MAX_NCON below the model's contact capacity"); }
    max_ncon = atoi(v);
  }
  if (max_nefc > 1024 || max_ncon > 512) { delete m; return fail(MGX_E_CAPACITY, "capacity above 1024 rows / 512 contacts"); }
  max_nefc = (max_nefc + 3) & ~3;  // the staged solver sweeps rows in blocks of 4
  if (max_nefc < 4 || max_ncon < 1) { delete m; return fail(MGX_E_ARG, "row / contact capacity too small"); }
  int rb = precision == MGX_F32 ? 4 : 8;
  // broadphase survivor list: 128 for the small candidate sets (soccer 251, parkour 48 pairs),
  // up to 768 for large ones (bipedal 3185 pairs)
  int max_active = d->npair <= 256 ? 128 : (d->npair < 768 ? d->npair : 768);
  // the staged soccer pipeline handles Euler + PGS models up to 64 * MGX_EFC_SLOTS rows
  m->staged_ok = d->integrator == 0 && d->solver == 0 && max_nefc <= 64 * MGX_EFC_SLOTS && condim13 &&
                 d->nv <= 56;  // the solver's block table holds 7 dof groups of 8 (pgs_load_tab)
  // the monolithic layout of a staged model (its reset settle steps, the rare fixup resets,
  // --mono, mgx_debug_forward) keeps rows in LDS at the default 192 rows / 64 contacts; the
  // staged step itself carries the model's full capacity
  // the staged RK4 step (mgx_rk_staged.h, bipedal_rescue): RK4 + PGS, nv 49..64 (four register
  // entries per solver lane, a 16-word block table)
  m->staged_rk_ok = d->integrator == 1 && d->solver == 0 && condim13 && d->nv > 48 && d->nv <= 64 &&
                    max_nefc <= 1024 && max_ncon <= 192;  // three contact-metadata lane sets (RK_NCS)
  // ... and of a staged RK4 model (its checkAcc template, --mono) at most 512 rows, whose per-row
  // LDS arrays fit next to its working set with the rows in global scratch
  // A staged Euler model whose monolithic layout keeps its rows in global scratch (parkour) carries
  // the full capacity there too: only its per-row scalars are in LDS.
  const bool mono_lds_rows = !(d->layout_flags & MGX_ROWS_IN_SCRATCH);
  const int mono_nefc = m->staged_ok && mono_lds_rows && max_nefc > 192 ? 192
                        : (m->staged_rk_ok && max_nefc > 512 ? 512 : max_nefc);
  const int mono_ncon = m->staged_ok && mono_lds_rows && max_ncon > 64 ? 64 : max_ncon;
  m->L = make_layout(d, rb, mono_ncon, mono_nefc, max_active);
  // rows that do not fit next to the rest of the per-env LDS working set go to global scratch
  if (m->L.bytes > 160 * 1024 || (d->layout_flags & MGX_ROWS_IN_SCRATCH))
    m->L = make_layout(d, rb, mono_ncon, mono_nefc, max_active, true);
  const bool any_staged = m->staged_ok || m->staged_rk_ok;
  m->Ls = make_staged_layout(d, rb, max_ncon, any_staged ? max_nefc : 4, m->staged_ok ? 128 : max_active,
                             m->hooks.gcon);
  m->Lf = finisher_layout(m->Ls, rb);
  {
    const int tight = m->hooks.tight_bp >= 0 ? (m->hooks.tight_bp != 0) : (d->npair > MGX_TIGHT_BROADPHASE_PAIRS);
    m->L.tight_bp = m->Ls.tight_bp = m->Lf.tight_bp = tight;
  }
  int rc;
  if (precision == MGX_F32) {
    rc = build_model<float>(d, device, m, m->mf);
    m->mf.L = m->L; m->mfs = m->mf; m->mfs.L = m->Ls; m->mff = m->mf; m->mff.L = m->Lf;
  } else {
    rc = build_model<double>(d, device, m, m->md);
    m->md.L = m->L; m->mds = m->md; m->mds.L = m->Ls; m->mdf = m->md; m->mdf.L = m->Lf;
  }
  if (rc != MGX_OK) { delete m; return rc; }
  if (m->L.bytes > 160 * 1024) { delete m; return fail(MGX_E_CAPACITY, "per-env LDS exceeds 160 KiB"); }
  int r2 = step_kernels_configure(m);
  if (r2 != MGX_OK) { delete m; return r2; }
  if (m->wide) {
    r2 = wide_kernels_configure(m);
    if (r2 != MGX_OK) { delete m; return r2; }
  }
  r2 = precision == MGX_F32
               ? (set_lds(k_soccer<float, 0>, m->L.bytes) | set_lds(k_soccer<float, 1>, m->L.bytes) |
                  set_lds(k_soccer_logic<float>, m->L.bytes) | set_lds(k_soccer_template<float>, m->L.bytes))
               : (set_lds(k_soccer<double, 0>, m->L.bytes) | set_lds(k_soccer<double, 1>, m->L.bytes) |
                  set_lds(k_soccer_logic<double>, m->L.bytes) | set_lds(k_soccer_template<double>, m->L.bytes));
  if (r2 != MGX_OK) { delete m; return r2; }
  if (m->staged_ok) {
    int sl = pgs_lds_bytes(m, m->Ls.max_nefc);  // the settle kernel's (settle_lds_bytes)
    if (m->Ls.bytes > sl) sl = m->Ls.bytes;
    if (m->Lf.bytes > sl) sl = m->Lf.bytes;
    r2 = staged_kernels_configure(precision, m->Ls.bytes, m->Lf.bytes, sl);
    if (r2 != MGX_OK) { delete m; return r2; }
    int pl = pgs_lds_bytes(m, m->Ls.max_nefc);  // the global-B launch's
    if (pl < 96 * 1024) pl = 96 * 1024;  // the arena (MGX_PGS_ARENA tuning up to 96 KiB)
    if (pl > 160 * 1024) { delete m; return fail(MGX_E_CAPACITY, "solver LDS exceeds 160 KiB: lower MGX_MAX_NEFC"); }
    int r3 = pgs_configure_lds(precision, pl, wide_arena_bytes(m) + 64);
    if (r3 != MGX_OK) { delete m; return r3; }
  }
  *out = m;
  return MGX_OK;
}

int mgx_model_destroy(mgx_model* m) {
  if (!m) return MGX_OK;
  if (m->dbuf) (void)hipFree(m->dbuf);
  delete m;
  return MGX_OK;
}

int mgx_model_get_info(const mgx_model* m, mgx_model_info* o) {
  if (!m || !o) return fail(MGX_E_ARG, "null argument");
  int nq, nv, nu, nb, nj, ng;
  if (m->precision == MGX_F32) { nq = m->mf.nq; nv = m->mf.nv; nu = m->mf.nu; nb = m->mf.nbody; nj = m->mf.njnt; ng = m->mf.ngeom; }
  else { nq = m->md.nq; nv = m->md.nv; nu = m->md.nu; nb = m->md.nbody; nj = m->md.njnt; ng = m->md.ngeom; }
  o->nq = nq; o->nv = nv; o->nu = nu; o->nbody = nb; o->njnt = nj; o->ngeom = ng; o->npair = m->npair;
  o->max_nv = MGX_MAX_NV; o->max_nbody = 4096; o->max_ncon = m->L.max_ncon; o->max_nefc = m->L.max_nefc;
  o->max_njnt = 1 << 20; o->precision = m->precision; o->lds_bytes_per_env = m->L.bytes;
  o->lds_bytes_rows = m->Ls.bytes; o->lds_bytes_finish = m->Lf.bytes;
  o->scratch_bytes_per_env = m->L.gB ? m->L.gB_stride * (m->precision == MGX_F32 ? 4 : 8) : 0;
  return MGX_OK;
}

int mgx_soccer_configure(mgx_model* m, const mgx_soccer_ids* ids) {
  if (!m || !ids) return fail(MGX_E_ARG, "null argument");
  if (m->wide) return fail(MGX_E_UNSUPPORTED, MGX_WIDE_MSG);
  if (m->L.gB || (m->precision == MGX_F32 ? m->mf.integrator : m->md.integrator) != 0)
    return fail(MGX_E_UNSUPPORTED, "the soccer kernels need an Euler model whose rows fit LDS");
  if ((m->precision == MGX_F32 ? m->mf.solver : m->md.solver) != 0)
    return fail(MGX_E_UNSUPPORTED, "the soccer kernels solve with PGS (soccer_env.py:150-151)");
  if (ids->max_episode_steps <= 0) return fail(MGX_E_ARG, "max_episode_steps must be > 0");
  if (m->precision == MGX_F32) fill_ids(m->sf, ids, m->mf, nullptr);
  else fill_ids(m->sd, ids, m->md, nullptr);
  m->soccer_ok = true;
  return MGX_OK;
}

// Reset-specific tables (noise joints) ride in the same ids struct; set via this helper.
int mgx_soccer_configure_reset(mgx_model* m, int root_qposadr, int n_noise, const int32_t* noise_qposadr,
                               const double* noise_range) {
  if (!m || n_noise < 0 || n_noise > 29 || (n_noise && (!noise_qposadr || !noise_range)))
    return fail(MGX_E_ARG, "bad reset table");
  auto fill = [&](auto& o) {
    o.root_qposadr = root_qposadr;
    o.n_noise = n_noise;
    for (int i = 0; i < n_noise; i++) {
      o.noise_qposadr[i] = noise_qposadr[i];
      o.noise_lo[i] = noise_range[2 * i];
      o.noise_hi[i] = noise_range[2 * i + 1];
    }
  };
  if (m->precision == MGX_F32) fill(m->sf); else fill(m->sd);
  return MGX_OK;
}

int mgx_soccer_step(const mgx_model* m, const mgx_state* s, const mgx_soccer_env* e, const float* action, float* obs,
                    double* reward, uint8_t* terminated, uint8_t* truncated, float* final_obs, int autoreset,
                    uint64_t seed, int env_offset, int n_env, const uint8_t* mask, void* stream) {
  if (!m || !e || !action || !obs || !reward || !terminated || !truncated) return fail(MGX_E_ARG, "null argument");
  if (e->action_f64 != 0 && e->action_f64 != 1) return fail(MGX_E_ARG, "action_f64 must be 0 (float32) or 1 (float64)");
  if (!m->soccer_ok) return fail(MGX_E_ARG, "mgx_soccer_configure not called");
  if (autoreset && !e->episode) return fail(MGX_E_ARG, "autoreset needs the episode counter buffer");
  int rc = check_state(s);
  if (rc) return rc;
  if (n_env <= 0) return MGX_OK;
  hipStream_t st = (hipStream_t)stream;
  if (e->workspace) {
    if (!m->staged_ok) return fail(MGX_E_UNSUPPORTED, "staged step: model exceeds the staged solver's capacity");
    if (e->banks < 0 || e->banks > 16) return fail(MGX_E_ARG, "banks must be in [0, 16]");
    if (m->precision == MGX_F32)
      return soccer_step_staged<float>(m, m->mf, m->mfs, m->mff, m->sf, s, e, action, obs, reward, terminated,
                                       truncated, final_obs, autoreset, seed, env_offset, n_env, mask, st);
    return soccer_step_staged<double>(m, m->md, m->mds, m->mdf, m->sd, s, e, action, obs, reward, terminated, truncated,
                                      final_obs, autoreset, seed, env_offset, n_env, mask, st);
  }
  Pipe none{};
  if (m->precision == MGX_F32)
    hipLaunchKernelGGL((k_soccer<float, 0>), dim3(n_env), dim3(64), m->L.bytes, st, m->mf, m->sf, *s, *e, action,
                       (const float*)nullptr, obs, reward, terminated, truncated, final_obs, autoreset, seed,
                       env_offset, n_env, mask, none, 0);
  else
    hipLaunchKernelGGL((k_soccer<double, 0>), dim3(n_env), dim3(64), m->L.bytes, st, m->md, m->sd, *s, *e, action,
                       (const double*)nullptr, obs, reward, terminated, truncated, final_obs, autoreset, seed,
                       env_offset, n_env, mask, none, 0);
  HIPCHK(hipGetLastError());
  return MGX_OK;
}

int mgx_soccer_reset(const mgx_model* m, const mgx_state* s, const mgx_soccer_env* e, const void* draws, float* obs,
                     uint64_t seed, int env_offset, int n_env, const uint8_t* mask, void* stream) {
  if (!m || !e || !obs) return fail(MGX_E_ARG, "null argument");
  if (!m->soccer_ok) return fail(MGX_E_ARG, "mgx_soccer_configure not called");
  if (!draws && !e->episode) return fail(MGX_E_ARG, "device draws need the episode counter buffer");
  int rc = check_state(s);
  if (rc) return rc;
  if (n_env <= 0) return MGX_OK;
  hipStream_t st = (hipStream_t)stream;
  if (e->workspace) {
    if (!m->staged_ok) return fail(MGX_E_UNSUPPORTED, "staged step: model exceeds the staged solver's capacity");
    if (e->banks < 0 || e->banks > 16) return fail(MGX_E_ARG, "banks must be in [0, 16]");
    if (m->precision == MGX_F32)
      return soccer_reset_staged<float>(m, m->mf, m->mfs, m->mff, m->sf, s, e, (const float*)draws, obs, seed,
                                        env_offset, n_env, mask, st);
    return soccer_reset_staged<double>(m, m->md, m->mds, m->mdf, m->sd, s, e, (const double*)draws, obs, seed,
                                       env_offset, n_env, mask, st);
  }
  Pipe none{};
  if (m->precision == MGX_F32)
    hipLaunchKernelGGL((k_soccer<float, 1>), dim3(n_env), dim3(64), m->L.bytes, st, m->mf, m->sf, *s, *e,
                       (const float*)nullptr, (const float*)draws, obs, (double*)nullptr, (uint8_t*)nullptr,
                       (uint8_t*)nullptr, (float*)nullptr, 0, seed, env_offset, n_env, mask, none, 0);
  else
    hipLaunchKernelGGL((k_soccer<double, 1>), dim3(n_env), dim3(64), m->L.bytes, st, m->md, m->sd, *s, *e,
                       (const float*)nullptr, (const double*)draws, obs, (double*)nullptr, (uint8_t*)nullptr,
                       (uint8_t*)nullptr, (float*)nullptr, 0, seed, env_offset, n_env, mask, none, 0);
  HIPCHK(hipGetLastError());
  return MGX_OK;
}

int64_t mgx_soccer_workspace_bytes(const mgx_model* m, int n_env, int banks) {
  if (!m || n_env <= 0 || banks < 0 || banks > 16) return fail(MGX_E_ARG, "bad argument");
  if (!m->staged_ok) return fail(MGX_E_UNSUPPORTED, "staged step: model exceeds the staged solver's capacity");
  return (int64_t)make_pipe(m, nullptr, n_env, banks, nullptr);
}

int mgx_soccer_workspace_layout(const mgx_model* m, int n_env, int banks, int64_t* out, int n_out) {
  if (!m || !out || n_env <= 0 || banks < 0 || banks > 16 || n_out < 10) return fail(MGX_E_ARG, "bad argument");
  if (!m->staged_ok) return fail(MGX_E_UNSUPPORTED, "staged step: model exceeds the staged solver's capacity");
  Pipe P;
  make_pipe(m, nullptr, n_env, banks, &P);
  const int64_t v[11] = {(int64_t)P.o_ctr, (int64_t)P.o_ne, (int64_t)P.o_k2list, (int64_t)P.o_blk, (int64_t)P.o_B,
                         P.bcap, P.maxE, P.capE, P.S, m->precision == MGX_F32 ? 4 : 8, (int64_t)P.o_k2big};
  for (int i = 0; i < (n_out < 11 ? n_out : 11); i++) out[i] = v[i];
  return MGX_OK;
}

int mgx_soccer_workspace_init(const mgx_model* m, void* workspace, uint64_t bytes, int n_env, int banks, void* stream) {
  if (!m || !workspace || n_env <= 0 || banks < 0 || banks > 16) return fail(MGX_E_ARG, "bad argument");
  Pipe P;
  size_t need = make_pipe(m, workspace, n_env, banks, &P);
  if (bytes < need) return fail(MGX_E_ARG, "workspace smaller than mgx_soccer_workspace_bytes");
  hipStream_t st = (hipStream_t)stream;
  HIPCHK(hipMemsetAsync(workspace, 0, need, st));
  size_t nb = (size_t)n_env * (banks > 0 ? banks : 1);
  HIPCHK(hipMemsetAsync(P.base + P.o_bk, 0xFF, nb * 4, st));  // bank settle counters = -1 (empty)
  if (m->precision == MGX_F32)
    hipLaunchKernelGGL(k_soccer_template<float>, dim3(1), dim3(64), m->L.bytes, st, m->mf, P);
  else
    hipLaunchKernelGGL(k_soccer_template<double>, dim3(1), dim3(64), m->L.bytes, st, m->md, P);
  HIPCHK(hipGetLastError());
  return MGX_OK;
}

int mgx_soccer_logic_test(const mgx_model* m, const mgx_soccer_logic_io* io, int n_env, void* stream) {
  if (!m || !io) return fail(MGX_E_ARG, "null argument");
  if (!m->soccer_ok) return fail(MGX_E_ARG, "mgx_soccer_configure not called");
  if (io->max_contacts > m->L.max_ncon) return fail(MGX_E_CAPACITY, "max_contacts exceeds the contact capacity");
  if (n_env <= 0) return MGX_OK;
  hipStream_t st = (hipStream_t)stream;
  if (m->precision == MGX_F32)
    hipLaunchKernelGGL(k_soccer_logic<float>, dim3(n_env), dim3(64), m->L.bytes, st, m->mf, m->sf, *io, n_env);
  else
    hipLaunchKernelGGL(k_soccer_logic<double>, dim3(n_env), dim3(64), m->L.bytes, st, m->md, m->sd, *io, n_env);
  HIPCHK(hipGetLastError());
  return MGX_OK;
}

}  // extern "C"
