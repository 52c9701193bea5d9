// mgx_assembly.h — robotic_arm_assembly_env task logic fused around the physics steps.
//
// Restates, per env and on the GPU, the reference's Python around mj_step
// (robotic_arm_assembly_env/assembly_env.py):
//   step():       :220-250 (np.clip to the float32 action bounds, ctrl :252-265, 10 mj_steps)
//   task state:   :267-297 over the gripper-pad contacts :299-322 (per-geom tags from the host)
//   reward:       :331-387 (float64, the reference's order), "force" :389-397
//   termination:  :399-417, truncation :240, observation :419-472 (quirk A1 layout)
//   reset:        :162-218 (deterministic: mj_resetData, home pose + bins, 10 mj_steps)
// Frames (xpos, xquat) and the contact list are those of the last substep's forward pass, as
// MuJoCo leaves them in mjData after mj_step; qpos/qvel are post-integration. The model solves
// with Newton (complete_model.xml:4), so the kernels instantiate mj_step_env<T, false, true>.
// Quirk A3 (list(set(names))[0] with several touched components) takes the first in sequence
// order; oracle/assembly_logic.py documents the quirks.
#pragma once
#include "../../include/mgx.h"
#include "mgx_soccer.h"

namespace mgx {

enum { AI_STEP = 0, AI_HELD = 1, AI_PHASE = 2, AI_PROG = 3, AI_STATUS = 4, AI_N = 16 };
enum { AS_IN_BIN = 0, AS_HELD = 1, AS_ASSEMBLED = 2, AS_DROPPED = 3, AS_DAMAGED = 4 };
enum { AP_IDLE = 0, AP_PICKUP = 1, AP_TRANSPORT = 2, AP_ALIGN = 3, AP_INSERT = 4 };

// np.clip(action, low, high) in the action's dtype; ctrl[0:7] = a[0:7]; ctrl[7] = ctrl[8] = a[7] /
// 1000.0 (float32 / Python float stays float32 under NEP 50; a float64 action divides in float64).
// The reward does not read the action (:331-385).
template <typename T>
__device__ __forceinline__ void assembly_pre(const DevModel<T>& m, Env<T>& e, const mgx_assembly_ids& ids, ActRow act) {
  const int l = lane_id();
  if (l < 9) {
    if (act.f64) {
      double a = act.d()[l];
      const double lo = (double)ids.action_low[l], hi = (double)ids.action_high[l];
      a = a < lo ? lo : (a > hi ? hi : a);
      if (l < 7) e.ctrl[l] = (T)a;
      if (l == 7) {
        const double g = a / 1000.0;
        e.ctrl[7] = (T)g;
        e.ctrl[8] = (T)g;
      }
    } else {
      float a = act.f()[l];
      a = a < ids.action_low[l] ? ids.action_low[l] : (a > ids.action_high[l] ? ids.action_high[l] : a);
      if (l < 7) e.ctrl[l] = (T)a;
      if (l == 7) {
        const float g = a / 1000.0f;
        e.ctrl[7] = (T)g;
        e.ctrl[8] = (T)g;
      }
    }
  }
  wsync();
}

// max |dist| * 1000 over the contacts (:389-397); 0 with none
template <typename T>
__device__ __forceinline__ double assembly_max_force(const Env<T>& e, int ncon) {
#pragma clang fp contract(off)
  double mf = 0.0;
  for (int c = 0; c < ncon; c++) {
    const double f = fabs((double)e.con_dist[c]) * 1000.0;
    mf = f > mf ? f : mf;
  }
  return mf;
}

// bit mask of the components touched by a gripper pad (:299-322)
template <typename T>
__device__ __forceinline__ int assembly_touched(const Env<T>& e, const mgx_assembly_ids& ids, int ncon) {
  int mask = 0;
  for (int c = 0; c < ncon; c++) {
    const int g1 = e.con_geom[2 * c], g2 = e.con_geom[2 * c + 1];
    int k = -1;
    if (ids.geom_pad[g1]) k = ids.geom_comp[g2];
    else if (ids.geom_pad[g2]) k = ids.geom_comp[g1];
    if (k >= 0) mask |= 1 << k;
  }
  return mask;
}

__device__ __forceinline__ double assembly_target_dist(const double* p, const double* t) {
  return norm3_np(p[0] - t[0], p[1] - t[1], p[2] - t[2]);
}

// _get_observation (:419-472), quirk A1 layout; float32 of the stale forward frames and the
// post-step state. site_xpos = xpos[body] + xmat[body] site_pos with xmat = quat2mat(xquat),
// the matrix the forward pass built from the same normalised quaternion.
template <typename T>
__device__ __forceinline__ void assembly_obs(const DevModel<T>& m, const Env<T>& e, const mgx_assembly_ids& ids,
                                             int held, int phase, int prog, double mf, float* obs) {
  const int l = lane_id();
  for (int i = l; i < MGX_ASSEMBLY_OBS; i += 64) {
    double v;
    if (i < 7) v = (double)e.qpos[i];
    else if (i < 14) v = (double)e.qvel[i - 7];
    else if (i == 14) {
#pragma clang fp contract(off)
      v = ((double)e.qpos[7] + (double)e.qpos[8]) / 2.0 * 1000.0;
    } else if (i == 15) v = mf;
    else if (i < 19) {
      T R[9], p[3];
      quat2mat(R, e.xquat + 4 * ids.ee_body);
      const T sp[3] = {(T)ids.ee_pos[0], (T)ids.ee_pos[1], (T)ids.ee_pos[2]};
      mulmatvec3(p, R, sp);
      v = (double)(p[i - 16] + e.xpos[3 * ids.ee_body + i - 16]);
    } else if (i < 23) v = i == 19 ? 1.0 : 0.0;
    else if (i < 79) {
      const int c = (i - 23) / 7, k = (i - 23) % 7;
      v = k < 3 ? (double)e.xpos[3 * ids.comp_body[c] + k] : (k == 3 ? 1.0 : 0.0);
    } else if (i < 87) v = (prog >> (i - 79)) & 1 ? 1.0 : 0.0;
    else if (i == 87) v = held >= 0 ? 1.0 : 0.0;
    else if (i == 88) v = (double)held;
    else if (i < 104) v = 0.5;
    else if (i == 108) {
#pragma clang fp contract(off)
      v = (double)__builtin_popcount(prog) / 9.0 * 100.0;
    } else if (i == 109) v = (double)phase;
    else v = 0.0;
    obs[i] = (float)v;
  }
}

// _update_task_state + _calculate_reward + _check_termination on lane 0 (float64, reference
// order; the integer terms are exact in float64). st: the env's ints row (updated in place).
template <typename T>
__device__ __forceinline__ double assembly_logic_lane0(const DevModel<T>& m, const Env<T>& e,
                                                       const mgx_assembly_ids& ids, int* st, double mf, int touched,
                                                       bool* term) {
#pragma clang fp contract(off)
  auto comp_pos = [&](int c, double* p) {
    for (int k = 0; k < 3; k++) p[k] = (double)e.xpos[3 * ids.comp_body[c] + k];
  };
  // _update_task_state (:267-297)
  if (touched) {
    if (st[AI_HELD] < 0) {
      const int h = __builtin_ctz(touched);
      st[AI_HELD] = h;
      st[AI_PHASE] = AP_PICKUP;
      st[AI_STATUS + h] = AS_HELD;
    } else {
      st[AI_PHASE] = AP_TRANSPORT;
    }
  } else if (st[AI_HELD] >= 0) {
    const int h = st[AI_HELD];
    double p[3];
    comp_pos(h, p);
    if (assembly_target_dist(p, ids.targets + 3 * h) < 0.002) {
      st[AI_PROG] |= 1 << h;
      st[AI_STATUS + h] = AS_ASSEMBLED;
      st[AI_PHASE] = AP_INSERT;
    } else {
      st[AI_STATUS + h] = AS_DROPPED;
      st[AI_PHASE] = AP_IDLE;
    }
    st[AI_HELD] = -1;
  } else {
    st[AI_PHASE] = AP_IDLE;
  }
  // _calculate_reward (:331-387)
  double r = -10.0;
  if (st[AI_PHASE] == AP_PICKUP && st[AI_HELD] >= 0) r += 1000.0;
  for (int c = 0; c < MGX_ASSEMBLY_NCOMP; c++)
    if (((st[AI_PROG] >> c) & 1) && st[AI_STATUS + c] == AS_ASSEMBLED) r += ids.place_reward[c];
  if (st[AI_HELD] >= 0) {
    const int h = st[AI_HELD];
    double p[3];
    comp_pos(h, p);
    const double d = assembly_target_dist(p, ids.targets + 3 * h);
    if (d < 0.05) r += 300.0 * (1.0 - d / 0.05);
  }
  if (mf > 50.0) r -= 5000.0;
  else if (mf < 10.0) r += 200.0;
  // -np.sum(np.abs(qvel[0:7])) * 10: a 7-element add.reduce from the identity, in order
  double s = -0.0;
  for (int k = 0; k < 7; k++) s += fabs((double)e.qvel[k]);
  s = 0.0 + s;
  r += -s * 10.0;
  for (int c = 0; c < MGX_ASSEMBLY_NCOMP; c++) {
    if (st[AI_STATUS + c] == AS_DROPPED) r -= 2000.0;
    else if (st[AI_STATUS + c] == AS_DAMAGED) r -= 5000.0;
  }
  const bool all = st[AI_PROG] == (1 << MGX_ASSEMBLY_NCOMP) - 1;
  if (all) r += 10000.0;
  // _check_termination (:399-417)
  bool t = all;
  for (int c = 0; c < MGX_ASSEMBLY_NCOMP; c++) t = t || st[AI_STATUS + c] == AS_DAMAGED;
  for (int k = 0; k < 7; k++) {
    const double q = (double)e.qpos[k];
    t = t || q < ids.joint_low[k] || q > ids.joint_high[k];
  }
  *term = t;
  return r;
}

// Post-physics: counter, task state, reward, termination, truncation, obs. Returns done.
template <typename T>
__device__ __forceinline__ bool assembly_post(const DevModel<T>& m, Env<T>& e, const mgx_assembly_ids& ids,
                                              mgx_assembly_env ae, int env, float* obs, double* reward,
                                              uint8_t* terminated, uint8_t* truncated) {
  const int l = lane_id();
  int* st = ae.ints + (size_t)env * AI_N;
  const int ncon = __builtin_amdgcn_readfirstlane(e.ncon);
  const double mf = assembly_max_force(e, ncon);
  bool term = false, trunc = false;
  int held = 0, phase = 0, prog = 0;
  if (l == 0) {
    st[AI_STEP] += 1;
    const int touched = assembly_touched(e, ids, ncon);
    const double r = assembly_logic_lane0(m, e, ids, st, mf, touched, &term);
    trunc = st[AI_STEP] >= ids.max_episode_steps;
    ae.cumulative[env] += r;
    reward[env] = r;
    terminated[env] = term;
    truncated[env] = trunc;
    held = st[AI_HELD]; phase = st[AI_PHASE]; prog = st[AI_PROG];
  }
  held = __builtin_amdgcn_readfirstlane(held);
  phase = __builtin_amdgcn_readfirstlane(phase);
  prog = __builtin_amdgcn_readfirstlane(prog);
  assembly_obs(m, e, ids, held, phase, prog, mf, obs + (size_t)env * MGX_ASSEMBLY_OBS);
  const bool done = __builtin_amdgcn_readfirstlane((int)(term || trunc)) != 0;
  wsync();
  return done;
}

// reset() (:162-218), split around its 10 mj_steps so the task kernel keeps one physics call
// site: the prologue runs mj_resetData, qpos = reset_qpos (home pose + bins) and clears the
// tracking state; the epilogue writes the observation of the settled state.
template <typename T>
__device__ __forceinline__ void assembly_reset_prologue(const DevModel<T>& m, Env<T>& e, mgx_assembly_env ae, int env) {
  const int l = lane_id();
  reset_env(m, e);
  for (int k = l; k < m.nq; k += 64) e.qpos[k] = (T)ae.reset_qpos[k];
  int* st = ae.ints + (size_t)env * AI_N;
  if (l < AI_N) st[l] = l == AI_HELD ? -1 : 0;
  if (l == 0) ae.cumulative[env] = 0.0;
  wsync();
}

template <typename T>
__device__ __forceinline__ void assembly_reset_epilogue(const DevModel<T>& m, Env<T>& e, const mgx_assembly_ids& ids,
                                                        int env, float* obs) {
  const int ncon = __builtin_amdgcn_readfirstlane(e.ncon);
  assembly_obs(m, e, ids, -1, AP_IDLE, 0, assembly_max_force(e, ncon), obs + (size_t)env * MGX_ASSEMBLY_OBS);
  wsync();
}

}  // namespace mgx
