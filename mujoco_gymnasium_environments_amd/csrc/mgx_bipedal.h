// mgx_bipedal.h — bipedal_rescue_env task logic fused around the RK4 physics step.
//
// Restates, per env and on the GPU, the reference's Python around mj_step:
//   step():        bipedal_rescue_env/rescue_env.py:416-471 (clip :420, ctrl[:26] :423-424,
//                  energy :427-429 in float32, one RK4 mj_step :432, counter :435)
//   interactions:  :510-543 (capacity tested once before the pickup loop; gripper :757-763)
//   observation:   :545-600 (102 floats; foot "forces" :741-751 = sum |dist| of the first
//                  10 contacts into slot 0)
//   reward:        :602-668 (the _prev_* attributes are created lazily and survive reset,
//                  quirk B3; closest_victim_distance restarts at +inf so the approach term
//                  can be +inf on the first step after a reset)
//   termination:   :670-697 (the _fall_timer attribute also survives reset)
//   stats:         :699-706, reset :347-396 with _randomize_initial_state :473-508
// Frames (xpos/xquat, contacts) are those the last RK4 stage left, as MuJoCo leaves them in
// mjData; qpos/qvel are post-integration. Reward arithmetic is float64 on lane 0 whatever the
// physics precision; 2-D distances follow numpy's norm (sqrt of an FMA dot), energy follows
// numpy's float32 pairwise sum.
#pragma once
#include "../../include/mgx.h"
#include "mgx_soccer.h"

namespace mgx {

struct BipedalIds {
  int torso, victims[5];
  int obs_qposadr[26], obs_dofadr[26];  // joint_indices -> qpos / dof address (rescue_env.py:298-308)
  int root_x, root_y, root_z, root_dof;  // qpos addresses of root_x/y/z, dof address of root_x
  int victim_x[5], victim_y[5];          // qpos addresses of victim{i}_x / _y
  int n_act, max_episode_steps;
};

__device__ __forceinline__ double norm2_np(double x, double y) { return sqrt(fma(y, y, x * x)); }

// numpy add.reduce over 26 contiguous values in the action's dtype (float32 or float64; pairwise:
// 8 accumulators, tree, tail)
template <typename A>
__device__ __forceinline__ A np_sum26_abs_clip(const A* a) {
#pragma clang fp contract(off)
  A v[26];
  for (int j = 0; j < 26; j++) {
    A x = a[j];
    x = x < (A)-100 ? (A)-100 : (x > (A)100 ? (A)100 : x);
    v[j] = x < (A)0 ? -x : x;
  }
  A r[8];
  for (int j = 0; j < 8; j++) r[j] = (v[j] + v[j + 8]) + v[j + 16];
  A res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  res += v[24];
  res += v[25];
  return res;
}

// numpy type of current_energy / energy_used (mgx_bipedal_env.energy_kind)
enum { EK_PY = 0, EK_F64 = 1, EK_F32 = 2 };

// action clip -> ctrl[:26], energy bookkeeping (rescue_env.py:419-429) in numpy's arithmetic: the
// cost np.sum(np.abs(a)) * 0.001 has the action's dtype; current_energy -= cost (and energy_used +=
// cost) stays float32 while both are float32 (a Python float, after reset, becomes float32) and is
// float64 from the first float64 operand on
template <typename T>
__device__ __forceinline__ void bipedal_pre(const DevModel<T>& m, Env<T>& e, const BipedalIds& ids, ActRow act,
                                            mgx_bipedal_env be, int env) {
#pragma clang fp contract(off)
  int l = lane_id();
  if (l < ids.n_act) {
    if (act.f64) {
      double a = act.d()[l];
      a = a < -100.0 ? -100.0 : (a > 100.0 ? 100.0 : a);
      e.ctrl[l] = (T)a;
    } else {
      float a = act.f()[l];
      a = a < -100.0f ? -100.0f : (a > 100.0f ? 100.0f : a);
      e.ctrl[l] = (T)a;
    }
  }
  if (l == 0) {
    int kind = be.energy_kind ? be.energy_kind[env] : EK_F32;
    if (act.f64 || kind == EK_F64) {
      const double cost = act.f64 ? np_sum26_abs_clip(act.d()) * 0.001 : (double)(np_sum26_abs_clip(act.f()) * 0.001f);
      be.energy[env] = be.energy[env] - cost;
      be.energy_used[env] = be.energy_used[env] + cost;
      kind = EK_F64;
    } else {
      const float cost = np_sum26_abs_clip(act.f()) * 0.001f;
      be.energy[env] = (double)((float)be.energy[env] - cost);
      be.energy_used[env] = (double)((float)be.energy_used[env] + cost);
      kind = EK_F32;
    }
    if (be.energy_kind) be.energy_kind[env] = (uint8_t)kind;
  }
  wsync();
}

// victim pickup / safe-zone drop-off (rescue_env.py:510-543); lane 0
template <typename T>
__device__ __forceinline__ void bipedal_interactions(const Env<T>& e, const BipedalIds& ids, mgx_bipedal_env be, int env,
                                                     int step) {
  const T* r = e.xpos + 3 * ids.torso;
  double rx = (double)r[0], ry = (double)r[1];
  int resc = be.rescued[env], car = be.carried[env];
  bool carrying = be.carrying[env] != 0;
  if (__popc(car) < 2) {
    for (int i = 0; i < 5; i++) {
      if (((resc | car) >> i) & 1) continue;
      const T* v = e.xpos + 3 * ids.victims[i];
      double d = norm2_np(rx - (double)v[0], ry - (double)v[1]);
      if (d < 1.0 && d < 0.8) { car |= 1 << i; carrying = true; }
    }
  }
  if (carrying) {
    double sz = norm2_np(rx - 20.0, ry - 0.0);
    if (sz < 3.0) {
      int n = __popc(car);
      resc |= car;
      be.victims_rescued[env] += n;
      if (n > 0 && be.ttfr[env] != be.ttfr[env]) be.ttfr[env] = (double)step * 0.02;
      car = 0;
      carrying = false;
    }
  }
  be.rescued[env] = resc;
  be.carried[env] = car;
  be.carrying[env] = carrying;
}

// Observation: 102 float32 (rescue_env.py:545-600)
template <typename T>
__device__ __forceinline__ void bipedal_obs(const DevModel<T>& m, const Env<T>& e, const BipedalIds& ids, int step, int resc,
                                            int car, double energy, bool energy64, float* obs) {
  int l = lane_id();
  const T* r = e.xpos + 3 * ids.torso;
  // slot 65: sum over the first min(ncon, 10) contacts of |dist|, sequential float64
  double f = 0.0;
  int nc = e.ncon < 10 ? e.ncon : 10;
  for (int c = 0; c < nc; c++) f += fabs((double)e.con_dist[c]);
  for (int i = l; i < 102; i += 64) {
    double v = 0.0;
    if (i < 52) v = (i & 1) ? (double)e.qvel[ids.obs_dofadr[i >> 1]] : (double)e.qpos[ids.obs_qposadr[i >> 1]];
    else if (i < 55) v = (double)r[i - 52];
    else if (i < 59) v = (double)e.xquat[4 * ids.torso + (i - 55)];
    else if (i < 65) v = (double)e.qvel[ids.root_dof + (i - 59)];
    else if (i == 65) v = f;
    else if (i < 69) v = 0.0;
    else if (i < 89) {
      int k = (i - 69) >> 2, c = (i - 69) & 3;
      if (c < 2) v = (double)e.xpos[3 * ids.victims[k] + c];
      else v = (((c == 2 ? resc : car) >> k) & 1) ? 1.0 : 0.0;
    } else if (i < 92) {
      const double sz[3] = {20.0, 0.0, 0.0};
      v = sz[i - 89] - (double)r[i - 89];
    } else if (i == 92) {  // current_energy / energy_limit in current_energy's numpy type
      obs[i] = energy64 ? (float)(energy / 1000.0) : (float)energy / 1000.0f;
      continue;
    } else if (i == 93) v = 1.0 - ((double)step / (double)ids.max_episode_steps);
    else if (i == 94) v = (double)__popc(car);
    else if (i == 95) v = (double)__popc(resc);
    else {
      const double fp[2][3] = {{-5.0, -3.0, 0.0}, {8.0, 6.0, 0.0}};
      int k = (i - 96) / 3, c = (i - 96) % 3;
      v = fp[k][c] - (double)r[c];
    }
    obs[i] = (float)v;
  }
}

template <typename T>
__device__ __forceinline__ bool bipedal_upright(const Env<T>& e, const BipedalIds& ids) {
  T q[4] = {e.xquat[4 * ids.torso], e.xquat[4 * ids.torso + 1], e.xquat[4 * ids.torso + 2], e.xquat[4 * ids.torso + 3]};
  T R[9];
  quat2mat(R, q);
  return R[8] > (T)0.7;
}

// counter, interactions, obs, reward, termination, stats, prev position (rescue_env.py:435-467);
// returns done
template <typename T>
__device__ __forceinline__ bool bipedal_post(const DevModel<T>& m, Env<T>& e, const BipedalIds& ids, ActRow act,
                                             mgx_bipedal_env be, int env, float* obs, double* reward, uint8_t* terminated,
                                             uint8_t* truncated, uint8_t* upright_out = nullptr) {
#pragma clang fp contract(off)
  int l = lane_id();
  int st = be.step[env] + 1;
  if (l == 0) {
    be.step[env] = st;
    bipedal_interactions(e, ids, be, env, st);
  }
  wsync();
  int resc = be.rescued[env], car = be.carried[env];
  bool upright = bipedal_upright(e, ids);
  const bool e64 = be.energy_kind && be.energy_kind[env] == EK_F64;
  bipedal_obs(m, e, ids, st, resc, car, be.energy[env], e64, obs + (size_t)env * 102);
  int done = 0;
  if (l == 0) {
    const T* rp = e.xpos + 3 * ids.torso;
    double rx = (double)rp[0], ry = (double)rp[1];
    int nres = __popc(resc), ncar = __popc(car);
    double r = 0.0;
    int pr = be.prev_rescued[env], pc = be.prev_carried[env];
    if (pr >= 0 && nres - pr > 0) r += 5000.0 * (double)(nres - pr);
    be.prev_rescued[env] = nres;
    if (pc >= 0 && ncar - pc > 0) r += 1000.0 * (double)(ncar - pc);
    be.prev_carried[env] = ncar;
    double mind = __builtin_inf();
    for (int i = 0; i < 5; i++) {
      if (((resc | car) >> i) & 1) continue;
      const T* v = e.xpos + 3 * ids.victims[i];
      double d = norm2_np(rx - (double)v[0], ry - (double)v[1]);
      if (d < mind) mind = d;  // Python min(a, b): b only when b < a
    }
    double closest = be.closest[env];
    if (mind < closest && mind < 10.0) r += 100.0 * (closest - mind);
    be.closest[env] = mind;
    if (be.carrying[env]) {
      double sz = norm2_np(rx - 20.0, ry - 0.0);
      double psz = be.prev_sz[env];
      if (psz == psz && sz < psz) r += 200.0 * (psz - sz);
      be.prev_sz[env] = sz;
    }
    if (upright) r += 50.0;
    else { r += -500.0; be.falls[env] += 1; }
    // energy_usage = np.sum(np.abs(action)) * 0.001 in the action's dtype (:650-652)
    if (act.f64 ? np_sum26_abs_clip(act.d()) * 0.001 < 0.5 : np_sum26_abs_clip(act.f()) * 0.001f < 0.5f) r += 10.0;
    if (norm2_np(rx - -5.0, ry - -3.0) < 1.5) r += -200.0;
    if (norm2_np(rx - 8.0, ry - 6.0) < 1.2) r += -200.0;
    int nc = e.ncon < 20 ? e.ncon : 20;
    for (int c = 0; c < nc; c++)
      if (fabs((double)e.con_dist[c]) > 0.1) { r += -100.0; be.collisions[env] += 1; break; }
    r += -1.0;
    // termination (rescue_env.py:670-697): early returns leave later state untouched
    bool term = false;
    if (nres == 5) term = true;
    else {
      if (!upright) {
        int ft = be.fall_timer[env];
        if (ft < 0) ft = 0;
        ft += 1;
        be.fall_timer[env] = ft;
        if (ft > 100) term = true;
      } else {
        be.fall_timer[env] = 0;
      }
      if (!term) term = be.energy[env] <= 0.0 || fabs(rx) > 25.0 || fabs(ry) > 25.0;
    }
    bool trunc = st >= ids.max_episode_steps;
    double* pp = be.prev_robot_pos + 3 * (size_t)env;
    be.distance[env] += norm2_np(rx - pp[0], ry - pp[1]);
    pp[0] = rx; pp[1] = ry; pp[2] = (double)rp[2];
    reward[env] = r;
    terminated[env] = term;
    truncated[env] = trunc;
    if (upright_out) upright_out[env] = upright;
    done = term || trunc;
  }
  wsync();
  return __shfl(done, 0) != 0;
}

// Philox draws for the vector env's resets: lane j < 12 -> draw j of `episode`, in the
// reference's order and ranges (robot x, y ~ U(-5, 5), then per victim dx, dy ~ U(-1, 1))
template <typename T>
__device__ __forceinline__ void bipedal_philox_draws(uint64_t seed, uint32_t genv, uint32_t episode, T* out) {
  int j = lane_id();
  if (j < 12) {
    uint32_t c[4] = {episode, (uint32_t)j, 0xB1BEDu, 0u};
    philox4x32(c, (uint32_t)seed ^ genv, (uint32_t)(seed >> 32));
    double u = ((double)(c[0] >> 5) * 67108864.0 + (double)(c[1] >> 6)) * (1.0 / 9007199254740992.0);
    double lo = j < 2 ? -5.0 : -1.0, hi = j < 2 ? 5.0 : 1.0;
    out[j] = (T)(lo + (hi - lo) * u);
  }
}

// reset() (rescue_env.py:373-414), split around its 10 settle mj_step's (:390-391) so the task
// kernel keeps one physics call site: the prologue runs mj_resetData, the tracking reset and
// _randomize_initial_state from the 12 draws (read before the physics reuses the LDS); the
// epilogue writes the observation and prev_robot_pos. The _prev_* / _fall_timer attributes are
// left alone (quirk B3).
template <typename T>
__device__ __forceinline__ void bipedal_reset_prologue(const DevModel<T>& m, Env<T>& e, const BipedalIds& ids,
                                                       const T* draws, mgx_bipedal_env be, int env) {
  int l = lane_id();
  T d[12];
  for (int j = 0; j < 12; j++) d[j] = draws[j];  // uniform reads: every lane holds all 12 in registers
  reset_env(m, e);
  if (l == 0) {
    e.qpos[ids.root_x] = d[0];
    e.qpos[ids.root_y] = d[1];
    e.qpos[ids.root_z] = (T)1.2;
    for (int i = 0; i < 5; i++) {
      e.qpos[ids.victim_x[i]] = e.qpos[ids.victim_x[i]] + d[2 + 2 * i];
      e.qpos[ids.victim_y[i]] = e.qpos[ids.victim_y[i]] + d[3 + 2 * i];
    }
    be.step[env] = 0;
    be.energy[env] = 1000.0;  // Python floats again (energy_limit, 0.0)
    be.energy_used[env] = 0.0;
    if (be.energy_kind) be.energy_kind[env] = EK_PY;
    be.rescued[env] = 0;
    be.carried[env] = 0;
    be.carrying[env] = 0;
    be.closest[env] = __builtin_inf();
    be.victims_rescued[env] = 0;
    be.distance[env] = 0.0;
    be.ttfr[env] = __builtin_nan("");
    be.falls[env] = 0;
    be.collisions[env] = 0;
  }
  wsync();
}

template <typename T>
__device__ __forceinline__ void bipedal_reset_epilogue(const DevModel<T>& m, Env<T>& e, const BipedalIds& ids,
                                                       mgx_bipedal_env be, int env, float* obs) {
  int l = lane_id();
  bipedal_obs(m, e, ids, 0, 0, 0, 1000.0, false, obs + (size_t)env * 102);
  if (l < 3) be.prev_robot_pos[3 * (size_t)env + l] = (double)e.xpos[3 * ids.torso + l];
  wsync();
}

}  // namespace mgx
