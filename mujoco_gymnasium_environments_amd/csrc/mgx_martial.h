// mgx_martial.h — humanoid_martial_arts_env task logic fused around the physics step.
//
// Restates, per env and on the GPU, the reference's Python around mj_step:
//   step():       humanoid_martial_arts_env/martial_arts_env.py:489-523 (clip :492,
//                 ctrl = action * actuator_ctrlrange[:, 1] :495, one mj_step :498)
//   observation:  :525-560 (113 floats: torso xpos/xquat/cvel, qpos[7:], qvel[6:], dummies,
//                 constant placeholders, stance timer; quirk M2)
//   reward:       :562-606 (float64 on lane 0, numpy promotion of the float32 energy term)
//   termination:  :608-621, truncation :511, statistics :632-640 (prev_torso_pos survives reset,
//                 quirk M3), reset :442-487 (the pose lands on dummy1's free joint, quirk M1)
// Frames (xpos, xquat, cvel) are those of the step's forward pass, as MuJoCo leaves them in
// mjData after mj_step; qpos/qvel are post-integration. The model solves with Newton
// (martial_arts_scene.xml:163), so the kernels instantiate mj_step_env<T, false, true>.
#pragma once
#include "../../include/mgx.h"
#include "mgx_soccer.h"

namespace mgx {

#define MGX_MARTIAL_OBS 113
enum { MS_STANCE = 0, MS_DIST = 1, MS_PREV = 2, MS_N = 5 };
enum { MI_STEP = 0, MI_TECH = 1, MI_FALLS = 2, MI_HASPREV = 3, MI_N = 4 };

struct MartialIds {
  int torso, right_hand, left_hand, right_foot, left_foot, dummy1, dummy2;
  int n_act, max_episode_steps;
  double ctrl_scale[32];
};

// np.linalg.norm of a float64 2-vector: sqrt of the BLAS dot (one FMA)
__device__ __forceinline__ double martial_norm2(double x, double y) { return sqrt(fma(y, y, x * x)); }

// numpy add.reduce of |clip(a, -1, 1)| over n contiguous values in the action's dtype (float32
// or float64; pairwise: 8 accumulators over the first 8*floor(n/8), tree (01)(23) / (45)(67), then
// the tail)
template <typename A>
__device__ __forceinline__ A np_sum_abs_clip1(const A* action, int n) {
#pragma clang fp contract(off)
  auto v = [&](int u) {
    A a = action[u];
    a = a < (A)-1 ? (A)-1 : (a > (A)1 ? (A)1 : a);
    return a < (A)0 ? -a : a;
  };
  if (n < 8) {
    A res = 0;
    for (int u = 0; u < n; u++) res += v(u);
    return res;
  }
  A r[8];
  for (int k = 0; k < 8; k++) r[k] = v(k);
  int i = 8;
  for (; i + 8 <= n; i += 8)
    for (int k = 0; k < 8; k++) r[k] += v(i + k);
  A res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; i++) res += v(i);
  return res;
}

// clip -> ctrl (martial_arts_env.py:492-495): the clipped action (float32, or float64 for a float64
// policy) times the float64 ctrlrange bound
template <typename T>
__device__ __forceinline__ void martial_pre(const DevModel<T>& m, Env<T>& e, const MartialIds& ids, ActRow act) {
  const int l = lane_id();
  if (l < ids.n_act) {
    double a;
    if (act.f64) {
      a = act.d()[l];
      a = a < -1.0 ? -1.0 : (a > 1.0 ? 1.0 : a);
    } else {
      float af = act.f()[l];
      a = (double)(af < -1.0f ? -1.0f : (af > 1.0f ? 1.0f : af));
    }
    e.ctrl[l] = (T)(a * ids.ctrl_scale[l]);
  }
  wsync();
}

// _get_observation (:525-560): float32 of the stale forward frames and the post-step state
template <typename T>
__device__ __forceinline__ void martial_obs(const DevModel<T>& m, const Env<T>& e, const MartialIds& ids, double stance,
                                            float* obs) {
  const int l = lane_id();
  const int nq7 = m.nq - 7, nv6 = m.nv - 6;
  for (int i = l; i < MGX_MARTIAL_OBS; i += 64) {
    double v = 0;
    int k = i;
    if (k < 3) v = (double)e.xpos[3 * ids.torso + k];
    else if ((k -= 3) < 4) v = (double)e.xquat[4 * ids.torso + k];
    else if ((k -= 4) < 6) v = (double)e.cvel[6 * ids.torso + k];  // [:3] angular, [3:] linear
    else if ((k -= 6) < nq7) v = (double)e.qpos[7 + k];
    else if ((k -= nq7) < nv6) v = (double)e.qvel[6 + k];
    else if ((k -= nv6) < 3) v = (double)e.xpos[3 * ids.dummy1 + k];
    else if ((k -= 3) < 3) v = (double)e.xpos[3 * ids.dummy2 + k];
    else if ((k -= 3) < 3) v = k == 1 ? -2.0 : (k == 2 ? 1.0 : 0.0);
    else if ((k -= 3) < 6) v = 0.0;  // force placeholders, technique_accuracy, len(combo_chain)
    else v = stance;
    obs[i] = (float)v;
  }
}

// _calculate_reward (:562-606) with the reference's numpy types: the reward is a Python float
// until an np.float64 enters (min(1.0, h / 1.75) returns the np.float64 only when it is < 1;
// the approach term); the energy term np.sum(np.abs(action)) * 0.01 is np.float32, so a
// still-Python-float reward becomes float32 there and the approach term promotes it back. A
// float64 action (e64) makes the energy term np.float64, and the reward float64 from there on.
// Advances the stance timer and techniques_performed as the reference does.
__device__ __forceinline__ double martial_reward_np(double h, double rh, double lh, double rf, double lf, double ang,
                                                    double dist, float energy, double* stance, int* tech,
                                                    bool e64 = false, double energy64 = 0.0) {
#pragma clang fp contract(off)
  double r = 0.0;
  bool is64 = false;
  double x = h / 1.75;
  if (x < 1.0) { r += 100.0 * x; is64 = true; }
  else r += 100.0 * 1.0;
  if (rh > 2.0 || lh > 2.0) { r += 500.0; *tech += 1; }
  if (rf > 3.0 || lf > 3.0) { r += 800.0; *tech += 1; }
  if (ang < 0.5) {
    *stance += 0.01667;
    r += 200.0 * 0.01667;
  }
  const float ecost = energy * 0.01f;
  if (e64) r -= energy64 * 0.01;
  else if (is64) r -= (double)ecost;
  else r = (double)((float)r - ecost);
  if (dist < 2.0) r += 50.0 * (2.0 - dist);
  return r;
}

// Post-physics: counter, obs, reward, termination, truncation, statistics. Returns done.
template <typename T>
__device__ __forceinline__ bool martial_post(const DevModel<T>& m, Env<T>& e, const MartialIds& ids, ActRow act,
                                             mgx_martial_env me, int env, float* obs, double* reward,
                                             uint8_t* terminated, uint8_t* truncated) {
#pragma clang fp contract(off)
  const int l = lane_id();
  double* S = me.scal + (size_t)env * MS_N;
  int* I = me.ints + (size_t)env * MI_N;
  const double stance0 = S[MS_STANCE];
  const int st = I[MI_STEP] + 1;
  martial_obs(m, e, ids, stance0, obs + (size_t)env * MGX_MARTIAL_OBS);
  bool term = false, trunc = false;
  if (l == 0) {
    auto nrm3 = [&](int b, int off) {
      const T* c = e.cvel + 6 * b + off;
      return norm3_np((double)c[0], (double)c[1], (double)c[2]);
    };
    const T* tp = e.xpos + 3 * ids.torso;
    const T* d1 = e.xpos + 3 * ids.dummy1;
    const double tx = tp[0], ty = tp[1], tz = tp[2];
    double stance = stance0;
    int tech = I[MI_TECH], falls = I[MI_FALLS];
    const double r = martial_reward_np(tz, nrm3(ids.right_hand, 0), nrm3(ids.left_hand, 0), nrm3(ids.right_foot, 0),
                                       nrm3(ids.left_foot, 0), nrm3(ids.torso, 3),
                                       martial_norm2((double)d1[0] - tx, (double)d1[1] - ty),
                                       act.f64 ? 0.0f : np_sum_abs_clip1(act.f(), ids.n_act), &stance, &tech, act.f64 != 0,
                                       act.f64 ? np_sum_abs_clip1(act.d(), ids.n_act) : 0.0);
    if (tz < 0.5) { falls += 1; term = true; }
    else term = fabs(tx) > 5.5 || fabs(ty) > 5.5;
    trunc = st >= ids.max_episode_steps;
    // _update_statistics: prev_torso_pos appears at the first step with current_step > 1
    if (st > 1) {
      if (I[MI_HASPREV]) S[MS_DIST] += martial_norm2(tx - S[MS_PREV], ty - S[MS_PREV + 1]);
      S[MS_PREV] = tx; S[MS_PREV + 1] = ty; S[MS_PREV + 2] = tz;
      I[MI_HASPREV] = 1;
    }
    S[MS_STANCE] = stance;
    I[MI_STEP] = st;
    I[MI_TECH] = tech;
    I[MI_FALLS] = falls;
    reward[env] = r;
    terminated[env] = term;
    truncated[env] = trunc;
  }
  const bool done = __builtin_amdgcn_readfirstlane((int)(term || trunc)) != 0;
  wsync();
  return done;
}

// Reset draws for the vector env: Philox4x32-10 keyed by (seed, global env index), counter =
// (episode, word); the two uniform(-0.5, 0.5) of martial_arts_env.py:462-463
template <typename T>
__device__ __forceinline__ void martial_philox_draws(uint64_t seed, uint32_t genv, uint32_t episode, T* out) {
  const int j = lane_id();
  if (j < 2) {
    uint32_t c[4] = {episode, (uint32_t)j, 0x4A475Au, 0u};
    philox4x32(c, (uint32_t)seed ^ genv, (uint32_t)(seed >> 32));
    double u = ((double)(c[0] >> 5) * 67108864.0 + (double)(c[1] >> 6)) * (1.0 / 9007199254740992.0);
    out[j] = (T)(-0.5 + 1.0 * u);
  }
}

// reset() (:442-487): mj_resetData, qpos[0:3] = (0, 0, 1.4) + the draws on x / y, qpos[3:7] =
// identity (dummy1's free joint, quirk M1), tracking state cleared (prev_torso_pos kept,
// quirk M3), mj_forward, observation
template <typename T>
__device__ __forceinline__ void martial_reset_body(const DevModel<T>& m, Env<T>& e, const MartialIds& ids, T d0, T d1,
                                                   mgx_martial_env me, int env, float* obs) {
  const int l = lane_id();
  reset_env(m, e);
  double* S = me.scal + (size_t)env * MS_N;
  int* I = me.ints + (size_t)env * MI_N;
  if (l == 0) {
    e.qpos[0] = (T)(0.0 + (double)d0); e.qpos[1] = (T)(0.0 + (double)d1); e.qpos[2] = (T)1.4;
    e.qpos[3] = 1; e.qpos[4] = 0; e.qpos[5] = 0; e.qpos[6] = 0;
    S[MS_STANCE] = 0.0; S[MS_DIST] = 0.0;
    I[MI_STEP] = 0; I[MI_TECH] = 0; I[MI_FALLS] = 0;
  }
  wsync();
  forward<T, true>(m, e);
  martial_obs(m, e, ids, 0.0, obs + (size_t)env * MGX_MARTIAL_OBS);
  wsync();
}

}  // namespace mgx
