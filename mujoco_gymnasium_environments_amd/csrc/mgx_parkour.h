// mgx_parkour.h — quadruped_parkour_env task logic fused around 10 physics substeps.
//
// Restates, per env and on the GPU, the reference's Python around mj_step:
//   step():            quadruped_parkour_env/parkour_env.py:356-394 (clip :360, ctrl[:16]
//                      :363-364, 10 mj_step's :367-368, obstacle motors after physics :371,
//                      truncation tested before the counter increments :381,384)
//   observation:       :396-468 (95 floats: post-integration qpos/qvel, stale xpos; foot
//                      "contacts" compare contact geom ids with foot BODY ids :470-485, quirk
//                      P2; constant lidar :504-530; next-two-obstacle table :532-557; terrain
//                      constants :619-634; the distance slot is never reached, P4)
//   reward:            :646-725 (numpy-2 promotion reproduced: float32 after the energy term
//                      unless the progress term made the reward an np.float64)
//   termination:       :727-755
//   dynamic obstacles: :776-795 (t = step_count * 0.01 with the pre-increment count)
//   reset:             :314-354, _randomize_obstacles :757-774 (joint ids as qpos indices, P1)
#pragma once
#include "../../include/mgx.h"
#include "mgx_soccer.h"

namespace mgx {

template <typename T>
struct ParkourIds {
  int torso, feet[4];
  int platform_qpos, pendulum_qpos;  // joint ids used as qpos indices (quirk P1)
  int platform_act, pendulum_act;    // actuator ids of the obstacle motors
  int n_leg, max_episode_steps;
  float act_lim[16];                 // action_space bounds, float32 (parkour_env.py:236-249)
};

// per-env task state: mgx_parkour_env (include/mgx.h), env-major device buffers
using ParkourState = mgx_parkour_env;

__device__ __constant__ static const float kParkourObs[12][4] = {
    // x, type code, height, difficulty (parkour_env.py:282-297, :559-617)
    {8.0f, 1.0f, 0.225f, 0.3f}, {16.0f, 2.0f, 0.2f, 0.6f},  {24.0f, 3.0f, 0.5f, 0.8f},  {30.0f, 4.0f, 0.6f, 0.4f},
    {36.0f, 5.0f, 0.6f, 0.7f},  {44.0f, 6.0f, 0.3f, 0.9f},  {50.0f, 7.0f, 0.08f, 0.5f}, {58.0f, 8.0f, 0.4f, 0.6f},
    {72.0f, 9.0f, 0.25f, 0.4f}, {78.0f, 10.0f, 0.3f, 0.8f}, {88.0f, 11.0f, 0.0f, 1.0f}, {92.0f, 12.0f, 0.2f, 1.0f}};
// the table's float64 values as the reference holds them (Python floats)
__device__ __forceinline__ double parkour_obs_d(int k, int f) {
  const double t[12][4] = {{8.0, 1.0, 0.225, 0.3}, {16.0, 2.0, 0.2, 0.6},  {24.0, 3.0, 0.5, 0.8},
                           {30.0, 4.0, 0.6, 0.4},  {36.0, 5.0, 0.6, 0.7},  {44.0, 6.0, 0.3, 0.9},
                           {50.0, 7.0, 0.08, 0.5}, {58.0, 8.0, 0.4, 0.6},  {72.0, 9.0, 0.25, 0.4},
                           {78.0, 10.0, 0.3, 0.8}, {88.0, 11.0, 0.0, 1.0}, {92.0, 12.0, 0.2, 1.0}};
  return t[k][f];
}

// action clip against the float32 bounds -> ctrl[:n_leg] (parkour_env.py:359-364), in the action's
// dtype (a float64 action stays float64)
template <typename T>
__device__ __forceinline__ void parkour_pre(const DevModel<T>& m, Env<T>& e, const ParkourIds<T>& ids, ActRow act) {
  int l = lane_id();
  if (l < ids.n_leg) {
    if (act.f64) {
      double a = act.d()[l], lim = (double)ids.act_lim[l];
      a = a < -lim ? -lim : (a > lim ? lim : a);
      e.ctrl[l] = (T)a;
    } else {
      float a = act.f()[l], lim = ids.act_lim[l];
      a = a < -lim ? -lim : (a > lim ? lim : a);
      e.ctrl[l] = (T)a;
    }
  }
  wsync();
}

// foot "contact" bitmask: bit i set if any contact's geom1/geom2 equals feet[i] (body ids!)
template <typename T>
__device__ __forceinline__ int parkour_foot_mask(const Env<T>& e, const ParkourIds<T>& ids) {
  int mask = 0;
  for (int base = 0; base < e.ncon; base += 64) {
    int c = base + lane_id();
    int g1 = -2, g2 = -2;
    if (c < e.ncon) { g1 = e.con_geom[2 * c]; g2 = e.con_geom[2 * c + 1]; }
    for (int i = 0; i < 4; i++) {
      bool hit = c < e.ncon && (g1 == ids.feet[i] || g2 == ids.feet[i]);
      if (ballot(hit)) mask |= 1 << i;
    }
  }
  return mask;
}

// the reference's np.sum(np.abs(clip(a))) over 16 values in the action's dtype (float32 or
// float64): numpy's pairwise sum (eight partial sums r[j] = a[j] + a[j+8], then
// ((r0+r1)+(r2+r3)) + ((r4+r5)+(r6+r7)))
template <typename A>
__device__ __forceinline__ A np_sum16_abs_clip(const A* a, const float* lim) {
#pragma clang fp contract(off)
  A v[16];
  for (int j = 0; j < 16; j++) {
    A x = a[j], lo = (A)-lim[j], hi = (A)lim[j];
    x = x < lo ? lo : (x > hi ? hi : x);
    v[j] = x < (A)0 ? -x : x;
  }
  A r[8];
  for (int j = 0; j < 8; j++) r[j] = v[j] + v[j + 8];
  return ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
}

// Observation: 95 float32 (parkour_env.py:396-468)
template <typename T>
__device__ __forceinline__ void parkour_obs(const DevModel<T>& m, const Env<T>& e, const ParkourIds<T>& ids, int foot_mask,
                                            float* obs) {
  int l = lane_id();
  const T* tx = e.xpos + 3 * ids.torso;
  // next two obstacles beyond the torso x (first two table entries with pos > x)
  double x = (double)tx[0];
  int k0 = -1, k1 = -1;
  for (int k = 0; k < 12; k++) {
    if (parkour_obs_d(k, 0) > x) {
      if (k0 < 0) k0 = k;
      else if (k1 < 0) k1 = k;
    }
  }
  for (int i = l; i < 95; i += 64) {
    float v = 0.0f;
    if (i < 16) v = (float)e.qpos[7 + i];
    else if (i < 32) v = (float)e.qvel[6 + (i - 16)];
    else if (i < 36) v = (float)e.qpos[3 + (i - 32)];
    else if (i < 42) v = (float)e.qvel[i - 36];
    else if (i < 45) v = (float)e.qpos[i - 42];
    else if (i < 49) v = (foot_mask >> (i - 45)) & 1 ? 1.0f : 0.0f;
    else if (i < 61) {
      int f = (i - 49) / 3, c = (i - 49) % 3;
      v = (float)(e.xpos[3 * ids.feet[f] + c] - tx[c]);
    } else if (i < 85) v = 10.0f;
    else if (i < 93) {
      int slot = (i - 85) / 4, f = (i - 85) % 4;
      int k = slot == 0 ? k0 : k1;
      if (k >= 0) v = f == 0 ? (float)(parkour_obs_d(k, 0) - x) : kParkourObs[k][f];
    } else if (i == 93) v = 0.0f;
    else v = 0.8f;
    obs[i] = v;
  }
}

// reward + termination + counters (parkour_env.py:646-755, :381-385); returns done
template <typename T>
__device__ __forceinline__ bool parkour_post(const DevModel<T>& m, Env<T>& e, const ParkourIds<T>& ids, ActRow act,
                                             ParkourState ps, int env, float* obs, double* reward, uint8_t* terminated,
                                             uint8_t* truncated) {
#pragma clang fp contract(off)
  int l = lane_id();
  int st = ps.step[env];
  // dynamic obstacles for the NEXT step's physics (t from the pre-increment count)
  if (l == 0) {
    double t = (double)st * 0.01;
    if (ids.platform_act >= 0) e.ctrl[ids.platform_act] = (T)(50.0 * sin(0.5 * t));
    if (ids.pendulum_act >= 0) e.ctrl[ids.pendulum_act] = (T)(100.0 * sin(0.3 * t));
  }
  int fm = parkour_foot_mask(e, ids);
  parkour_obs(m, e, ids, fm, obs + (size_t)env * 95);
  wsync();
  T* lp = (T*)ps.last_position + 3 * (size_t)env;
  const T* tx = e.xpos + 3 * ids.torso;
  double x = (double)tx[0], y = (double)tx[1], z = (double)tx[2];
  int done = 0;
  if (l == 0) {
    int reached = ps.reached[env], falls = ps.fall_count[env], stuck = ps.stuck[env];
    double mp = (double)((T*)ps.max_progress)[env];
    double r = 0.0;
    r -= 20.0;
    double progress = x - (double)lp[0];
    if (progress > 0) {
      r += progress * 500.0;
      mp = mp > x ? mp : x;
    } else if (progress < -0.1) {
      r -= 100.0;
    }
    const int cps[6] = {15, 30, 45, 60, 75, 90};
    for (int b = 0; b < 6; b++)
      if (!((reached >> b) & 1) && x >= (double)cps[b]) { reached |= 1 << b; r += 1000.0; }
    for (int b = 0; b < 12; b++)
      if (!((reached >> (6 + b)) & 1) && x > parkour_obs_d(b, 0) + 2.0) {
        reached |= 1 << (6 + b);
        r += 1000.0 + parkour_obs_d(b, 3) * 1000.0;
      }
    if (x >= 98.0) r += 5000.0;
    if (fabs((double)e.qpos[3]) > 0.7) r += 100.0;
    int nfeet = __popc(fm);
    if (nfeet >= 1 && nfeet <= 3) r += 200.0;
    bool f32 = !(progress > 0);
    float rf = 0.0f;
    if (act.f64) {
      // float64 action: np.float64 effort, so the reward is np.float64 from here on
      r = r - np_sum16_abs_clip(act.d(), ids.act_lim) * 0.1;
      f32 = false;
    } else {
      const float effort = np_sum16_abs_clip(act.f(), ids.act_lim) * 0.1f;
      if (f32) rf = (float)r - effort;
      else r = r - (double)effort;
    }
    bool low = z < 0.2, many = e.ncon > 8;
    if (low) falls += 1;
    bool still = fabs(progress) < 0.01;
    stuck = still ? stuck + 1 : 0;
    bool stuck_pen = still && stuck > 100;
    if (f32) {
      if (low) rf -= 2000.0f;
      if (many) rf -= 500.0f;
      if (stuck_pen) rf -= 100.0f;
      r = (double)rf;
    } else {
      if (low) r -= 2000.0;
      if (many) r -= 500.0;
      if (stuck_pen) r -= 100.0;
    }
    bool term = x >= 98.0 || z < 0.15 || fabs(y) > 10.0 || stuck > 1000 || falls > 3;
    bool trunc = st >= ids.max_episode_steps;
    // episode_reward += reward with numpy promotion (oracle/parkour_logic.py accumulate)
    int kind = ps.er_kind[env];
    double er = ps.episode_reward[env];
    if (f32 && kind != 1) { er = (double)((float)er + (float)r); kind = 2; }
    else { er = er + r; kind = 1; }
    ps.episode_reward[env] = er;
    ps.er_kind[env] = (uint8_t)kind;
    ps.reached[env] = reached;
    ps.fall_count[env] = falls;
    ps.stuck[env] = stuck;
    ps.step[env] = st + 1;
    ((T*)ps.max_progress)[env] = (T)mp;
    reward[env] = r;
    terminated[env] = term;
    truncated[env] = trunc;
    done = term || trunc;
  }
  wsync();
  if (l < 3) lp[l] = tx[l];
  return __shfl(done, 0) != 0;
}

// Philox draws for the vector env's parkour resets: lane j < 2 -> draw j of `episode`
template <typename T>
__device__ __forceinline__ void parkour_philox_draws(uint64_t seed, uint32_t genv, uint32_t episode, T* out) {
  int j = lane_id();
  if (j < 2) {
    uint32_t c[4] = {episode, (uint32_t)j, 0x9A4C0u, 0u};
    philox4x32(c, (uint32_t)seed ^ genv, (uint32_t)(seed >> 32));
    double u = ((double)(c[0] >> 5) * 67108864.0 + (double)(c[1] >> 6)) * (1.0 / 9007199254740992.0);
    double lo = j == 0 ? -1.5 : -1.0, hi = j == 0 ? 1.5 : 1.0;
    out[j] = (T)(lo + (hi - lo) * u);
  }
}

// reset(): mj_resetData, start pose, obstacle draws (P1), tracking reset, 10 settle steps, obs
template <typename T>
__device__ __forceinline__ int parkour_reset_body(const DevModel<T>& m, Env<T>& e, const ParkourIds<T>& ids, T d0, T d1,
                                                  ParkourState ps, int env, float* obs) {
  reset_env(m, e);
  int l = lane_id();
  if (l == 0) {
    e.qpos[0] = (T)2.0; e.qpos[1] = (T)0.0; e.qpos[2] = (T)0.6;
    e.qpos[3] = (T)1; e.qpos[4] = 0; e.qpos[5] = 0; e.qpos[6] = 0;
    e.qpos[ids.platform_qpos] = d0;
    e.qpos[ids.pendulum_qpos] = d1;
  }
  wsync();
  int warn = 0;
  for (int k = 0; k < 10; k++) warn += mj_step_env(m, e);  // parkour_env.py:347-348
  int fm = parkour_foot_mask(e, ids);
  parkour_obs(m, e, ids, fm, obs + (size_t)env * 95);
  T* lp = (T*)ps.last_position + 3 * (size_t)env;
  if (l == 0) {
    lp[0] = (T)2.0; lp[1] = (T)0.0; lp[2] = (T)0.6;
    ((T*)ps.max_progress)[env] = 0;
    ps.episode_reward[env] = 0.0;
    ps.er_kind[env] = 0;
    ps.reached[env] = 0; ps.fall_count[env] = 0; ps.stuck[env] = 0; ps.step[env] = 0;
  }
  wsync();
  return warn;
}

}  // namespace mgx
