// mgx_soccer.h — humanoid_soccer_env task logic fused around the physics step.
//
// Restates, per env and on the GPU, the reference's Python around mj_step:
//   step():          humanoid_soccer_env/soccer_env.py:398-452
//   goalkeeper:      :506-524   (reads the STALE ball xpos of the previous forward pass,
//                                writes qfrc_applied[joint id 0]; persists otherwise)
//   wind:            :526-537   (xfrc_applied[ball, :2] accumulates while ball z > 0.5)
//   observation:     :539-631   (80 floats; "torso" velocities are qvel[0:6] = goalkeeper +
//                                ball dofs)
//   reward:          :633-690, ball contact :787-803, upright :818-833
//   termination:     :692-716, truncation :427
//   reset:           :347-396, randomisation :454-504 (applied with the aliasing quirk S1)
#pragma once
#include "mgx_physics.h"

namespace mgx {

template <typename T>
struct SoccerIds {
  int torso, ball, goalkeeper, ball_geom, right_foot, left_foot, field_geom;
  int ball_qposadr, ball_dofadr, gk_qposadr, gk_qfrc_index, max_episode_steps;
  int obs_qposadr[25], obs_dofadr[25];
  T obs_lo[25], obs_hi[25];
  uint64_t robot_mask_lo, robot_mask_hi;
  int root_qposadr;        // jnt_qposadr[0] (soccer_env.py:463,468)
  int noise_qposadr[29];   // joint_indices -> qposadr (soccer_env.py:480-488)
  T noise_lo[29], noise_hi[29];
  int n_noise;
};

// One env's action row: float32, or float64 (mgx_soccer_env.action_f64) — the reference's np.clip
// against the float32 action_space bounds keeps a float64 policy's action float64, so ctrl and
// the energy term then follow in float64 (soccer_env.py:401-405, :674).
using SoccerAct = ActRow;

// Pre-physics env logic: action clip -> ctrl, goalkeeper, wind (soccer_env.py:401-411)
template <typename T>
__device__ __forceinline__ void soccer_pre(const DevModel<T>& m, Env<T>& e, const SoccerIds<T>& ids, SoccerAct act,
                           const T* prev_ball, const T* wind) {
  int l = lane_id();
  for (int u = l; u < m.nu; u += 64) {
    if (act.f64) {
      double a = static_cast<const double*>(act.p)[u];
      a = a < -150.0 ? -150.0 : (a > 150.0 ? 150.0 : a);  // float64 action, float32 bounds: float64
      e.ctrl[u] = (T)a;
    } else {
      float a = static_cast<const float*>(act.p)[u];
      a = a < -150.0f ? -150.0f : (a > 150.0f ? 150.0f : a);   // action_space bounds, float32
      e.ctrl[u] = (T)a;
    }
  }
  // goalkeeper P-controller on the stale ball position
  T bx = prev_ball[0], by = prev_ball[1], bz = prev_ball[2];
  if (bx < (T)-10) {
    T target = clampv(by, (T)-3, (T)3);
    T err = target - e.qpos[ids.gk_qposadr];
    T force = clampv((T)50 * err, (T)-100, (T)100);
    if (l == ids.gk_qfrc_index) e.qfrc_applied = force;
  }
  // wind on the ball body while airborne
  if (bz > (T)0.5 && l < 2) e.xfrc[6 * ids.ball + l] += wind[0] * wind[1 + l] * (T)0.1;
  wsync();
}

template <typename T>
__device__ __forceinline__ T clip1(T x) { return clampv(x, (T)-1, (T)1); }

template <typename T>
__device__ __forceinline__ T norm3v(T a, T b, T c) { return sqrt(a * a + b * b + c * c); }

// Observation (80 floats) from the forward-pass frames + post-integration qpos/qvel.
template <typename T>
__device__ __forceinline__ void soccer_obs(const DevModel<T>& m, Env<T>& e, const SoccerIds<T>& ids, int step, float* obs) {
  int l = lane_id();
  // foot "contact forces": last matching contact wins (soccer_env.py:765-785)
  int lastR = -1, lastL = -1;
  for (int base = 0; base < e.ncon; base += 64) {
    int c = base + l;
    bool mr = false, ml = false;
    if (c < e.ncon) {
      int g1 = e.con_geom[2 * c], g2 = e.con_geom[2 * c + 1];
      mr = (g1 == ids.right_foot && g2 == 0) || (g2 == ids.right_foot && g1 == 0);
      ml = (g1 == ids.left_foot && g2 == 0) || (g2 == ids.left_foot && g1 == 0);
    }
    unsigned long long br = ballot(mr), bl = ballot(ml);
    if (br) lastR = base + 63 - __clzll(br);
    if (bl) lastL = base + 63 - __clzll(bl);
  }
  const T* tx = e.xpos + 3 * ids.torso;
  const T* bxp = e.xpos + 3 * ids.ball;
  for (int i = l; i < 80; i += 64) {
    T v = 0;
    if (i < 25) {
      T q = e.qpos[ids.obs_qposadr[i]], lo = ids.obs_lo[i], hi = ids.obs_hi[i];
      v = lo < hi ? clip1((T)2 * (q - lo) / (hi - lo) - (T)1) : (T)0;
    } else if (i < 50) {
      v = clip1(e.qvel[ids.obs_dofadr[i - 25]] / (T)10);
    } else if (i < 54) {
      v = e.xquat[4 * ids.torso + (i - 50)];
    } else if (i < 57) {
      v = clip1(e.qvel[i - 54] / (T)5);
    } else if (i < 60) {
      v = clip1(e.qvel[3 + (i - 57)] / (T)10);
    } else if (i < 63) {
      v = clip1((bxp[i - 60] - tx[i - 60]) / (T)30);
    } else if (i < 66) {
      v = clip1(e.qvel[ids.ball_dofadr + (i - 63)] / (T)20);
    } else if (i < 69) {
      const T goal[3] = {(T)24.5, (T)0, (T)1.22};
      v = clip1((goal[i - 66] - tx[i - 66]) / (T)30);
    } else if (i < 73) {
      int k = i - 69;
      int c = k < 2 ? lastR : lastL;
      T f = 0;
      if (c >= 0) {
        f = (k & 1) == 0 ? e.con_dist[c] : e.con_mu[c];
      }
      v = clip1(f / (T)1000);
    } else if (i < 76) {
      v = clip1(e.subtree_com[3 * ids.torso + (i - 73)] / (T)30);
    } else if (i == 76) {
      v = (T)1 - (T)step / (T)ids.max_episode_steps;
    } else if (i == 77) {
      T d = norm3v(bxp[0] - tx[0], bxp[1] - tx[1], bxp[2] - tx[2]);
      v = clampv(d / (T)50, (T)0, (T)1);
    } else {
      v = clip1(e.xpos[3 * ids.goalkeeper + (i - 78)] / (T)15);
    }
    obs[i] = (float)v;
  }
}

template <typename T>
__device__ __forceinline__ bool soccer_ball_contact(Env<T>& e, const SoccerIds<T>& ids) {
  bool hit = false;
  for (int base = 0; base < e.ncon; base += 64) {
    int c = base + lane_id();
    if (c < e.ncon) {
      int g1 = e.con_geom[2 * c], g2 = e.con_geom[2 * c + 1];
      if (g1 == ids.ball_geom || g2 == ids.ball_geom) {
        int other = g1 == ids.ball_geom ? g2 : g1;
        uint64_t mask = other < 64 ? ids.robot_mask_lo : ids.robot_mask_hi;
        if (other < 128 && ((mask >> (other & 63)) & 1ull)) hit = true;
      }
    }
  }
  return ballot(hit) != 0ull;
}

template <typename T>
__device__ __forceinline__ bool soccer_upright(const Env<T>& e, const SoccerIds<T>& ids) {
  T q[4] = {e.xquat[4 * ids.torso], e.xquat[4 * ids.torso + 1], e.xquat[4 * ids.torso + 2], e.xquat[4 * ids.torso + 3]};
  T R[9];
  quat2mat(R, q);
  return R[8] > (T)0.7;
}

// numpy's np.linalg.norm of a float64 3-vector: sqrt of the BLAS dot, which rounds as two FMAs
__device__ __forceinline__ double norm3_np(double x, double y, double z) { return sqrt(fma(z, z, fma(y, y, x * x))); }

// numpy add.reduce of the squared clipped actions (soccer_env.py:674) in the action's dtype
// (float32 or float64: numpy's pairwise sum is the same for both): 8 accumulators over the first
// 8*floor(n/8) values, tree (01)(23) / (45)(67), then the tail
template <typename A>
__device__ __forceinline__ A np_sumsq_clip(const A* action, int n) {
#pragma clang fp contract(off)
  auto sq = [&](int u) {
    A a = action[u];
    a = a < (A)-150 ? (A)-150 : (a > (A)150 ? (A)150 : a);
    return a * a;
  };
  if (n < 8) {
    A res = 0;
    for (int u = 0; u < n; u++) res += sq(u);
    return res;
  }
  A r[8];
  for (int k = 0; k < 8; k++) r[k] = sq(k);
  int i = 8;
  for (; i + 8 <= n; i += 8)
    for (int k = 0; k < 8; k++) r[k] += sq(i + k);
  A res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; i++) res += sq(i);
  return res;
}
__device__ __forceinline__ float np_sumsq_clip_f32(const float* action, int n) { return np_sumsq_clip(action, n); }

// _calculate_reward (soccer_env.py:633-690) with the reference's numpy arithmetic, lane-uniform:
// the reward is a Python float until an np.float64 term (approach / forward progress, from
// np.linalg.norm) is added; the energy term -0.1 * np.sum(np.square(a)) is np.float32, so a
// still-Python-float reward becomes float32 there (NEP 50) and a later np.float64 term (ball
// progress) promotes it back. Positions enter as float64 whatever the physics precision.
__device__ __forceinline__ double soccer_reward_np(bool goal_now, bool ball_contact, bool upright, const double* bp,
                                                   const double* tx, const double* pb, const double* pr,
                                                   float energy, bool e64 = false, double energy64 = 0.0) {
#pragma clang fp contract(off)
  double r = 0.0;
  bool is64 = false;
  if (goal_now) r += 10000.0;
  if (ball_contact) r += 1000.0;
  double cur_bd = norm3_np(bp[0] - tx[0], bp[1] - tx[1], bp[2] - tx[2]);
  double prev_bd = norm3_np(pb[0] - pr[0], pb[1] - pr[1], pb[2] - pr[2]);
  if (cur_bd < prev_bd && cur_bd > 2.0) { r += 500.0 * (prev_bd - cur_bd); is64 = true; }
  if (upright) r += 200.0;
  double prev_gd = norm3_np(pr[0] - 24.5, pr[1] - 0.0, pr[2] - 0.0);
  double cur_gd = norm3_np(tx[0] - 24.5, tx[1] - 0.0, tx[2] - 0.0);
  if (cur_gd < prev_gd) { r += 100.0 * (prev_gd - cur_gd); is64 = true; }
  const float eterm = -0.1f * energy;
  if (e64) {  // float64 action: the energy term and everything after it in float64
    r += -0.1 * energy64;
    if (!upright) r += -1000.0;
  } else if (is64) {
    r += (double)eterm;
    if (!upright) r += -1000.0;
  } else {
    float rf = (float)r + eterm;
    if (!upright) rf += -1000.0f;
    r = (double)rf;
  }
  double prev_bgd = norm3_np(pb[0] - 24.5, pb[1] - 0.0, pb[2] - 0.0);
  double cur_bgd = norm3_np(bp[0] - 24.5, bp[1] - 0.0, bp[2] - 0.0);
  if (cur_bgd < prev_bgd) r += 300.0 * (prev_bgd - cur_bgd);
  return r;
}

// Post-physics: step count, obs, reward, termination, stats, prev snapshots
template <typename T>
__device__ __forceinline__ bool soccer_post(const DevModel<T>& m, Env<T>& e, const SoccerIds<T>& ids, SoccerAct act, int* step,
                            uint8_t* goal_scored, T* prev_ball, T* prev_robot, T* stats, float* obs, double* reward,
                            uint8_t* terminated, uint8_t* truncated, uint8_t* flags = nullptr) {
#pragma clang fp contract(off)
  int l = lane_id();
  int st = *step + 1;
  soccer_obs(m, e, ids, st, obs);
  const T* tx = e.xpos + 3 * ids.torso;
  const T* bp = e.xpos + 3 * ids.ball;
  bool goal_now = bp[0] > (T)24 && fabs(bp[1]) < (T)3.66 && bp[2] < (T)2.44;
  bool ball_contact = soccer_ball_contact(e, ids);
  bool upright = soccer_upright(e, ids);
  const double bpd[3] = {(double)bp[0], (double)bp[1], (double)bp[2]};
  const double txd[3] = {(double)tx[0], (double)tx[1], (double)tx[2]};
  const double pbd[3] = {(double)prev_ball[0], (double)prev_ball[1], (double)prev_ball[2]};
  const double prd[3] = {(double)prev_robot[0], (double)prev_robot[1], (double)prev_robot[2]};
  const double r =
      act.f64 ? soccer_reward_np(goal_now, ball_contact, upright, bpd, txd, pbd, prd, 0.0f, true,
                                 np_sumsq_clip(static_cast<const double*>(act.p), m.nu))
              : soccer_reward_np(goal_now, ball_contact, upright, bpd, txd, pbd, prd,
                                 np_sumsq_clip_f32(static_cast<const float*>(act.p), m.nu));
  bool gs = (*goal_scored != 0) || goal_now;
  bool term = gs || (!upright && st > 100) ||
              (fabs(bp[0]) > (T)30 || fabs(bp[1]) > (T)20 || bp[2] < (T)-1 || bp[2] > (T)10) ||
              (fabs(tx[0]) > (T)30 || fabs(tx[1]) > (T)20 || tx[2] < (T)0 || tx[2] > (T)5);
  bool trunc = st >= ids.max_episode_steps;
  // episode stats (soccer_env.py:640-662 in the reward, :718-730 after the flags), then the
  // prev_* snapshots (:444-446)
  double bv = norm3_np((double)e.qvel[ids.ball_dofadr], (double)e.qvel[ids.ball_dofadr + 1],
                       (double)e.qvel[ids.ball_dofadr + 2]);
  double dist = norm3_np(txd[0] - prd[0], txd[1] - prd[1], txd[2] - prd[2]);
  wsync();
  if (l == 0) {
    if (goal_now) stats[0] += 1;
    if (ball_contact) stats[1] += 1;
    if (upright) stats[3] = (T)((double)stats[3] + (double)m.timestep);
    stats[2] = (T)((double)stats[2] + dist);
    stats[4] = (double)stats[4] >= bv ? stats[4] : (T)bv;
    *reward = r;
    *terminated = term;
    *truncated = trunc;
    *goal_scored = gs;
    *step = st;
    if (flags) { flags[0] = ball_contact; flags[1] = upright; }
  }
  if (l < 3) { prev_ball[l] = bp[l]; prev_robot[l] = tx[l]; }
  return term || trunc;
}

// Counter-based reset draws for the vector env: Philox4x32-10 keyed by (seed, global env
// index), counter = (episode, word). Independent of how envs are sharded over GPUs.
__device__ __forceinline__ void philox4x32(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; r++) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
    uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}
// the reference's ranges, in draw order (soccer_env.py:458-504)
__device__ __forceinline__ void soccer_draw_ranges(int j, int n_noise, double* lo, double* hi) {
  if (j == 0) { *lo = -15; *hi = -5; }
  else if (j == 1) { *lo = -10; *hi = 10; }
  else if (j == 2) { *lo = -0.5; *hi = 0.5; }
  else if (j < 3 + n_noise) { *lo = -0.1; *hi = 0.1; }
  else if (j == 3 + n_noise) { *lo = -2; *hi = 2; }
  else if (j == 4 + n_noise) { *lo = 0; *hi = 2; }
  else if (j == 5 + n_noise) { *lo = 0; *hi = 6.283185307179586; }
  else { *lo = 0.05; *hi = 0.15; }
}
// lane j < 36 produces draw j of episode `episode` for global env `genv` into `out` (LDS/global)
template <typename T>
__device__ __forceinline__ void soccer_philox_draws(uint64_t seed, uint32_t genv, uint32_t episode, int n_noise, T* out) {
  int j = lane_id();
  if (j < 36) {
    uint32_t c[4] = {episode, (uint32_t)j, 0x50C3Eu, 0u};
    philox4x32(c, (uint32_t)seed ^ genv, (uint32_t)(seed >> 32));
    double u = ((double)(c[0] >> 5) * 67108864.0 + (double)(c[1] >> 6)) * (1.0 / 9007199254740992.0);
    double lo, hi;
    soccer_draw_ranges(j, n_noise, &lo, &hi);
    out[j] = (T)(lo + (hi - lo) * u);
  }
}

// Reset: mj_resetData + the reference's randomisation (draws in reference order), with the
// jnt_qposadr[0] aliasing quirk (the robot pose lands on goalkeeper + ball qpos).
template <typename T>
__device__ __forceinline__ void soccer_apply_reset(const DevModel<T>& m, Env<T>& e, const SoccerIds<T>& ids, const T* draws, T* wind) {
  reset_env(m, e);
  int l = lane_id();
  if (l == 0) {
    T rx = draws[0], ry = draws[1], ang = draws[2];
    int a0 = ids.root_qposadr;
    e.qpos[a0] = rx; e.qpos[a0 + 1] = ry; e.qpos[a0 + 2] = (T)1.4;
    e.qpos[a0 + 3] = cos(ang / 2); e.qpos[a0 + 4] = 0; e.qpos[a0 + 5] = 0; e.qpos[a0 + 6] = sin(ang / 2);
    e.qpos[ids.ball_qposadr] = rx + (T)2; e.qpos[ids.ball_qposadr + 1] = ry; e.qpos[ids.ball_qposadr + 2] = (T)0.15;
    for (int i = 0; i < ids.n_noise; i++) {
      T lo = ids.noise_lo[i], hi = ids.noise_hi[i];
      e.qpos[ids.noise_qposadr[i]] = clampv((lo + hi) / (T)2 + draws[3 + i], lo, hi);
    }
    e.qpos[ids.gk_qposadr] = draws[3 + ids.n_noise];
    wind[0] = draws[4 + ids.n_noise];
    wind[1] = cos(draws[5 + ids.n_noise]);
    wind[2] = sin(draws[5 + ids.n_noise]);
  }
  wsync();
}

}  // namespace mgx
