// mgx_dancing.h — humanoid_dancing_env task logic fused around the RK4 physics step.
//
// Restates, per env and on the GPU, the reference's Python around mj_step:
//   step():      humanoid_dancing_env/dancing_env.py:833-894 (clip :837, ctrl :840; rhythm
//                :924-937 and spotlight :939-955 BEFORE mj_step, reading the stale torso xpos;
//                counter :849)
//   observation: :1028-1120 (94 floats; joint i's range normalises qpos[7 + i] -- the model
//                has no root joint -- slots past nq / nv are 0)
//   reward:      :1122-1207 (float64; the energy term is a float32 product, numpy pairwise sum)
//   termination: :1209-1235 (fall_start_step created lazily, deleted when upright, survives
//                reset)
//   after:       _update_episode_stats :1004-1026, _update_crowd_excitement :975-1002,
//                _check_move_transition :957-973
//   reset:       :763-831, _generate_dance_sequence :896-905, _set_initial_pose :907-922
//                (qpos[0:7] of the first seven hinges); spotlight / disco rotation persist.
#pragma once
#include "../../include/mgx.h"
#include "mgx_soccer.h"

namespace mgx {

// scal[] slots of mgx_dancing_env (include/mgx.h)
enum {
  DS_TBEAT = 0, DS_DISCO = 1, DS_SPOT = 2, DS_COMBO = 5, DS_SCORE = 6, DS_MSTART = 7, DS_CROWD = 8, DS_APPLAUSE = 9,
  DS_STATS = 10, DS_TORSO = 15, DS_N = 18
};
// ints[] slots
enum { DI_STEP = 0, DI_BEATS = 1, DI_MEASURE = 2, DI_MOVE = 3, DI_HISTLEN = 4, DI_FALLSTART = 5, DI_FALLPRESENT = 6,
       DI_N = 8 };
#define MGX_DANCE_SEQ 20
#define MGX_DANCE_OBS 94

struct DancingIds {
  int torso, right_foot, left_foot, floor, stage;
  int n_act, max_episode_steps, n_range;   // n_range = joints whose range normalises qpos[7 + i]
  double jnt_lo[32], jnt_hi[32];
};

__device__ __forceinline__ int dance_difficulty(int mv) {
  const int d[10] = {1, 2, 2, 3, 2, 1, 2, 3, 2, 4};   // dancing_env.py:57-68
  return d[mv < 0 ? 0 : (mv > 9 ? 9 : mv)];
}

__device__ __forceinline__ double clipd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }

// numpy pairwise add.reduce over 29 contiguous values (8 accumulators over 24, tree, tail 5)
template <typename R>
__device__ __forceinline__ R np_sum29(const R* v) {
#pragma clang fp contract(off)
  R r[8];
  for (int j = 0; j < 8; j++) r[j] = (v[j] + v[j + 8]) + v[j + 16];
  R res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (int j = 24; j < 29; j++) res += v[j];
  return res;
}

// action clip (in the action's dtype) -> ctrl, rhythm, disco ball, spotlight (dancing_env.py:835-846)
template <typename T>
__device__ __forceinline__ void dancing_pre(const DevModel<T>& m, Env<T>& e, const DancingIds& ids, ActRow act,
                                            mgx_dancing_env de, int env) {
#pragma clang fp contract(off)
  int l = lane_id();
  if (l < ids.n_act) {
    if (act.f64) {
      double a = act.d()[l];
      a = a < -200.0 ? -200.0 : (a > 200.0 ? 200.0 : a);
      e.ctrl[l] = (T)a;
    } else {
      float a = act.f()[l];
      a = a < -200.0f ? -200.0f : (a > 200.0f ? 200.0f : a);
      e.ctrl[l] = (T)a;
    }
  }
  if (l == 0) {
    double* S = de.scal + (size_t)env * DS_N;
    int* I = de.ints + (size_t)env * DI_N;
    double t = S[DS_TBEAT] + 0.01667;
    if (t >= 0.5) {
      t -= 0.5;
      I[DI_BEATS] += 1;
      if (I[DI_BEATS] % 4 == 0) I[DI_MEASURE] += 1;
    }
    S[DS_TBEAT] = t;
    double d = S[DS_DISCO] + 0.5 * 0.01667;
    if (d > 2 * 3.141592653589793) d -= 2 * 3.141592653589793;
    S[DS_DISCO] = d;
    const double tg[3] = {S[DS_TORSO], S[DS_TORSO + 1], 5.0};
    for (int k = 0; k < 3; k++) S[DS_SPOT + k] = S[DS_SPOT + k] + 0.1 * (tg[k] - S[DS_SPOT + k]);
  }
  wsync();
}

// foot indicators (dancing_env.py:1249-1266): bit 0 right, bit 1 left
template <typename T>
__device__ __forceinline__ int dancing_feet(const Env<T>& e, const DancingIds& ids) {
  int mask = 0;
  for (int base = 0; base < e.ncon; base += 64) {
    int c = base + lane_id();
    bool r = false, lf = false;
    if (c < e.ncon) {
      int g1 = e.con_geom[2 * c], g2 = e.con_geom[2 * c + 1];
      bool gr1 = g1 == ids.floor || g1 == ids.stage, gr2 = g2 == ids.floor || g2 == ids.stage;
      r = (g1 == ids.right_foot && gr2) || (g2 == ids.right_foot && gr1);
      lf = (g1 == ids.left_foot && gr2) || (g2 == ids.left_foot && gr1);
    }
    if (ballot(r)) mask |= 1;
    if (ballot(lf)) mask |= 2;
  }
  return mask;
}

// Observation: 94 float32 (dancing_env.py:1028-1120)
template <typename T>
__device__ __forceinline__ void dancing_obs(const DevModel<T>& m, const Env<T>& e, const DancingIds& ids, const double* S,
                                            const int* I, const int* moves, float* obs) {
  int l = lane_id();
  int feet = dancing_feet(e, ids);
  const T* tx = e.xpos + 3 * ids.torso;
  for (int i = l; i < MGX_DANCE_OBS; i += 64) {
    double v = 0.0;
    if (i < 29) {
      if (i < ids.n_range && 7 + i < m.nq) {
        double lo = ids.jnt_lo[i], hi = ids.jnt_hi[i];
        v = lo < hi ? clipd(2 * ((double)e.qpos[7 + i] - lo) / (hi - lo) - 1, -1.0, 1.0) : 0.0;
      }
    } else if (i < 58) {
      int k = i - 29;
      v = k < m.nv - 6 ? clipd((double)e.qvel[6 + k] / 10.0, -1.0, 1.0) : 0.0;
    } else if (i < 62) v = (double)e.xquat[4 * ids.torso + (i - 58)];
    else if (i < 65) v = clipd((double)e.qvel[i - 62] / 5.0, -1.0, 1.0);
    else if (i < 68) v = clipd((double)e.qvel[3 + (i - 65)] / 10.0, -1.0, 1.0);
    else if (i < 71) v = clipd((double)e.subtree_com[3 * ids.torso + (i - 68)] / 10.0, -1.0, 1.0);
    else if (i < 73) v = (feet >> (i - 71)) & 1 ? 1.0 : 0.0;
    else if (i < 76) v = 0.0;
    else if (i == 76) v = S[DS_TBEAT] / 0.5;
    else if (i == 77) v = (0.5 - S[DS_TBEAT]) / 0.5;
    else if (i < 88) v = (I[DI_MOVE] < MGX_DANCE_SEQ && moves[I[DI_MOVE]] == i - 78) ? 1.0 : 0.0;
    else if (i == 88) v = clipd(S[DS_COMBO] / 10.0, 0.0, 1.0);
    else if (i == 89) v = S[DS_CROWD];
    else if (i < 93) v = clipd((S[DS_SPOT + (i - 90)] - (double)tx[i - 90]) / 10.0, -1.0, 1.0);
    else {
      double u = S[DS_STATS] / 1000.0;
      v = 1.0 - (u < 1.0 ? u : 1.0);
    }
    obs[i] = (float)v;
  }
}

template <typename T>
__device__ __forceinline__ bool dancing_upright(const Env<T>& e, const DancingIds& ids) {
  T q[4] = {e.xquat[4 * ids.torso], e.xquat[4 * ids.torso + 1], e.xquat[4 * ids.torso + 2], e.xquat[4 * ids.torso + 3]};
  T R[9];
  quat2mat(R, q);
  return R[8] > (T)0.7;
}

// counter, obs, reward, termination, stats, crowd, move transition, prev snapshots
// (dancing_env.py:849-892); returns done
template <typename T>
__device__ __forceinline__ bool dancing_post(const DevModel<T>& m, Env<T>& e, const DancingIds& ids, ActRow act,
                                             mgx_dancing_env de, int env, float* obs, double* reward, uint8_t* terminated,
                                             uint8_t* truncated) {
#pragma clang fp contract(off)
  int l = lane_id();
  double* S = de.scal + (size_t)env * DS_N;
  int* I = de.ints + (size_t)env * DI_N;
  int* H = de.hist + (size_t)env * 3;
  const int* moves = de.moves + (size_t)env * MGX_DANCE_SEQ;
  const double* dur = de.durations + (size_t)env * MGX_DANCE_SEQ;
  double* pj = de.prev_jvel + (size_t)env * (m.nv - 6);
  if (l == 0) I[DI_STEP] += 1;
  wsync();
  dancing_obs(m, e, ids, S, I, moves, obs + (size_t)env * MGX_DANCE_OBS);
  // joint-velocity norms over qvel[6:] (float64 wave sums)
  bool jl = l >= 6 && l < m.nv;
  double qv = jl ? (double)e.qvel[l] : 0.0;
  double dv = jl ? qv - pj[l - 6] : 0.0;
  double mm = sqrt(wave_sum(qv * qv));
  double jerk = sqrt(wave_sum(dv * dv));
  bool up = dancing_upright(e, ids);
  int done = 0;
  wsync();
  if (l == 0) {
    int st = I[DI_STEP];
    double r = 0.0;
    double bp = S[DS_TBEAT] / 0.5;
    double combo = S[DS_COMBO];
    if (bp < 0.1 || bp > 0.9) {
      if (mm > 1.0) { r += 100.0; combo = combo + 0.1 < 10.0 ? combo + 0.1 : 10.0; }
      else combo = combo - 0.05 > 1.0 ? combo - 0.05 : 1.0;
    }
    if (up) {
      r += 30.0;
      if (jerk > 0.5) r += 30.0 * 0.5;
    }
    r += 20.0 * exp(-0.1 * jerk);
    int hl = I[DI_HISTLEN];
    if (hl > 2) {
      int a = H[0], b = H[1], c = H[2];   // the last three moves (hist_len > 2 fills all slots)
      if (a != b && a != c && b != c) r += 50.0;
    }
    int mi = I[DI_MOVE];
    double elapsed = (double)st * 0.01667 - S[DS_MSTART];
    if (mi < MGX_DANCE_SEQ && elapsed > dur[mi] * 0.8) r += 200.0 * (double)dance_difficulty(moves[mi]);
    double used = 0.0;
    for (int i = 0; i < ids.n_range && 7 + i < m.nq; i++) {
      double lo = ids.jnt_lo[i], hi = ids.jnt_hi[i];
      if (lo < hi) used += fabs((double)e.qpos[7 + i] - (lo + hi) / 2) / (hi - lo);
    }
    if (used > 5.0) r += 100.0 * 0.1;
    // energy_penalty * np.sum(np.square(action)) in the action's dtype (:1186-1187)
    if (act.f64) {
      double sq[29];
      for (int j = 0; j < 29; j++) {
        double x = act.d()[j];
        x = x < -200.0 ? -200.0 : (x > 200.0 ? 200.0 : x);
        sq[j] = x * x;
      }
      r += -0.05 * np_sum29(sq);
    } else {
      float sq[29];
      for (int j = 0; j < 29; j++) {
        float x = act.f()[j];
        x = x < -200.0f ? -200.0f : (x > 200.0f ? 200.0f : x);
        sq[j] = x * x;
      }
      r += (double)(-0.05f * np_sum29(sq));
    }
    if (!up) { r += -500.0; combo = 1.0; }
    if (bp > 0.2 && bp < 0.8 && mm > 3.0) r += -50.0 * 0.1;
    if (r > 0) r *= combo;
    double score = S[DS_SCORE] + r;
    // termination (dancing_env.py:1209-1235)
    bool term = false;
    if (!up) {
      if (!I[DI_FALLPRESENT]) { I[DI_FALLPRESENT] = 1; I[DI_FALLSTART] = st; }
      else if (st - I[DI_FALLSTART] > 120) term = true;
    } else if (I[DI_FALLPRESENT]) {
      I[DI_FALLPRESENT] = 0;
      I[DI_FALLSTART] = 0;
    }
    const T* tx = e.xpos + 3 * ids.torso;
    double rx = (double)tx[0], ry = (double)tx[1], rz = (double)tx[2];
    if (!term) term = sqrt(fma(ry, ry, rx * rx)) > 15.0 || rz < 0.0 || rz > 5.0;
    bool trunc = st >= ids.max_episode_steps;
    // _update_episode_stats: energy = numpy pairwise sum of |ctrl| (float64)
    double ac[29];
    for (int j = 0; j < 29; j++) ac[j] = j < m.nu ? fabs((double)e.ctrl[j]) : 0.0;
    S[DS_STATS] += np_sum29(ac) * 0.01667;
    if (bp < 0.1 || bp > 0.9) S[DS_STATS + 1] += 0.01667;
    double lc = (double)(int)combo;
    S[DS_STATS + 2] = S[DS_STATS + 2] > lc ? S[DS_STATS + 2] : lc;
    S[DS_STATS + 3] = S[DS_CROWD];
    S[DS_STATS + 4] = score;
    // _update_crowd_excitement
    double tb = S[DS_TBEAT];
    double on = (tb < 0.1 || tb > 0.5 - 0.1) ? 0.1 : 0.0;
    double cf = (combo / 10.0 < 1.0 ? combo / 10.0 : 1.0) * 0.2;
    double df = mi < MGX_DANCE_SEQ ? (double)dance_difficulty(moves[mi]) / 4.0 * 0.1 : 0.0;
    double crowd = clipd(S[DS_CROWD] + (on + cf + df) * 0.01, 0.0, 1.0);
    crowd *= 0.999;
    S[DS_CROWD] = crowd;
    S[DS_APPLAUSE] = crowd * 100.0;
    // _check_move_transition
    double now = (double)st * 0.01667;
    if (mi < MGX_DANCE_SEQ && now - S[DS_MSTART] >= dur[mi]) {
      mi += 1;
      S[DS_MSTART] = now;
      if (mi < MGX_DANCE_SEQ) {
        int nm = moves[mi];
        if (hl < 3) H[hl] = nm;
        else { H[0] = H[1]; H[1] = H[2]; H[2] = nm; }
        I[DI_HISTLEN] = hl + 1;
      }
      I[DI_MOVE] = mi;
    }
    S[DS_COMBO] = combo;
    S[DS_SCORE] = score;
    S[DS_TORSO] = rx; S[DS_TORSO + 1] = ry; S[DS_TORSO + 2] = rz;
    reward[env] = r;
    terminated[env] = term;
    truncated[env] = trunc;
    done = term || trunc;
  }
  wsync();
  if (jl) pj[l - 6] = qv;
  return __shfl(done, 0) != 0;
}

// Philox draws for the vector env's resets: lane j < 40 -> draw j (even: move index
// floor(10 u), odd: duration U(1, 3)), the reference's order (dancing_env.py:896-905)
template <typename T>
__device__ __forceinline__ void dancing_philox_draws(uint64_t seed, uint32_t genv, uint32_t episode, T* out) {
  int j = lane_id();
  if (j < 2 * MGX_DANCE_SEQ) {
    uint32_t c[4] = {episode, (uint32_t)j, 0xDA4CEu, 0u};
    philox4x32(c, (uint32_t)seed ^ genv, (uint32_t)(seed >> 32));
    double u = ((double)(c[0] >> 5) * 67108864.0 + (double)(c[1] >> 6)) * (1.0 / 9007199254740992.0);
    double v = (j & 1) ? 1.0 + 2.0 * u : floor(10.0 * u);
    out[j] = (T)(v > 9.0 && !(j & 1) ? 9.0 : v);
  }
}

// reset() (dancing_env.py:763-830), split around its 10 settle RK4 steps so the task kernel
// keeps one physics call site: the prologue stores the move sequence (draws read in place,
// global for host draws or LDS for Philox, before the physics reuses the LDS), runs
// mj_resetData, counters and the initial pose; the epilogue writes the observation and the
// prev snapshots. Spotlight, disco rotation and fall_start_step are left alone.
template <typename T>
__device__ __forceinline__ void dancing_reset_prologue(const DevModel<T>& m, Env<T>& e, const T* draws,
                                                       mgx_dancing_env de, int env) {
  int l = lane_id();
  double* S = de.scal + (size_t)env * DS_N;
  int* I = de.ints + (size_t)env * DI_N;
  if (l < MGX_DANCE_SEQ) {
    de.moves[(size_t)env * MGX_DANCE_SEQ + l] = (int)draws[2 * l];
    de.durations[(size_t)env * MGX_DANCE_SEQ + l] = (double)draws[2 * l + 1];
  }
  reset_env(m, e);
  if (l == 0) {
    e.qpos[0] = 0; e.qpos[1] = 0; e.qpos[2] = (T)1.8;
    e.qpos[3] = 1; e.qpos[4] = 0; e.qpos[5] = 0; e.qpos[6] = 0;
    I[DI_STEP] = 0; I[DI_BEATS] = 0; I[DI_MEASURE] = 0; I[DI_MOVE] = 0; I[DI_HISTLEN] = 0;
    S[DS_TBEAT] = 0.0; S[DS_SCORE] = 0.0; S[DS_COMBO] = 1.0; S[DS_CROWD] = 0.5; S[DS_APPLAUSE] = 0.0;
    S[DS_MSTART] = 0.0;
    for (int k = 0; k < 5; k++) S[DS_STATS + k] = 0.0;
    int* H = de.hist + (size_t)env * 3;
    H[0] = H[1] = H[2] = -1;
  }
  wsync();
  for (int k = 7 + l; k < m.nq && k - 7 < m.njnt; k += 64) e.qpos[k] = 0;
  wsync();
}

template <typename T>
__device__ __forceinline__ void dancing_reset_epilogue(const DevModel<T>& m, Env<T>& e, const DancingIds& ids,
                                                       mgx_dancing_env de, int env, float* obs) {
  int l = lane_id();
  double* S = de.scal + (size_t)env * DS_N;
  int* I = de.ints + (size_t)env * DI_N;
  dancing_obs(m, e, ids, S, I, de.moves + (size_t)env * MGX_DANCE_SEQ, obs + (size_t)env * MGX_DANCE_OBS);
  if (l >= 6 && l < m.nv) de.prev_jvel[(size_t)env * (m.nv - 6) + (l - 6)] = (double)e.qvel[l];
  if (l < 3) S[DS_TORSO + l] = (double)e.xpos[3 * ids.torso + l];
  wsync();
}

}  // namespace mgx
