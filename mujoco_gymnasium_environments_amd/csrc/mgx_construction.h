// mgx_construction.h — humanoid_construction_env task logic fused around the wide physics step.
//
// Restates, per env and on the GPU, the reference's Python around mj_step:
//   step():       humanoid_construction_env/construction_env.py:586-623 (clip :589, ctrl = action
//                 :592, one RK4 mj_step :595, current_step += 1 :598)
//   progress:     :702-719          reward: :661-700 (np.float32 from the energy term on, C2)
//   termination:  :721-737 (fall, task complete -> tasks_completed += 1, safety), truncation :608
//   observation:  :625-659 (135 floats while observation_space declares 125, C1)
//   reset:        :547-584 (mj_resetData, task then wind / rain / temperature draws, no forward
//                 pass and no settle steps, C4)
// Pinned bit for bit against the reference's own step() / reset() outputs
// (tests/golden/construction_*.npz, oracle/construction_logic.py). xpos is the last RK4 stage's
// kinematics, as MuJoCo leaves it in mjData after mj_step.
#pragma once
#include "../../include/mgx.h"
#include "mgx_soccer.h"
#include "mgx_wide.h"

namespace mgx {

enum { CS_PROGRESS = 0, CS_WIND = 1, CS_RAIN = 2, CS_TEMP = 3, CS_N = 4 };
enum { CI_TASK = 0, CI_STEP = 1, CI_BLOCKS = 2, CI_VIOL = 3, CI_DONE = 4, CI_N = 5 };

struct ConstructionIds {
  int humanoid, n_act, max_episode_steps;
  float action_limit;
};

// numpy add.reduce of |clip(a, -lim, lim)| over n contiguous values in the action's dtype (float32
// or float64; pairwise: 8 accumulators over the first 8*floor(n/8), tree (01)(23) / (45)(67), then
// the tail)
template <typename A>
__device__ __forceinline__ A np_sum_abs(const A* a, int n, A lim) {
#pragma clang fp contract(off)
  auto v = [&](int u) {
    A x = a[u];
    x = x < -lim ? -lim : (x > lim ? lim : x);
    return x < (A)0 ? -x : x;
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

// clip (against the float32 action_space bounds, in the action's dtype) -> ctrl (:589-592)
template <typename T>
__device__ __forceinline__ void construction_pre(const DevModel<T>& m, Env<T>& e, const ConstructionIds& ids, ActRow act) {
  const int l = lane_id();
  if (l < ids.n_act) {
    if (act.f64) {
      double a = act.d()[l];
      const double lim = (double)ids.action_limit;
      a = a < -lim ? -lim : (a > lim ? lim : a);
      e.ctrl[l] = (T)a;
    } else {
      float a = act.f()[l];
      const float lim = ids.action_limit;
      a = a < -lim ? -lim : (a > lim ? lim : a);
      e.ctrl[l] = (T)a;
    }
  }
  wsync();
}

// _get_observation (:625-659)
template <typename T>
__device__ __forceinline__ void construction_obs(const DevModel<T>& m, const Env<T>& e, const double* S, const int* I,
                                                 float* obs) {
  const int l = lane_id();
  for (int i = l; i < MGX_CONSTRUCTION_OBS; i += 64) {
    float v = 0.0f;
    if (i < 30) v = (float)(double)e.qpos[i];
    else if (i < 60) v = (float)(double)e.qvel[i - 30];
    else if (i >= 90 && i < 94) v = i - 90 == I[CI_TASK] ? 1.0f : 0.0f;
    else if (i == 94) v = (float)S[CS_PROGRESS];
    else if (i == 100) v = (float)(S[CS_WIND] / 10.0);
    else if (i == 101) v = (float)S[CS_RAIN];
    else if (i == 102) v = (float)(S[CS_TEMP] / 50.0);
    else if (i == 110) v = 1.0f;  // hard_hat_on never changes
    else if (i == 111) v = (float)((double)I[CI_VIOL] / 10.0);
    else if (i == 115) v = (float)((double)I[CI_BLOCKS] / 20.0);
    obs[i] = v;
  }
}

// after mj_step: counter, progress, reward, flags, observation, total reward (:598-620). Returns
// terminated || truncated (uniform).
template <typename T>
__device__ __forceinline__ bool construction_post(const DevModel<T>& m, const Env<T>& e, const ConstructionIds& ids,
                                                  ActRow act, mgx_construction_env ce, int env, float* obs,
                                                  double* reward, uint8_t* terminated, uint8_t* truncated) {
  const int l = lane_id();
  double* S = ce.scal + (size_t)env * CS_N;
  int* I = ce.ints + (size_t)env * CI_N;
  bool term = false, trunc = false;
  if (l == 0) {
#pragma clang fp contract(off)
    const int step = I[CI_STEP] + 1;
    I[CI_STEP] = step;
    const int task = I[CI_TASK];
    // _update_task_progress (:702-719): min(1.0, int / int)
    double prog = S[CS_PROGRESS];
    if (task == 0) prog = fmin(1.0, (double)I[CI_BLOCKS] / 5.0);
    else if (task == 1) prog = fmin(1.0, (double)step / 500.0);
    else if (task == 2) prog = fmin(1.0, (double)step / 300.0);
    else prog = fmin(1.0, (double)I[CI_BLOCKS] / 10.0);
    S[CS_PROGRESS] = prog;
    // _calculate_reward (:661-700): Python floats until the energy term makes it np.float32
    double r = 0.0;
    if (task == 0) r += prog * 500.0;
    else if (task == 1) r += 200.0 * 0.1;
    else if (task == 2) r += 300.0 * 0.1;
    else r += prog * 100.0;
    r += 100.0 * 0.01;                       // hard_hat_on
    r -= (double)(I[CI_VIOL] * 100);
    const double hz = (double)e.xpos[3 * ids.humanoid + 2];
    double rv;
    if (act.f64) {  // a float64 action: np.float64 energy term, the reward float64 from there on
      r += -0.2 * np_sum_abs(act.d(), ids.n_act, (double)ids.action_limit);
      if (hz > 1.0) r += 5.0;
      else r += -2000.0;
      rv = r;
    } else {
      const float energy = -0.2f * np_sum_abs(act.f(), ids.n_act, ids.action_limit);
      float r32 = (float)r + energy;
      if (hz > 1.0) r32 += 5.0f;               // stability_reward * 0.1
      else r32 += -2000.0f;                    // fall_penalty
      rv = (double)r32;
    }
    reward[env] = rv;
    // _check_terminated (:721-737)
    if (hz < 0.5) term = true;
    else if (prog >= 1.0) { I[CI_DONE] += 1; term = true; }
    else term = I[CI_VIOL] > 3;
    trunc = step >= ids.max_episode_steps;
    terminated[env] = term;
    truncated[env] = trunc;
    // episode_stats['total_reward'] += reward: float32 while both are float32 (0.0 after reset is a
    // Python float), float64 from the first float64 reward on (total_kind, as bipedal's energy)
    int kind = ce.total_kind ? ce.total_kind[env] : 2;
    if (act.f64 || kind == 1) {
      ce.total_reward[env] = ce.total_reward[env] + rv;
      kind = 1;
    } else {
      ce.total_reward[env] = (double)((float)ce.total_reward[env] + (float)rv);
      kind = 2;
    }
    if (ce.total_kind) ce.total_kind[env] = (uint8_t)kind;
  }
  wsync();
  construction_obs(m, e, S, I, obs + (size_t)env * MGX_CONSTRUCTION_OBS);
  const bool done = __builtin_amdgcn_readfirstlane((int)(term || trunc)) != 0;
  wsync();
  return done;
}

// Reset draws for the vector env: Philox4x32-10 keyed by (seed, global env index), counter =
// (episode, word): the task index (np_random.choice over 4 tasks), uniform(0, 5), uniform(0, 0.5),
// uniform(15, 35) of construction_env.py:560, :574-576
template <typename T>
__device__ __forceinline__ void construction_philox_draws(uint64_t seed, uint32_t genv, uint32_t episode, T* out) {
  const int j = lane_id();
  if (j < 4) {
    uint32_t c[4] = {episode, (uint32_t)j, 0xC0757Cu, 0u};
    philox4x32(c, (uint32_t)seed ^ genv, (uint32_t)(seed >> 32));
    double u = ((double)(c[0] >> 5) * 67108864.0 + (double)(c[1] >> 6)) * (1.0 / 9007199254740992.0);
    double v;
    if (j == 0) { v = floor(4.0 * u); v = v > 3.0 ? 3.0 : v; }
    else if (j == 1) v = 5.0 * u;
    else if (j == 2) v = 0.5 * u;
    else v = 15.0 + 20.0 * u;
    out[j] = (T)v;
  }
}

// reset() (:547-584): mj_resetData, counters, the draws, observation of qpos0 / zero qvel
template <typename T>
__device__ __forceinline__ void construction_reset_body(const DevModel<T>& m, WEnv<T>& w, const T* draws,
                                                        mgx_construction_env ce, int env, float* obs) {
  const int l = lane_id();
  wreset_env(m, w);
  double* S = ce.scal + (size_t)env * CS_N;
  int* I = ce.ints + (size_t)env * CI_N;
  if (l == 0) {
    I[CI_TASK] = (int)(double)draws[0];
    I[CI_STEP] = 0; I[CI_BLOCKS] = 0; I[CI_VIOL] = 0; I[CI_DONE] = 0;
    S[CS_PROGRESS] = 0.0;
    S[CS_WIND] = (double)draws[1]; S[CS_RAIN] = (double)draws[2]; S[CS_TEMP] = (double)draws[3];
    ce.total_reward[env] = 0.0;
    if (ce.total_kind) ce.total_kind[env] = 0;
  }
  wsync();
  construction_obs(m, w.e, S, I, obs + (size_t)env * MGX_CONSTRUCTION_OBS);
  wsync();
}

}  // namespace mgx
