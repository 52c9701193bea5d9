// mgx_rk_staged.hip — the staged RK4 step of bipedal_rescue (BASELINE configs[3]).
//
// The monolithic bipedal kernel runs one RK4 mj_step per wave: four forward passes, each with
// its own 50-sweep PGS over ~150 rows (rescue_env.py:148 RK4, :146 PGS) — 71% of the env step is
// that serial solve, and the fp64 working set (118 KB of LDS) holds one env per CU. Here each RK4
// stage k = 0..3 is the staged soccer pipeline's three kernels over the same workspace layout:
//
//   R(k)  k_rk_rows    wave per slot: stage state -> forward up to the constraint rows
//                      (stage_rows: B rows, row scalars, carry -> pipe)
//   S(k)  k_pgs_groups the lane-group PGS (16 lanes per slot, four slots per wave; 16-word block
//                      table for nv 57..64), slots over the main launch's LDS rows beside it
//   F(k)  k_rk_finish  wave per env: qacc of the stage; k = 0 checkAcc; k < 3 the next stage's
//                      state X[k+1] = X[0] '+' h sum_j A[k][j] X'[j]; k = 3 mj_advance with
//                      sum_j B_j X'[j], then the task logic (rescue_env.py:435-467) and autoreset
//
// The arithmetic per stage is mj_RungeKutta's (mgx_physics.h rk4: same coefficient sums in the
// same order; the frames the task logic reads are the last stage's, as MuJoCo leaves them).
// Reset banks: each env keeps R post-settle reset states ahead (Philox draws keyed by (seed,
// global env, episode)); a bank advances one RK4 step per env step as an extra slot of the same
// launches. reset() and a reset whose bank is not ready run k_rk_settle: the same stages, in one
// wave, through the same device code and flags (one translation unit), so a reset has one
// arithmetic whatever the bank count.
#include <map>
#include <mutex>

#include "mgx_internal.h"

using namespace mgx;

MGX_PROF_SETTER(mgx_prof_set_buffer_rk_staged)

namespace mgx {

constexpr int RK_NCS = 3;   // contact-metadata lane sets of the row builder: up to 192 contacts
// B in the dof-granular layout (mgx_staged.h DOFB): this pipeline streams B from HBM every sweep
constexpr int RK_LPS = 16;  // solver lanes per slot
constexpr int RK_EPL = 4;   // solver register entries per lane (nv 49..64)
constexpr int RK_OBS = 102; // rescue_env.py:545-600
enum { RK_IDLE = 0, RK_ACTIVE = 1 };
enum { RK_SETTLE_RESET = 0, RK_SETTLE_FIXUP = 1 };

// per-slot RK4 carry (P.o_rk): X[0] positions, the next stage's positions, v[4][64], f[4][64], t0
template <typename T>
struct RkCarry {
  T *q0, *x, *v, *f, *t;
};
template <typename T>
__device__ __forceinline__ RkCarry<T> rk_carry(const DevModel<T>& m, const Pipe& P, int slot) {
  T* b = P.at<T>(P.o_rk) + (size_t)slot * P.rk_stride;
  const int nq4 = (m.nq + 3) & ~3;
  RkCarry<T> r;
  r.q0 = b;
  r.x = b + nq4;
  r.v = b + 2 * nq4;
  r.f = r.v + 4 * 64;
  r.t = r.f + 4 * 64;
  return r;
}

// ---------------------------------------------------------------- banks (bipedal)
// record bi restarts for `episode` from 12 draws in LDS (rescue_env.py:473-508 after mj_resetData;
// the task's tracking reset is applied when the bank is installed)
template <typename T>
__device__ __forceinline__ void rk_bank_init_draws(const DevModel<T>& m, Env<T>& e, const BipedalIds& ids, const Pipe& P,
                                                   int bi, int episode, uint64_t seed, const T* draws) {
  int l = lane_id();
  T d[12];
  for (int j = 0; j < 12; j++) d[j] = draws[j];
  wsync();
  reset_env(m, e);
  if (l == 0) {
    e.qpos[ids.root_x] = d[0];
    e.qpos[ids.root_y] = d[1];
    e.qpos[ids.root_z] = (T)1.2;
    for (int i = 0; i < 5; i++) {
      e.qpos[ids.victim_x[i]] = e.qpos[ids.victim_x[i]] + d[2 + 2 * i];
      e.qpos[ids.victim_y[i]] = e.qpos[ids.victim_y[i]] + d[3 + 2 * i];
    }
  }
  wsync();
  copy_g(P.at<T>(P.o_bq) + (size_t)bi * m.nq, e.qpos, m.nq);
  if (l < m.nv) {
    P.at<T>(P.o_bv)[(size_t)bi * m.nv + l] = 0;
    P.at<T>(P.o_ba)[(size_t)bi * m.nv + l] = 0;
  }
  if (l == 0) {
    P.at<T>(P.o_btime)[bi] = 0;
    P.at<int>(P.o_bwarn)[bi] = 0;
    P.at<int>(P.o_bep)[bi] = episode;
    P.at<uint64_t>(P.o_bseed)[bi] = seed;
    P.at<int>(P.o_bk)[bi] = 0;
  }
  wsync();
}
template <typename T>
__device__ __forceinline__ void rk_bank_init(const DevModel<T>& m, Env<T>& e, const BipedalIds& ids, const Pipe& P,
                                             int env, int bi, int episode, uint64_t seed, int env_offset) {
  bipedal_philox_draws(seed, (uint32_t)(env_offset + env), (uint32_t)episode, e.vec3);
  wsync();
  rk_bank_init_draws(m, e, ids, P, bi, episode, seed, e.vec3);
}

// settle finished: the reset observation and prev_robot_pos (rescue_env.py:393-396)
template <typename T>
__device__ __forceinline__ void rk_bank_finalize(const DevModel<T>& m, Env<T>& e, const BipedalIds& ids, const Pipe& P,
                                                 int bi) {
  bipedal_obs(m, e, ids, 0, 0, 0, 1000.0, false, P.at<float>(P.o_bobs) + (size_t)bi * RK_OBS);
  int l = lane_id();
  if (l < 3) P.at<T>(P.o_bprev)[(size_t)bi * 6 + l] = e.xpos[3 * ids.torso + l];
  wsync();
}

// the settled reset of record bi becomes env's live state for episode E: state, the tracking
// reset of rescue_env.py:347-372 (the _prev_* / _fall_timer attributes survive, quirk B3), obs,
// prev_robot_pos; episode E + 1
template <typename T>
__device__ __forceinline__ void rk_bank_copy_live(const DevModel<T>& m, const Pipe& P, mgx_state s, mgx_bipedal_env be,
                                                  float* obs, int env, int bi, int E) {
  int l = lane_id();
  copy_g((T*)s.qpos + (size_t)env * m.nq, P.at<T>(P.o_bq) + (size_t)bi * m.nq, m.nq);
  copy_g((T*)s.qvel + (size_t)env * m.nv, P.at<T>(P.o_bv) + (size_t)bi * m.nv, m.nv);
  copy_g((T*)s.qacc_warmstart + (size_t)env * m.nv, P.at<T>(P.o_ba) + (size_t)bi * m.nv, m.nv);
  for (int k = l; k < m.nv; k += 64) ((T*)s.qfrc_applied)[(size_t)env * m.nv + k] = 0;
  for (int k = l; k < m.nu; k += 64) ((T*)s.ctrl)[(size_t)env * m.nu + k] = 0;
  for (int k = l; k < 6 * m.nbody; k += 64) ((T*)s.xfrc_applied)[(size_t)env * 6 * m.nbody + k] = 0;
  copy_g(obs + (size_t)env * RK_OBS, P.at<float>(P.o_bobs) + (size_t)bi * RK_OBS, RK_OBS);
  if (l < 3) be.prev_robot_pos[3 * (size_t)env + l] = (double)P.at<T>(P.o_bprev)[(size_t)bi * 6 + l];
  if (l == 0) {
    ((T*)s.time)[env] = P.at<T>(P.o_btime)[bi];
    if (s.warning) s.warning[env] += P.at<int>(P.o_bwarn)[bi];
    be.step[env] = 0;
    be.energy[env] = 1000.0;
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
    if (be.episode) be.episode[env] = E + 1;
  }
  wsync();
}

// ---------------------------------------------------------------- stage pieces
// R(k) body: the slot's stage state into the row builder's Env, then forward up to the rows.
// Live env (bi < 0): stage 0 reads the env's state and runs the pre-step logic; bank record bi:
// stage 0 reads the record (mj_resetData'd data: zero controls and applied forces). Stages 1..3
// read X[k] from the RK carry; controls / applied forces / warmstart from the live state (the
// stage-0 row builder wrote the step's controls there) or zeros / the record's warmstart.
template <typename T>
__device__ __forceinline__ void rk_rows_slot(const DevModel<T>& m, Env<T>& e, const BipedalIds& ids, mgx_state s,
                                             mgx_bipedal_env be, const float* action, const Pipe& P, int env, int bi,
                                             int slot, int stage, bool list_slot) {
  const int l = lane_id();
  int warn = 0;
  if (stage == 0) {
    if (bi < 0) {
      load_state(m, e, (T*)s.qpos, (T*)s.qvel, (T*)s.qacc_warmstart, (T*)s.ctrl, (T*)s.qfrc_applied,
                 (T*)s.xfrc_applied, (T*)s.time, env);
      bipedal_pre(m, e, ids, ActRow(action, be.action_f64, env, ids.n_act), be, env);
    } else {
      bank_load_state(m, e, P, bi);
    }
    if (any_bad(e.qpos, m.nq)) { reset_env(m, e); warn++; }  // mj_checkPos
    if (any_bad(e.qvel, m.nv)) { reset_env(m, e); warn++; }  // mj_checkVel
    if (bi < 0) {
      // the step's controls and applied forces (a bad-state reset zeroes them) for stages 1..3
      for (int k = l; k < m.nu; k += 64) ((T*)s.ctrl)[(size_t)env * m.nu + k] = e.ctrl[k];
      if (warn) {
        for (int k = l; k < m.nv; k += 64) ((T*)s.qfrc_applied)[(size_t)env * m.nv + k] = 0;
        for (int k = l; k < 6 * m.nbody; k += 64) ((T*)s.xfrc_applied)[(size_t)env * 6 * m.nbody + k] = 0;
      }
    }
    if (l == 0) P.at<int>(P.o_rks)[slot] = RK_ACTIVE;
  } else {
    const RkCarry<T> rk = rk_carry(m, P, slot);
    for (int k = l; k < m.nq; k += 64) e.qpos[k] = rk.x[k];
    for (int k = l; k < m.nv; k += 64) e.qvel[k] = rk.v[64 * stage + k];
    if (bi < 0) {
      for (int k = l; k < m.nu; k += 64) e.ctrl[k] = ((const T*)s.ctrl)[(size_t)env * m.nu + k];
      for (int k = l; k < 6 * m.nbody; k += 64) e.xfrc[k] = ((const T*)s.xfrc_applied)[(size_t)env * 6 * m.nbody + k];
      e.qfrc_applied = l < m.nv ? ((const T*)s.qfrc_applied)[(size_t)env * m.nv + l] : (T)0;
      e.qacc_ws = l < m.nv ? ((const T*)s.qacc_warmstart)[(size_t)env * m.nv + l] : (T)0;
    } else {
      for (int k = l; k < m.nu; k += 64) e.ctrl[k] = 0;
      for (int k = l; k < 6 * m.nbody; k += 64) e.xfrc[k] = 0;
      e.qfrc_applied = 0;
      e.qacc_ws = l < m.nv ? P.at<T>(P.o_ba)[(size_t)bi * m.nv + l] : (T)0;
    }
    e.time = rk.t[1];
    wsync();
  }
  stage_rows<T, RK_NCS, true>(m, e, P, slot, warn, list_slot);
}

// qacc of the stage from the solver's v (finish_physics' first half): qacc_smooth + L^-1 D^-1/2 v
template <typename T>
__device__ __forceinline__ T rk_stage_qacc(const DevModel<T>& m, Env<T>& e, const Pipe& P, int slot) {
  const int l = lane_id();
  const bool dl = l < m.nv;
  if (e.nefc > 0) {
    T v = dl ? P.at<T>(P.o_vout)[(size_t)slot * 64 + l] : (T)0;
    T D = dl ? e.qLD[m.dof_Madr[l]] : (T)1;
    T sqrtD = sqrt(D);
    T z = dl ? v / sqrtD : (T)0;
    z = solve_L(m, e, e.qLD, z);
    return e.qacc_smooth + z;
  }
  return e.qacc_smooth;
}

// end of the env step for the slot (state in f: post-integration qpos / qvel, the last stage's
// frames and contacts). Live env: state out, task logic, rollout sums, same-step autoreset (a
// ready bank, else the fixup list). Bank record: store, and finalize after the 10th settle step.
template <typename T>
__device__ __forceinline__ void rk_step_end(const DevModel<T>& m, Env<T>& f, const BipedalIds& ids, mgx_state s,
                                            mgx_bipedal_env be, const float* action, float* obs, double* reward,
                                            uint8_t* terminated, uint8_t* truncated, float* final_obs, int autoreset,
                                            uint64_t seed, int env_offset, const Pipe& P, int env, int bi, int warn,
                                            bool overflow) {
  const int l = lane_id();
  if (bi >= 0) {
    bank_store_state(m, f, P, bi, warn);
    wsync();
    const int k = P.at<int>(P.o_bk)[bi] + 1;
    if (k == 10) rk_bank_finalize(m, f, ids, P, bi);
    if (l == 0) P.at<int>(P.o_bk)[bi] = k;
    wsync();
    return;
  }
  store_state(m, f, (T*)s.qpos, (T*)s.qvel, (T*)s.qacc_warmstart, (T*)s.ctrl, (T*)s.qfrc_applied, (T*)s.xfrc_applied,
              (T*)s.time, env);
  if (l == 0 && s.warning) s.warning[env] += warn;
  if (l == 0 && s.overflow && overflow) s.overflow[env] += 1;
  const bool done =
      bipedal_post(m, f, ids, ActRow(action, be.action_f64, env, ids.n_act), be, env, obs, reward, terminated, truncated);
  if (be.rollout && l == 0) {
    T* ro = (T*)be.rollout + 4 * (size_t)env;
    ro[0] += (T)reward[env];
    ro[1] += (T)terminated[env];
    ro[2] += (T)truncated[env];
    ro[3] += (T)1;
  }
  if (!(done && autoreset)) return;
  if (final_obs)
    for (int i = l; i < RK_OBS; i += 64) final_obs[(size_t)env * RK_OBS + i] = obs[(size_t)env * RK_OBS + i];
  __threadfence();
  wsync();
  const int E = be.episode[env];
  bool ready = false;
  int bi2 = 0;
  if (P.R > 0) {
    bi2 = env * P.R + E % P.R;
    ready = P.at<int>(P.o_bk)[bi2] == 10 && P.at<int>(P.o_bep)[bi2] == E && P.at<uint64_t>(P.o_bseed)[bi2] == seed;
  }
  if (ready) {
    rk_bank_copy_live(m, P, s, be, obs, env, bi2, E);
    rk_bank_init(m, f, ids, P, env, bi2, E + P.R, seed, env_offset);
  } else if (l == 0) {
    P.at<int>(P.o_fix)[atomicAdd(P.ctr() + 5, 1)] = env;
  }
}

// F(k) body for one active slot (Env f: the finisher layout). Returns true when the slot's
// env step ended (stage 3, or a bad stage-0 qacc: mj_checkAcc -> the template).
template <typename T>
__device__ __forceinline__ bool rk_finish_slot(const DevModel<T>& m, Env<T>& f, const BipedalIds& ids, mgx_state s,
                                               mgx_bipedal_env be, const float* action, float* obs, double* reward,
                                               uint8_t* terminated, uint8_t* truncated, float* final_obs, int autoreset,
                                               uint64_t seed, int env_offset, const Pipe& P, int env, int bi, int slot,
                                               int stage) {
  const T A[9] = {(T)0.5, 0, 0, 0, (T)0.5, 0, 0, 0, (T)1};
  const T Bc[4] = {(T)(1.0 / 6.0), (T)(1.0 / 3.0), (T)(1.0 / 3.0), (T)(1.0 / 6.0)};
  const int l = lane_id();
  const bool dl = l < m.nv;
  const T h = m.timestep;
  int warn = load_carry(m, f, P, slot);
  const T qacc = rk_stage_qacc(m, f, P, slot);
  const RkCarry<T> rk = rk_carry(m, P, slot);
  int* rkw = P.at<int>(P.o_rkw) + slot;
  if (stage == 0) {
    if (ballot(dl && isbad(qacc)) != 0ull) {
      // mj_checkAcc: mj_resetData, forward, RK4 from the reset data — env-independent, computed
      // once per workspace (k_rk_template)
      load_template(m, f, P);
      warn++;
      rk_step_end(m, f, ids, s, be, action, obs, reward, terminated, truncated, final_obs, autoreset, seed, env_offset,
                  P, env, bi, warn, f.overflow != 0);
      if (l == 0) P.at<int>(P.o_rks)[slot] = RK_IDLE;
      return true;
    }
    for (int k = l; k < m.nq; k += 64) rk.q0[k] = f.qpos[k];
    if (dl) rk.v[l] = f.qvel[l];
    if (l == 0) {
      rk.t[0] = f.time;
      *rkw = warn + (f.overflow ? (1 << 20) : 0);
    }
  } else if (l == 0 && f.overflow) {
    *rkw |= 1 << 20;
  }
  if (dl) rk.f[64 * stage + l] = qacc;
  __threadfence();
  wsync();
  // v[j], f[j] of the earlier stages (this stage's: the carry's qvel and qacc)
  T v[4], a[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    v[j] = (dl && j < stage) ? rk.v[64 * j + l] : (T)0;
    a[j] = (dl && j < stage) ? rk.f[64 * j + l] : (T)0;
  }
  if (stage == 0) v[0] = dl ? f.qvel[l] : (T)0;
  else if (stage == 1) v[1] = dl ? f.qvel[l] : (T)0;
  else if (stage == 2) v[2] = dl ? f.qvel[l] : (T)0;
  else v[3] = dl ? f.qvel[l] : (T)0;
  if (stage == 0) a[0] = dl ? qacc : (T)0;
  else if (stage == 1) a[1] = dl ? qacc : (T)0;
  else if (stage == 2) a[2] = dl ? qacc : (T)0;
  else a[3] = dl ? qacc : (T)0;
  const T t0 = rk.t[0];
  T* dxv = f.vec3;
  if (stage < 3) {
    // X[i], i = stage + 1 (mgx_physics.h rk4: the same sums in the same order)
    const int i = stage + 1;
    T C = 0, dv = 0, da = 0;
    for (int j = 0; j < i; j++) {
      T c = A[(i - 1) * 3 + j];
      C += c;
      dv += c * v[j];
      da += c * a[j];
    }
    wsync();
    if (dl) dxv[l] = dv;
    for (int k = l; k < m.nq; k += 64) f.qpos[k] = rk.q0[k];
    wsync();
    integrate_pos(m, f.qpos, dxv, h);
    const T vi = v[0] + h * da;
    for (int k = l; k < m.nq; k += 64) rk.x[k] = f.qpos[k];
    if (dl) rk.v[64 * i + l] = vi;
    if (l == 0) rk.t[1] = t0 + C * h;
    __threadfence();
    wsync();
    return false;
  }
  // mj_advance with dX = sum_j B_j X'[j]; qacc_warmstart = the last evaluation's qacc
  T dv = 0, da = 0;
  for (int j = 0; j < 4; j++) { dv += Bc[j] * v[j]; da += Bc[j] * a[j]; }
  f.qacc_ws = qacc;
  wsync();
  for (int k = l; k < m.nq; k += 64) f.qpos[k] = rk.q0[k];
  if (dl) { dxv[l] = dv; f.qvel[l] = v[0] + h * da; }
  wsync();
  integrate_pos(m, f.qpos, dxv, h);
  f.time = t0 + h;
  const int w = *rkw;
  wsync();
  rk_step_end(m, f, ids, s, be, action, obs, reward, terminated, truncated, final_obs, autoreset, seed, env_offset, P,
              env, bi, w & ((1 << 20) - 1), (w >> 20) != 0);
  if (l == 0) P.at<int>(P.o_rks)[slot] = RK_IDLE;
  return true;
}

// ---------------------------------------------------------------- kernels
template <typename T>
__global__ void __launch_bounds__(64) k_rk_rows(DevModel<T> m, BipedalIds ids, mgx_state s, mgx_bipedal_env be,
                                                const float* action, int n_env, const uint8_t* mask, Pipe P, int banks,
                                                int stage) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x;
  if (stage == 0 && b == 0 && threadIdx.x == 0) P.ctr()[5] = 0;  // this step's fixup list
  int bi = -1;
  if (b < n_env) {
    if (mask && !mask[b]) return;
  } else {
    bi = b - n_env;
    if (!banks || bi >= n_env * P.R) return;
    if (stage == 0) {
      const int k = P.at<int>(P.o_bk)[bi];
      if (k < 0 || k >= 10) return;
    }
  }
  if (stage > 0 && P.at<int>(P.o_rks)[b] != RK_ACTIVE) return;
  Env<T> e;
  env_bind(m, e, smem);
  bind_carry_tail(m, e, P, b);
  rk_rows_slot(m, e, ids, s, be, action, P, b < n_env ? b : 0, bi, b, stage, true);
}

template <typename T>
__global__ void __launch_bounds__(64) k_rk_finish(DevModel<T> m, BipedalIds ids, mgx_state s, mgx_bipedal_env be,
                                                  const float* action, float* obs, double* reward, uint8_t* terminated,
                                                  uint8_t* truncated, float* final_obs, int autoreset, uint64_t seed,
                                                  int env_offset, int n_env, const uint8_t* mask, Pipe P, int banks,
                                                  int stage, int bank_part) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int* rks = P.at<int>(P.o_rks);
  if (bank_part) {
    // the bank records' stage (one wave per record), launched before the live part: a record
    // finishing its tenth settle step here is ready for this step's resets
    const int bi = blockIdx.x;
    if (bi >= n_env * P.R) return;
    const int slot = n_env + bi;
    if (rks[slot] != RK_ACTIVE) return;
    Env<T> f;
    env_bind(m, f, smem);
    rk_finish_slot(m, f, ids, s, be, action, obs, reward, terminated, truncated, final_obs, autoreset, seed, env_offset,
                   P, bi / P.R, bi, slot, stage);
    return;
  }
  const int env = blockIdx.x;
  if (env >= n_env) return;
  if (env == 0 && lane_id() == 0) {  // this stage's solver lists are consumed
    P.ctr()[3] = P.ctr()[1];
    P.ctr()[4] = P.ctr()[2];
    P.ctr()[1] = 0;
    P.ctr()[2] = 0;
  }
  if (env == 0)
    for (int b = lane_id(); b < P.nbk; b += 64) P.at<int>(P.o_hist)[b] = 0;
  Env<T> f;
  env_bind(m, f, smem);
  if (mask && !mask[env]) return;
  if (rks[env] != RK_ACTIVE) return;
  rk_finish_slot(m, f, ids, s, be, action, obs, reward, terminated, truncated, final_obs, autoreset, seed, env_offset, P,
                 env, -1, env, stage);
}

// One RK4 settle step of record bi in one wave, through pipe slot `slot`: the pipeline's stages
// in sequence (rk_rows_slot, the PGS of the one slot, rk_finish_slot).
template <typename T>
__device__ __forceinline__ void rk_settle_step(const DevModel<T>& Ms, const DevModel<T>& Mf, const BipedalIds& ids,
                                               mgx_state s, mgx_bipedal_env be, const Pipe& P, char* smem,
                                               int env, int bi, int slot, int maxit, T tol, T scale) {
  for (int stage = 0; stage < 4; stage++) {
    {
      Env<T> e;
      env_bind(Ms, e, smem);
      bind_carry_tail(Ms, e, P, slot);
      rk_rows_slot(Ms, e, ids, s, be, nullptr, P, env, bi, slot, stage, false);
    }
    __threadfence();
    __syncthreads();
    pgs_group<T, RK_EPL, RK_LPS, false, true, true>(P, smem, threadIdx.x < RK_LPS ? slot : -1, P.maxE, maxit, tol, scale,
                                               64 / RK_LPS);
    __threadfence();
    __syncthreads();
    Env<T> f;
    env_bind(Mf, f, smem);
    const bool end = rk_finish_slot(Mf, f, ids, s, be, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, 0, P,
                                    env, bi, slot, stage);
    __threadfence();
    __syncthreads();
    if (end) break;
  }
}

// Restart record bi for `episode` (host draws [12] or Philox) and settle it: 10 RK4 mj_steps
// (rescue_env.py:390-391); the record ends finalized with bk = 10.
template <typename T>
__device__ __forceinline__ void rk_settle_reset(const DevModel<T>& Ms, const DevModel<T>& Mf, const BipedalIds& ids,
                                                mgx_state s, mgx_bipedal_env be, const Pipe& P, char* smem,
                                                int env, int bi, int episode, const T* draws, uint64_t seed,
                                                int env_offset, int maxit, T tol, T scale) {
  {
    Env<T> e;
    env_bind(Ms, e, smem);
    bind_carry_tail(Ms, e, P, env);
    if (draws) {
      if (lane_id() < 12) e.vec3[lane_id()] = draws[lane_id()];
    } else {
      bipedal_philox_draws(seed, (uint32_t)(env_offset + env), (uint32_t)episode, e.vec3);
    }
    wsync();
    rk_bank_init_draws(Ms, e, ids, P, bi, episode, seed, e.vec3);
  }
  __threadfence();
  __syncthreads();
  for (int t = 0; t < 10; t++) rk_settle_step(Ms, Mf, ids, s, be, P, smem, env, bi, env, maxit, tol, scale);
}

// reset() of a staged batch (RK_SETTLE_RESET, one workgroup per env; with Philox draws and banks
// it also prefills the env's R banks) and the step's resets whose bank was not ready
// (RK_SETTLE_FIXUP, grid-stride over the finisher's list).
template <typename T>
__global__ void __launch_bounds__(64) k_rk_settle(DevModel<T> Ms, DevModel<T> Mf, BipedalIds ids, mgx_state s,
                                                  mgx_bipedal_env be, const T* draws, float* obs, uint64_t seed,
                                                  int env_offset, int n_env, const uint8_t* mask, Pipe P, int mode,
                                                  int maxit, T tol, T scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int cnt = mode == RK_SETTLE_FIXUP ? P.ctr()[5] : n_env;
  for (int i = blockIdx.x; i < cnt; i += gridDim.x) {
    const int env = mode == RK_SETTLE_FIXUP ? P.at<int>(P.o_fix)[i] : i;
    if (mode == RK_SETTLE_RESET && mask && !mask[env]) continue;
    const int E = be.episode ? be.episode[env] : 0;
    const int bi = P.R > 0 ? env * P.R + E % P.R : env;
    const T* d = draws ? draws + (size_t)env * 12 : nullptr;
    rk_settle_reset(Ms, Mf, ids, s, be, P, smem, env, bi, E, d, seed, env_offset, maxit, tol, scale);
    rk_bank_copy_live(Mf, P, s, be, obs, env, bi, E);
    if (P.R > 0 && mode == RK_SETTLE_FIXUP) {
      Env<T> e;
      env_bind(Ms, e, smem);
      bind_carry_tail(Ms, e, P, env);
      rk_bank_init(Ms, e, ids, P, env, bi, E + P.R, seed, env_offset);
    } else if (P.R > 0 && !draws) {
      for (int k = 1; k <= P.R; k++)
        rk_settle_reset(Ms, Mf, ids, s, be, P, smem, env, env * P.R + (E + k) % P.R, E + k, (const T*)nullptr, seed,
                        env_offset, maxit, tol, scale);
    } else if (lane_id() == 0) {
      P.at<int>(P.o_bk)[bi] = -1;  // a scratch record: nothing to settle
    }
    __threadfence();
    __syncthreads();
  }
}

// mj_checkAcc's outcome: mj_resetData, mj_forward, RK4 (monolithic layout, rows in the pipe's
// template scratch), into the template arrays load_template reads
template <typename T, bool GB>
__global__ void __launch_bounds__(64) k_rk_template(DevModel<T> m, Pipe P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Env<T> e;
  env_bind<T, GB>(m, e, smem, GB ? P.at<T>(P.o_tscr) : nullptr);
  const int l = lane_id();
  reset_env(m, e);
  forward<T>(m, e);
  rk4<T>(m, e);
  for (int k = l; k < m.nq; k += 64) P.at<T>(P.o_tq)[k] = e.qpos[k];
  for (int k = l; k < m.nv; k += 64) P.at<T>(P.o_tv)[k] = e.qvel[k];
  if (l < m.nv) P.at<T>(P.o_ta)[l] = e.qacc_ws;
  for (int k = l; k < 3 * m.nbody; k += 64) { P.at<T>(P.o_tx)[k] = e.xpos[k]; P.at<T>(P.o_tsc)[k] = e.subtree_com[k]; }
  for (int k = l; k < 4 * m.nbody; k += 64) P.at<T>(P.o_txq)[k] = e.xquat[k];
  const int nc = e.ncon < P.maxC ? e.ncon : P.maxC;
  for (int k = l; k < nc; k += 64) {
    P.at<int>(P.o_tcg)[2 * k] = e.con_geom[2 * k];
    P.at<int>(P.o_tcg)[2 * k + 1] = e.con_geom[2 * k + 1];
    P.at<T>(P.o_tcd)[k] = e.con_dist[k];
    P.at<T>(P.o_tcm)[k] = e.con_mu[k];
  }
  if (l == 0) { P.at<int>(P.o_tn)[0] = nc; P.at<T>(P.o_tt)[0] = e.time; }
}

}  // namespace mgx

// ------------------------------------------------------------------------- host side
namespace {

int fail(int code, const std::string& msg) { return host_fail(code, msg); }

struct RkSide {
  hipStream_t s;
  hipEvent_t rows, big;
};
RkSide* rk_side(hipStream_t st) {
  static std::mutex mu;
  static std::map<std::pair<hipStream_t, int>, RkSide*> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  auto key = std::make_pair(st, dev);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  RkSide* x = new RkSide{};
  if (hipStreamCreateWithFlags(&x->s, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&x->rows, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&x->big, hipEventDisableTiming) != hipSuccess) {
    delete x;
    x = nullptr;
  }
  cache[key] = x;
  return x;
}

int settle_lds(const mgx_model* m, const Pipe& P) {
  int b = staged_pgs_lds_bytes(m, P.maxE, RK_LPS, 1, 4);
  if (m->Ls.bytes > b) b = m->Ls.bytes;
  if (m->Lf.bytes > b) b = m->Lf.bytes;
  return b;
}

template <typename T>
void launch_rk_pgs(const Pipe& P, int slots, int lds, hipStream_t st, int maxit, T tol, T scale, int big) {
  const int spw = 64 / RK_LPS;
  const int grid = (slots + spw - 1) / spw;
  hipLaunchKernelGGL((k_pgs_groups<T, RK_EPL, RK_LPS, false, true, true>), dim3(grid), dim3(64), lds, st, P, maxit, tol, scale,
                     spw, big);
}

template <typename T>
int step_staged(const mgx_model* m, const DevModel<T>& M, const DevModel<T>& Ms, const DevModel<T>& Mf,
                const mgx_state* s, const mgx_bipedal_env* e, const float* action, float* obs, double* reward,
                uint8_t* terminated, uint8_t* truncated, float* final_obs, int autoreset, uint64_t seed, int env_offset,
                int n_env, const uint8_t* mask, hipStream_t st) {
  Pipe P;
  const int banks = autoreset ? e->banks : 0;
  const size_t need = make_staged_pipe(m, e->workspace, n_env, e->banks, &P, true, RK_OBS);
  if (e->workspace_bytes < need) return fail(MGX_E_ARG, "workspace smaller than mgx_bipedal_workspace_bytes");
  const int slots = n_env * (1 + banks);
  const T scale = (T)1 / (M.meaninertia * (T)(M.nv > 1 ? M.nv : 1));
  const int mlds = staged_pgs_lds_bytes(m, P.capE, RK_LPS, 1, 4), wlds = staged_pgs_lds_bytes(m, P.maxE, RK_LPS, 1, 4);
  const int wgrid = 64 / RK_LPS * MGX_PGS_WIDE_GRID;
  RkSide* side = m->hooks.side_stream ? rk_side(st) : nullptr;
  for (int k = 0; k < 4; k++) {
    hipLaunchKernelGGL(k_rk_rows<T>, dim3(slots), dim3(64), m->Ls.bytes, st, Ms, m->bp, *s, *e, action, n_env, mask, P,
                       banks, k);
    if (side) {
      MGX_HIPCHK(hipEventRecord(side->rows, st));
      MGX_HIPCHK(hipStreamWaitEvent(side->s, side->rows, 0));
      launch_rk_pgs<T>(P, wgrid, wlds, side->s, M.iterations, M.tolerance, scale, 1);
      MGX_HIPCHK(hipEventRecord(side->big, side->s));
      launch_rk_pgs<T>(P, slots, mlds, st, M.iterations, M.tolerance, scale, 0);
      MGX_HIPCHK(hipStreamWaitEvent(st, side->big, 0));
    } else {
      launch_rk_pgs<T>(P, slots, mlds, st, M.iterations, M.tolerance, scale, 0);
      launch_rk_pgs<T>(P, wgrid, wlds, st, M.iterations, M.tolerance, scale, 1);
    }
    if (banks && P.R > 0)
      hipLaunchKernelGGL(k_rk_finish<T>, dim3(n_env * P.R), dim3(64), m->Lf.bytes, st, Mf, m->bp, *s, *e, action, obs,
                         reward, terminated, truncated, final_obs, autoreset, seed, env_offset, n_env, mask, P, banks, k, 1);
    hipLaunchKernelGGL(k_rk_finish<T>, dim3(n_env), dim3(64), m->Lf.bytes, st, Mf, m->bp, *s, *e, action, obs, reward,
                       terminated, truncated, final_obs, autoreset, seed, env_offset, n_env, mask, P, banks, k, 0);
  }
  const int fgrid = n_env < 256 ? n_env : 256;
  hipLaunchKernelGGL(k_rk_settle<T>, dim3(fgrid), dim3(64), settle_lds(m, P), st, Ms, Mf, m->bp, *s, *e,
                     (const T*)nullptr, obs, seed, env_offset, n_env, (const uint8_t*)nullptr, P, (int)RK_SETTLE_FIXUP,
                     M.iterations, M.tolerance, scale);
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}

template <typename T>
int reset_staged(const mgx_model* m, const DevModel<T>& M, const DevModel<T>& Ms, const DevModel<T>& Mf,
                 const mgx_state* s, const mgx_bipedal_env* e, const T* draws, float* obs, uint64_t seed, int env_offset,
                 int n_env, const uint8_t* mask, hipStream_t st) {
  Pipe P;
  const size_t need = make_staged_pipe(m, e->workspace, n_env, e->banks, &P, true, RK_OBS);
  if (e->workspace_bytes < need) return fail(MGX_E_ARG, "workspace smaller than mgx_bipedal_workspace_bytes");
  const T scale = (T)1 / (M.meaninertia * (T)(M.nv > 1 ? M.nv : 1));
  hipLaunchKernelGGL(k_rk_settle<T>, dim3(n_env), dim3(64), settle_lds(m, P), st, Ms, Mf, m->bp, *s, *e, draws, obs, seed,
                     env_offset, n_env, mask, P, (int)RK_SETTLE_RESET, M.iterations, M.tolerance, scale);
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}

template <typename T>
int configure_t(const mgx_model* m) {
  Pipe P;
  make_staged_pipe(m, nullptr, 1, 1, &P, true, RK_OBS);
  const int wl = staged_pgs_lds_bytes(m, P.maxE, RK_LPS, 1, 4);
  if (wl > 160 * 1024) return fail(MGX_E_CAPACITY, "staged RK4 solver LDS exceeds 160 KiB");
  return mgx_set_lds(k_rk_rows<T>, m->Ls.bytes) | mgx_set_lds(k_rk_finish<T>, m->Lf.bytes) |
         mgx_set_lds(k_rk_settle<T>, settle_lds(m, P)) | mgx_set_lds(k_rk_template<T, true>, m->L.bytes) |
         mgx_set_lds(k_rk_template<T, false>, m->L.bytes) |
         mgx_set_lds(k_pgs_groups<T, RK_EPL, RK_LPS, false, true, true>, wl > 96 * 1024 ? wl : 96 * 1024);
}

}  // namespace

namespace mgx {
int bipedal_staged_configure(const mgx_model* m) {
  if (!m->staged_rk_ok) return MGX_OK;
  return m->precision == MGX_F32 ? configure_t<float>(m) : configure_t<double>(m);
}

int bipedal_step_staged(const mgx_model* m, const mgx_state* s, const mgx_bipedal_env* e, const float* action, float* obs,
                        double* reward, uint8_t* terminated, uint8_t* truncated, float* final_obs, int autoreset,
                        uint64_t seed, int env_offset, int n_env, const uint8_t* mask, hipStream_t st) {
  if (!m->staged_rk_ok) return fail(MGX_E_UNSUPPORTED, "staged RK4 step: model outside the staged pipeline's range");
  if (e->banks < 0 || e->banks > 16) return fail(MGX_E_ARG, "banks must be in [0, 16]");
  if (m->precision == MGX_F32)
    return step_staged<float>(m, m->mf, m->mfs, m->mff, s, e, action, obs, reward, terminated, truncated, final_obs,
                              autoreset, seed, env_offset, n_env, mask, st);
  return step_staged<double>(m, m->md, m->mds, m->mdf, s, e, action, obs, reward, terminated, truncated, final_obs,
                             autoreset, seed, env_offset, n_env, mask, st);
}

int bipedal_reset_staged(const mgx_model* m, const mgx_state* s, const mgx_bipedal_env* e, const void* draws,
                         float* obs, uint64_t seed, int env_offset, int n_env, const uint8_t* mask, hipStream_t st) {
  if (!m->staged_rk_ok) return fail(MGX_E_UNSUPPORTED, "staged RK4 step: model outside the staged pipeline's range");
  if (e->banks < 0 || e->banks > 16) return fail(MGX_E_ARG, "banks must be in [0, 16]");
  if (m->precision == MGX_F32)
    return reset_staged<float>(m, m->mf, m->mfs, m->mff, s, e, (const float*)draws, obs, seed, env_offset, n_env, mask,
                               st);
  return reset_staged<double>(m, m->md, m->mds, m->mdf, s, e, (const double*)draws, obs, seed, env_offset, n_env, mask,
                              st);
}

int64_t bipedal_workspace_bytes(const mgx_model* m, int n_env, int banks) {
  if (!m || n_env <= 0 || banks < 0 || banks > 16) return fail(MGX_E_ARG, "bad argument");
  if (!m->staged_rk_ok) return fail(MGX_E_UNSUPPORTED, "staged RK4 step: model outside the staged pipeline's range");
  return (int64_t)make_staged_pipe(m, nullptr, n_env, banks, nullptr, true, RK_OBS);
}

int bipedal_workspace_init(const mgx_model* m, void* workspace, uint64_t bytes, int n_env, int banks, hipStream_t st) {
  if (!m || !workspace || n_env <= 0 || banks < 0 || banks > 16) return fail(MGX_E_ARG, "bad argument");
  if (!m->staged_rk_ok) return fail(MGX_E_UNSUPPORTED, "staged RK4 step: model outside the staged pipeline's range");
  Pipe P;
  const size_t need = make_staged_pipe(m, workspace, n_env, banks, &P, true, RK_OBS);
  if (bytes < need) return fail(MGX_E_ARG, "workspace smaller than mgx_bipedal_workspace_bytes");
  MGX_HIPCHK(hipMemsetAsync(workspace, 0, need, st));
  const size_t nb = (size_t)n_env * (banks > 0 ? banks : 1);
  MGX_HIPCHK(hipMemsetAsync(P.base + P.o_bk, 0xFF, nb * 4, st));  // bank settle counters = -1 (empty)
  if (m->precision == MGX_F32) {
    if (m->L.gB) hipLaunchKernelGGL((k_rk_template<float, true>), dim3(1), dim3(64), m->L.bytes, st, m->mf, P);
    else hipLaunchKernelGGL((k_rk_template<float, false>), dim3(1), dim3(64), m->L.bytes, st, m->mf, P);
  } else {
    if (m->L.gB) hipLaunchKernelGGL((k_rk_template<double, true>), dim3(1), dim3(64), m->L.bytes, st, m->md, P);
    else hipLaunchKernelGGL((k_rk_template<double, false>), dim3(1), dim3(64), m->L.bytes, st, m->md, P);
  }
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}
}  // namespace mgx

extern "C" {
int mgx_bipedal_workspace_layout(const mgx_model* m, int n_env, int banks, int64_t* out, int n_out) {
  if (!m || !out || n_env <= 0 || banks < 0 || banks > 16 || n_out < 6) return fail(MGX_E_ARG, "bad argument");
  if (!m->staged_rk_ok) return fail(MGX_E_UNSUPPORTED, "staged RK4 step: model outside the staged pipeline's range");
  Pipe P;
  make_staged_pipe(m, nullptr, n_env, banks, &P, true, RK_OBS);
  const int64_t v[12] = {(int64_t)P.o_rk, P.rk_stride, (int64_t)P.o_rks, (int64_t)P.o_ne, P.S,
                         m->precision == MGX_F32 ? 4 : 8, (int64_t)P.o_scal, P.maxE, (int64_t)P.o_niter,
                         (int64_t)P.o_B, P.bcap, (int64_t)P.o_blk};
  for (int i = 0; i < (n_out < 12 ? n_out : 12); i++) out[i] = v[i];
  return MGX_OK;
}
int64_t mgx_bipedal_workspace_bytes(const mgx_model* m, int n_env, int banks) {
  return bipedal_workspace_bytes(m, n_env, banks);
}
int mgx_bipedal_workspace_init(const mgx_model* m, void* workspace, uint64_t bytes, int n_env, int banks, void* stream) {
  return bipedal_workspace_init(m, workspace, bytes, n_env, banks, (hipStream_t)stream);
}
}  // extern "C"
