// mgx_pk_staged.hip — the staged quadruped_parkour step (BASELINE configs[1]).
//
// The monolithic parkour kernel (mgx_parkour.hip) runs one env step per wave: clip, ten serial
// mj_step's of 1 ms (parkour_env.py:367-368, each with its own 50-sweep PGS), obstacle motors,
// observation / reward / termination. Here each physics substep k = 0..9 is the staged soccer
// pipeline's three kernels over the same workspace layout (mgx_staged.h):
//
//   R(k)  k_pk_rows     wave per slot: the state -> checkPos / checkVel -> forward up to the
//                       constraint rows (stage_rows); k = 0 also the action clip -> ctrl[:16]
//   S(k)  k_pgs_groups  the lane-group PGS (16 lanes per slot, four slots per wave, heaviest first)
//   F(k)  k_pk_finish   wave per slot: qacc, checkAcc, Euler -> the state; k = 9 the task logic
//                       (parkour_env.py:371-394: obstacle motors, obs, reward, termination) and
//                       the same-step autoreset
//
// Reset banks: a parkour reset is mj_resetData + the start pose + two obstacle draws + ten settle
// mj_step's (parkour_env.py:314-354). A bank record advances one settle step per substep launch
// as an extra slot, so a bank restarted at the end of env step t is ready at the end of step t+1
// (its tenth settle step runs in substep 9's bank finisher, before the live finisher that may
// install it): one bank per env covers every autoreset. reset() and a reset whose bank is not ready
// run k_pk_settle, the same stages in one wave, in this translation unit (one set of flags), so a
// reset has one arithmetic whatever the bank count.
#include "mgx_internal.h"

using namespace mgx;

namespace mgx {

constexpr int PK_LPS = 16;  // solver lanes per slot
constexpr int PK_OBS = 95;  // parkour_env.py:396-468
enum { PK_SETTLE_RESET = 0, PK_SETTLE_FIXUP = 1 };
enum { PK_SUBSTEPS = 10 };  // frame_skip (parkour_env.py:367-368)

// ---------------------------------------------------------------- banks
// record bi restarts for `episode`: mj_resetData, the start pose and the obstacle draws d0 / d1
// (parkour_reset_body's prologue), zero velocities / warmstart, settle counter 0
template <typename T>
__device__ __forceinline__ void pk_bank_init_draws(const DevModel<T>& m, Env<T>& e, const ParkourIds<T>& ids,
                                                   const Pipe& P, int bi, int episode, uint64_t seed, T d0, T d1) {
  const int l = lane_id();
  reset_env(m, e);
  if (l == 0) {
    e.qpos[0] = (T)2.0; e.qpos[1] = (T)0.0; e.qpos[2] = (T)0.6;
    e.qpos[3] = (T)1; e.qpos[4] = 0; e.qpos[5] = 0; e.qpos[6] = 0;
    e.qpos[ids.platform_qpos] = d0;
    e.qpos[ids.pendulum_qpos] = d1;
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
__device__ __forceinline__ void pk_bank_init(const DevModel<T>& m, Env<T>& e, const ParkourIds<T>& ids, const Pipe& P,
                                             int env, int bi, int episode, uint64_t seed, int env_offset) {
  parkour_philox_draws(seed, (uint32_t)(env_offset + env), (uint32_t)episode, e.vec1);
  wsync();
  const T d0 = e.vec1[0], d1 = e.vec1[1];
  wsync();
  pk_bank_init_draws(m, e, ids, P, bi, episode, seed, d0, d1);
}

// settle finished: the reset observation (parkour_reset_body's epilogue) from the last settle
// step's frames and contacts (the finisher's Env)
template <typename T>
__device__ __forceinline__ void pk_bank_finalize(const DevModel<T>& m, Env<T>& e, const ParkourIds<T>& ids,
                                                 const Pipe& P, int bi) {
  const int fm = parkour_foot_mask(e, ids);
  parkour_obs(m, e, ids, fm, P.at<float>(P.o_bobs) + (size_t)bi * PK_OBS);
  wsync();
}

// the settled reset of record bi becomes env's live state for episode E (parkour_env.py:314-354
// outcome: state, zero controls / applied forces, the tracking reset, obs); episode E + 1
template <typename T>
__device__ __forceinline__ void pk_bank_copy_live(const DevModel<T>& m, const Pipe& P, mgx_state s,
                                                  mgx_parkour_env ev, float* obs, int env, int bi, int E) {
  const int l = lane_id();
  copy_g((T*)s.qpos + (size_t)env * m.nq, P.at<T>(P.o_bq) + (size_t)bi * m.nq, m.nq);
  copy_g((T*)s.qvel + (size_t)env * m.nv, P.at<T>(P.o_bv) + (size_t)bi * m.nv, m.nv);
  copy_g((T*)s.qacc_warmstart + (size_t)env * m.nv, P.at<T>(P.o_ba) + (size_t)bi * m.nv, m.nv);
  for (int k = l; k < m.nv; k += 64) ((T*)s.qfrc_applied)[(size_t)env * m.nv + k] = 0;
  for (int k = l; k < m.nu; k += 64) ((T*)s.ctrl)[(size_t)env * m.nu + k] = 0;
  for (int k = l; k < 6 * m.nbody; k += 64) ((T*)s.xfrc_applied)[(size_t)env * 6 * m.nbody + k] = 0;
  copy_g(obs + (size_t)env * PK_OBS, P.at<float>(P.o_bobs) + (size_t)bi * PK_OBS, PK_OBS);
  T* lp = (T*)ev.last_position + 3 * (size_t)env;
  if (l == 0) {
    lp[0] = (T)2.0; lp[1] = (T)0.0; lp[2] = (T)0.6;
    ((T*)ev.max_progress)[env] = 0;
    ev.episode_reward[env] = 0.0;
    ev.er_kind[env] = 0;
    ev.reached[env] = 0; ev.fall_count[env] = 0; ev.stuck[env] = 0; ev.step[env] = 0;
    ((T*)s.time)[env] = P.at<T>(P.o_btime)[bi];
    if (s.warning) s.warning[env] += P.at<int>(P.o_bwarn)[bi];
    if (ev.episode) ev.episode[env] = E + 1;
  }
  wsync();
}

// ---------------------------------------------------------------- kernels
// R(k): live slot b < n_env (the env's state; k = 0: the action clip), or bank record b - n_env
// (its settle step bk, while 0 <= bk < 10)
template <typename T>
__global__ void __launch_bounds__(64) k_pk_rows(DevModel<T> m, ParkourIds<T> ids, mgx_state s, const float* action,
                                                int action_f64, int n_env, const uint8_t* mask, Pipe P, int banks,
                                                int sub) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x;
  Env<T> e;
  if (b < n_env) {
    if (mask && !mask[b]) return;
    env_bind(m, e, smem);
    bind_carry_tail(m, e, P, b);
    load_state(m, e, (T*)s.qpos, (T*)s.qvel, (T*)s.qacc_warmstart, (T*)s.ctrl, (T*)s.qfrc_applied, (T*)s.xfrc_applied,
               (T*)s.time, b);
    if (sub == 0) parkour_pre(m, e, ids, ActRow(action, action_f64, b, ids.n_leg));
  } else {
    const int bi = b - n_env;
    if (!banks || bi >= n_env * P.R) return;
    const int k = P.at<int>(P.o_bk)[bi];
    if (k < 0 || k >= 10) return;
    env_bind(m, e, smem);
    bind_carry_tail(m, e, P, b);
    bank_load_state(m, e, P, bi);
  }
  int warn = 0;  // mj_checkPos / mj_checkVel
  if (any_bad(e.qpos, m.nq)) { reset_env(m, e); warn++; }
  if (any_bad(e.qvel, m.nv)) { reset_env(m, e); warn++; }
  stage_rows(m, e, P, b, warn);
}

// F(k), bank part: record bi's settle step (one wave per record), launched before the live part so
// that a record completing its tenth step in substep 9 is ready for this step's resets
template <typename T>
__global__ void __launch_bounds__(64) k_pk_bank_finish(DevModel<T> m, ParkourIds<T> ids, int n_env, Pipe P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int bi = blockIdx.x;
  if (bi >= n_env * P.R) return;
  int k = P.at<int>(P.o_bk)[bi];
  if (k < 0 || k >= 10) return;
  Env<T> e;
  env_bind(m, e, smem);
  const int slot = n_env + bi;
  int warn = load_carry(m, e, P, slot);
  if (!finish_physics(m, e, P, slot)) {
    load_template(m, e, P);
    warn++;
  }
  bank_store_state(m, e, P, bi, warn);
  k++;
  if (k == 10) pk_bank_finalize(m, e, ids, P, bi);
  if (lane_id() == 0) P.at<int>(P.o_bk)[bi] = k;
}

// F(k), live part: the env's substep; after substep 9 the task logic and the autoreset. The
// overflow flag of the env step is the OR over its substeps (o_pko), counted once.
template <typename T>
__global__ void __launch_bounds__(64) k_pk_finish(DevModel<T> m, ParkourIds<T> ids, mgx_state s, mgx_parkour_env ev,
                                                  const float* action, float* obs, double* reward, uint8_t* terminated,
                                                  uint8_t* truncated, float* final_obs, int autoreset, uint64_t seed,
                                                  int env_offset, int n_env, const uint8_t* mask, Pipe P, int banks,
                                                  int sub) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int env = blockIdx.x;
  if (env >= n_env) return;
  const int l = lane_id();
  if (env == 0 && l == 0) {  // this substep's solver lists are consumed
    P.ctr()[3] = P.ctr()[1];
    P.ctr()[4] = P.ctr()[2];
    P.ctr()[1] = 0;
    P.ctr()[2] = 0;
    if (sub == 0) P.ctr()[5] = 0;  // the env step's fixup list
  }
  if (env == 0)
    for (int b = l; b < P.nbk; b += 64) P.at<int>(P.o_hist)[b] = 0;
  Env<T> e;
  env_bind(m, e, smem);
  if (mask && !mask[env]) return;
  int warn = load_carry(m, e, P, env);
  if (!finish_physics(m, e, P, env)) {
    load_template(m, e, P);
    warn++;
  }
  int* ovf = P.at<int>(P.o_rkw) + env;  // the env step's overflow flag (o_rkw: per-slot ints)
  const bool over = (sub > 0 && *ovf != 0) || e.overflow != 0;
  if (l == 0 && s.warning) s.warning[env] += warn;
  if (sub < PK_SUBSTEPS - 1) {
    store_state(m, e, (T*)s.qpos, (T*)s.qvel, (T*)s.qacc_warmstart, (T*)s.ctrl, (T*)s.qfrc_applied,
                (T*)s.xfrc_applied, (T*)s.time, env);
    if (l == 0) *ovf = over ? 1 : 0;
    return;
  }
  if (l == 0 && s.overflow && over) s.overflow[env] += 1;
  const bool done =
      parkour_post(m, e, ids, ActRow(action, ev.action_f64, env, ids.n_leg), ev, env, obs, reward, terminated, truncated);
  if (ev.rollout && l == 0) {
    T* ro = (T*)ev.rollout + 4 * (size_t)env;
    ro[0] += (T)reward[env];
    ro[1] += (T)terminated[env];
    ro[2] += (T)truncated[env];
    ro[3] += (T)1;
  }
  store_state(m, e, (T*)s.qpos, (T*)s.qvel, (T*)s.qacc_warmstart, (T*)s.ctrl, (T*)s.qfrc_applied, (T*)s.xfrc_applied,
              (T*)s.time, env);
  if (!(done && autoreset)) return;
  if (final_obs)
    for (int i = l; i < PK_OBS; i += 64) final_obs[(size_t)env * PK_OBS + i] = obs[(size_t)env * PK_OBS + i];
  __threadfence();
  wsync();
  const int E = ev.episode[env];
  bool ready = false;
  int bi = 0;
  if (banks && P.R > 0) {
    bi = env * P.R + E % P.R;
    ready = P.at<int>(P.o_bk)[bi] == 10 && P.at<int>(P.o_bep)[bi] == E && P.at<uint64_t>(P.o_bseed)[bi] == seed;
  }
  if (ready) {
    pk_bank_copy_live(m, P, s, ev, obs, env, bi, E);
    pk_bank_init(m, e, ids, P, env, bi, E + P.R, seed, env_offset);
  } else if (l == 0) {
    P.at<int>(P.o_fix)[atomicAdd(P.ctr() + 5, 1)] = env;
  }
}

// One settle step of record bi in one wave, through pipe slot `slot`: the pipeline's stages in
// sequence (stage_rows, the PGS of the one slot, finish_physics / checkAcc template, the record's
// store). Returns with the finisher's Env (layout Mf) in `smem`.
template <typename T, int EPL>
__device__ __forceinline__ void pk_settle_step(const DevModel<T>& Ms, const DevModel<T>& Mf, const ParkourIds<T>& ids,
                                               const Pipe& P, char* smem, Env<T>& f, int bi, int slot, int maxit, T tol,
                                               T scale, bool last) {
  {
    Env<T> e;
    env_bind(Ms, e, smem);
    bind_carry_tail(Ms, e, P, slot);
    bank_load_state(Ms, e, P, bi);
    int warn = 0;
    if (any_bad(e.qpos, Ms.nq)) { reset_env(Ms, e); warn++; }
    if (any_bad(e.qvel, Ms.nv)) { reset_env(Ms, e); warn++; }
    stage_rows(Ms, e, P, slot, warn, false);
  }
  __threadfence();
  __syncthreads();
  pgs_group<T, EPL, PK_LPS, false>(P, smem, threadIdx.x < PK_LPS ? slot : -1, P.maxE, maxit, tol, scale, 64 / PK_LPS);
  __threadfence();
  __syncthreads();
  env_bind(Mf, f, smem);
  int warn = load_carry(Mf, f, P, slot);
  if (!finish_physics(Mf, f, P, slot)) {
    load_template(Mf, f, P);
    warn++;
  }
  bank_store_state(Mf, f, P, bi, warn);
  if (last) pk_bank_finalize(Mf, f, ids, P, bi);
  __threadfence();
  __syncthreads();
}

// restart record bi for `episode` (host draws or Philox) and settle it (ten mj_step's); bk = 10
template <typename T, int EPL>
__device__ __forceinline__ void pk_settle_reset(const DevModel<T>& Ms, const DevModel<T>& Mf, const ParkourIds<T>& ids,
                                                const Pipe& P, char* smem, int env, int bi, int episode, const T* draws,
                                                uint64_t seed, int env_offset, int maxit, T tol, T scale) {
  {
    Env<T> e;
    env_bind(Ms, e, smem);
    bind_carry_tail(Ms, e, P, env);
    if (draws) {
      pk_bank_init_draws(Ms, e, ids, P, bi, episode, seed, draws[0], draws[1]);
    } else {
      pk_bank_init(Ms, e, ids, P, env, bi, episode, seed, env_offset);
    }
  }
  __threadfence();
  __syncthreads();
  Env<T> f;
  for (int t = 0; t < 10; t++) pk_settle_step<T, EPL>(Ms, Mf, ids, P, smem, f, bi, env, maxit, tol, scale, t == 9);
  if (lane_id() == 0) P.at<int>(P.o_bk)[bi] = 10;
  __threadfence();
  __syncthreads();
}

// reset() of a staged batch (PK_SETTLE_RESET: one workgroup per env; with Philox draws and banks it
// also prefills the env's banks) and the step's fallback for banks that were not ready
// (PK_SETTLE_FIXUP: grid-stride over the finisher's list)
template <typename T, int EPL>
__global__ void __launch_bounds__(64) k_pk_settle(DevModel<T> Ms, DevModel<T> Mf, ParkourIds<T> ids, mgx_state s,
                                                  mgx_parkour_env ev, const T* draws, float* obs, uint64_t seed,
                                                  int env_offset, int n_env, const uint8_t* mask, Pipe P, int mode,
                                                  int maxit, T tol, T scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int cnt = mode == PK_SETTLE_FIXUP ? P.ctr()[5] : n_env;
  for (int i = blockIdx.x; i < cnt; i += gridDim.x) {
    const int env = mode == PK_SETTLE_FIXUP ? P.at<int>(P.o_fix)[i] : i;
    if (mode == PK_SETTLE_RESET && mask && !mask[env]) continue;
    const int E = ev.episode ? ev.episode[env] : 0;
    const int bi = P.R > 0 ? env * P.R + E % P.R : env;
    const T* d = draws ? draws + 2 * (size_t)env : nullptr;
    pk_settle_reset<T, EPL>(Ms, Mf, ids, P, smem, env, bi, E, d, seed, env_offset, maxit, tol, scale);
    pk_bank_copy_live(Mf, P, s, ev, obs, env, bi, E);
    if (P.R > 0 && mode == PK_SETTLE_FIXUP) {
      Env<T> e;
      env_bind(Ms, e, smem);
      bind_carry_tail(Ms, e, P, env);
      pk_bank_init(Ms, e, ids, P, env, bi, E + P.R, seed, env_offset);
    } else if (P.R > 0 && !draws) {
      for (int k = 1; k <= P.R; k++)
        pk_settle_reset<T, EPL>(Ms, Mf, ids, P, smem, env, env * P.R + (E + k) % P.R, E + k, (const T*)nullptr, seed,
                                env_offset, maxit, tol, scale);
    } else if (lane_id() == 0) {
      P.at<int>(P.o_bk)[bi] = -1;  // a scratch record: nothing to settle
    }
    __threadfence();
    __syncthreads();
  }
}

// mj_checkAcc's outcome: mj_step from mj_resetData (monolithic layout; rows in the pipe's template
// scratch when the model keeps its rows in global memory), into the template arrays
template <typename T, bool GB>
__global__ void __launch_bounds__(64) k_pk_template(DevModel<T> m, Pipe P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Env<T> e;
  env_bind<T, GB>(m, e, smem, GB ? P.at<T>(P.o_tscr) : nullptr);
  const int l = lane_id();
  reset_env(m, e);
  forward(m, e);
  e.qacc_ws = e.qacc;
  euler(m, e);
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

// register entries per solver lane of the parkour model (16 lanes per slot: two 8-dof groups per
// entry): nv 33..48 -> 3
template <typename T>
int pk_epl(const DevModel<T>& M) {
  return ((M.nv + 7) / 8 + 1) / 2;
}

int pk_settle_lds(const mgx_model* m, const Pipe& P) {
  int b = staged_pgs_lds_bytes(m, P.maxE, PK_LPS, 0, 8);
  if (m->Ls.bytes > b) b = m->Ls.bytes;
  if (m->Lf.bytes > b) b = m->Lf.bytes;
  return b;
}

#define MGX_PK_EPL(EPL_VAR, CALL) \
  switch (EPL_VAR) {              \
    case 1: { constexpr int E = 1; CALL; } break; \
    case 2: { constexpr int E = 2; CALL; } break; \
    case 3: { constexpr int E = 3; CALL; } break; \
    default: { constexpr int E = 4; CALL; } break; \
  }

template <typename T>
int step_staged(const mgx_model* m, const DevModel<T>& M, const DevModel<T>& Ms, const DevModel<T>& Mf,
                const ParkourIds<T>& ids, const mgx_state* s, const mgx_parkour_env* e, const float* action,
                float* obs, double* reward, uint8_t* terminated, uint8_t* truncated, float* final_obs, int autoreset,
                uint64_t seed, int env_offset, int n_env, const uint8_t* mask, hipStream_t st) {
  Pipe P;
  const int banks = autoreset ? e->banks : 0;
  const size_t need = make_staged_pipe(m, e->workspace, n_env, e->banks, &P, false, PK_OBS);
  if (e->workspace_bytes < need) return fail(MGX_E_ARG, "workspace smaller than mgx_parkour_workspace_bytes");
  // parkour_staged_ok: every slot is solved by the main launch (a slot over capE rows, e.g. the
  // qpos0 pile-up after a bad-state reset, in its heaviest-first list with its scalars read from
  // the pipe: Pipe.hmain)
  const int slots = n_env * (1 + banks);
  const T scale = (T)1 / (M.meaninertia * (T)(M.nv > 1 ? M.nv : 1));
  const int mlds = std::max(staged_pgs_lds_bytes(m, P.capE, PK_LPS, 0, 8),
                           P.hmain ? staged_pgs_lds_bytes(m, P.maxE, PK_LPS, 1, 8) : 0);
  const int spw = 64 / PK_LPS, grid = (slots + spw - 1) / spw;
  for (int k = 0; k < PK_SUBSTEPS; k++) {
    hipLaunchKernelGGL(k_pk_rows<T>, dim3(slots), dim3(64), m->Ls.bytes, st, Ms, ids, *s, action, e->action_f64, n_env,
                       mask, P, banks, k);
    MGX_PK_EPL(pk_epl(M), hipLaunchKernelGGL((k_pgs_groups<T, E, PK_LPS, false>), dim3(grid), dim3(64), mlds, st, P,
                                             M.iterations, M.tolerance, scale, spw, 0));
    if (banks && P.R > 0)
      hipLaunchKernelGGL(k_pk_bank_finish<T>, dim3(n_env * P.R), dim3(64), m->Lf.bytes, st, Mf, ids, n_env, P);
    hipLaunchKernelGGL(k_pk_finish<T>, dim3(n_env), dim3(64), m->Lf.bytes, st, Mf, ids, *s, *e, action, obs, reward,
                       terminated, truncated, final_obs, autoreset, seed, env_offset, n_env, mask, P, banks, k);
  }
  const int fgrid = n_env < 256 ? n_env : 256;
  MGX_PK_EPL(pk_epl(M), hipLaunchKernelGGL((k_pk_settle<T, E>), dim3(fgrid), dim3(64), pk_settle_lds(m, P), st, Ms, Mf,
                                           ids, *s, *e, (const T*)nullptr, obs, seed, env_offset, n_env,
                                           (const uint8_t*)nullptr, P, (int)PK_SETTLE_FIXUP, M.iterations, M.tolerance,
                                           scale));
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}

template <typename T>
int reset_staged(const mgx_model* m, const DevModel<T>& M, const DevModel<T>& Ms, const DevModel<T>& Mf,
                 const ParkourIds<T>& ids, const mgx_state* s, const mgx_parkour_env* e, const T* draws, float* obs,
                 uint64_t seed, int env_offset, int n_env, const uint8_t* mask, hipStream_t st) {
  Pipe P;
  const size_t need = make_staged_pipe(m, e->workspace, n_env, e->banks, &P, false, PK_OBS);
  if (e->workspace_bytes < need) return fail(MGX_E_ARG, "workspace smaller than mgx_parkour_workspace_bytes");
  const T scale = (T)1 / (M.meaninertia * (T)(M.nv > 1 ? M.nv : 1));
  MGX_PK_EPL(pk_epl(M), hipLaunchKernelGGL((k_pk_settle<T, E>), dim3(n_env), dim3(64), pk_settle_lds(m, P), st, Ms, Mf,
                                           ids, *s, *e, draws, obs, seed, env_offset, n_env, mask, P,
                                           (int)PK_SETTLE_RESET, M.iterations, M.tolerance, scale));
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}

template <typename T>
int configure_t(const mgx_model* m) {
  Pipe P;
  make_staged_pipe(m, nullptr, 1, 1, &P, false, PK_OBS);
  const int pl = staged_pgs_lds_bytes(m, P.maxE, PK_LPS, 0, 8);
  if (pl > 160 * 1024) return fail(MGX_E_CAPACITY, "staged parkour solver LDS exceeds 160 KiB");
  int rc = mgx_set_lds(k_pk_rows<T>, m->Ls.bytes) | mgx_set_lds(k_pk_finish<T>, m->Lf.bytes) |
           mgx_set_lds(k_pk_bank_finish<T>, m->Lf.bytes) | mgx_set_lds(k_pk_template<T, true>, m->L.bytes) |
           mgx_set_lds(k_pk_template<T, false>, m->L.bytes);
  const int sl = pk_settle_lds(m, P);
#define MGX_PK_SET(E) rc |= mgx_set_lds(k_pk_settle<T, E>, sl) | mgx_set_lds(k_pgs_groups<T, E, PK_LPS, false>, pl);
  MGX_PK_SET(1) MGX_PK_SET(2) MGX_PK_SET(3) MGX_PK_SET(4)
#undef MGX_PK_SET
  return rc;
}

}  // namespace

namespace mgx {
// The staged parkour step runs the main solver launch only (no wide launch beside it): a model
// (with its hooks) whose pipe would need one is refused here, and the env falls back to the
// monolithic step (envs/parkour.py), which holds the same capacity.
bool parkour_staged_ok(const mgx_model* m) {
  const int nv = m->precision == MGX_F32 ? m->mf.nv : m->md.nv;
  if (!m->staged_ok || nv > 64 || pgs_lanes() != PK_LPS || m->hooks.pgs_lds_b) return false;
  Pipe P;
  make_staged_pipe(m, nullptr, 1, 1, &P, false, PK_OBS);
  return !P.sqg && (P.maxE <= P.capE || P.hmain);
}

int parkour_staged_configure(const mgx_model* m) {
  if (!parkour_staged_ok(m)) return MGX_OK;
  return m->precision == MGX_F32 ? configure_t<float>(m) : configure_t<double>(m);
}

int parkour_step_staged(const mgx_model* m, const mgx_state* s, const mgx_parkour_env* e, const float* action, float* obs,
                        double* reward, uint8_t* terminated, uint8_t* truncated, float* final_obs, int autoreset,
                        uint64_t seed, int env_offset, int n_env, const uint8_t* mask, hipStream_t st) {
  if (!parkour_staged_ok(m)) return fail(MGX_E_UNSUPPORTED, "staged parkour step: model outside the staged pipeline");
  if (e->banks < 0 || e->banks > 16) return fail(MGX_E_ARG, "banks must be in [0, 16]");
  if (m->precision == MGX_F32)
    return step_staged<float>(m, m->mf, m->mfs, m->mff, m->pkf, s, e, action, obs, reward, terminated, truncated,
                              final_obs, autoreset, seed, env_offset, n_env, mask, st);
  return step_staged<double>(m, m->md, m->mds, m->mdf, m->pkd, s, e, action, obs, reward, terminated, truncated,
                             final_obs, autoreset, seed, env_offset, n_env, mask, st);
}

int parkour_reset_staged(const mgx_model* m, const mgx_state* s, const mgx_parkour_env* e, const void* draws,
                         float* obs, uint64_t seed, int env_offset, int n_env, const uint8_t* mask, hipStream_t st) {
  if (!parkour_staged_ok(m)) return fail(MGX_E_UNSUPPORTED, "staged parkour step: model outside the staged pipeline");
  if (e->banks < 0 || e->banks > 16) return fail(MGX_E_ARG, "banks must be in [0, 16]");
  if (m->precision == MGX_F32)
    return reset_staged<float>(m, m->mf, m->mfs, m->mff, m->pkf, s, e, (const float*)draws, obs, seed, env_offset,
                               n_env, mask, st);
  return reset_staged<double>(m, m->md, m->mds, m->mdf, m->pkd, s, e, (const double*)draws, obs, seed, env_offset,
                              n_env, mask, st);
}

int64_t parkour_workspace_bytes(const mgx_model* m, int n_env, int banks) {
  if (!m || n_env <= 0 || banks < 0 || banks > 16) return fail(MGX_E_ARG, "bad argument");
  if (!parkour_staged_ok(m)) return fail(MGX_E_UNSUPPORTED, "staged parkour step: model outside the staged pipeline");
  return (int64_t)make_staged_pipe(m, nullptr, n_env, banks, nullptr, false, PK_OBS);
}

int parkour_workspace_init(const mgx_model* m, void* workspace, uint64_t bytes, int n_env, int banks, hipStream_t st) {
  if (!m || !workspace || n_env <= 0 || banks < 0 || banks > 16) return fail(MGX_E_ARG, "bad argument");
  if (!parkour_staged_ok(m)) return fail(MGX_E_UNSUPPORTED, "staged parkour step: model outside the staged pipeline");
  Pipe P;
  const size_t need = make_staged_pipe(m, workspace, n_env, banks, &P, false, PK_OBS);
  if (bytes < need) return fail(MGX_E_ARG, "workspace smaller than mgx_parkour_workspace_bytes");
  MGX_HIPCHK(hipMemsetAsync(workspace, 0, need, st));
  const size_t nb = (size_t)n_env * (banks > 0 ? banks : 1);
  MGX_HIPCHK(hipMemsetAsync(P.base + P.o_bk, 0xFF, nb * 4, st));  // bank settle counters = -1 (empty)
  if (m->precision == MGX_F32) {
    if (m->L.gB) hipLaunchKernelGGL((k_pk_template<float, true>), dim3(1), dim3(64), m->L.bytes, st, m->mf, P);
    else hipLaunchKernelGGL((k_pk_template<float, false>), dim3(1), dim3(64), m->L.bytes, st, m->mf, P);
  } else {
    if (m->L.gB) hipLaunchKernelGGL((k_pk_template<double, true>), dim3(1), dim3(64), m->L.bytes, st, m->md, P);
    else hipLaunchKernelGGL((k_pk_template<double, false>), dim3(1), dim3(64), m->L.bytes, st, m->md, P);
  }
  MGX_HIPCHK(hipGetLastError());
  return MGX_OK;
}
}  // namespace mgx
