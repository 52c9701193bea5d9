// mgx_physics.h — one mj_step for one env, executed by one wavefront.
//
// Stage order restates MuJoCo's mj_step [ext] as reached from the reference's hot path
// (humanoid_soccer_env/soccer_env.py:414): checkPos/Vel -> kinematics -> comPos -> CRB ->
// factorM -> collision -> makeConstraint -> (B = D^-1/2 L^-T J') -> comVel -> passive ->
// RNE -> actuation -> xfrc -> qacc_smooth -> PGS (warmstart) -> checkAcc -> Euler with
// implicit damping -> integratePos.
//
// Data placement: everything per-env lives in LDS; dof-indexed vectors that
// only feed solves live in registers (lane k = dof k) and move with readlane; the constraint
// Jacobian is never stored — each row is turned into B_r = D^-1/2 L^-T J_r' in place, so the
// Delassus operator is A = B B' + R and PGS keeps v = B' f in registers (one LDS row read and
// one wave reduction per row update).
#pragma once
#include "mgx_collide.h"

namespace mgx {

template <typename T>
struct Env {
  T *qpos, *qvel, *ctrl, *xfrc, *xpos, *xquat, *xmat, *xipos, *ximat, *subtree_com, *cinert, *crb, *cvel, *cfrc;
  T *xaxis, *xanchor, *cdof, *cdof_dot, *qLD, *qMH, *vec0, *vec1, *vec2, *vec3, *geom_xpos, *geom_xmat, *act_force, *cacc, *rowc;
  T *con_dist, *con_pos, *con_frame, *con_mu;  // con_mu = |friction[0:2]| (soccer obs)
  // per-row constraint data, AoS with stride 8 so the solver fetches a row's scalars with one
  // 16-byte LDS read: [0] b, [1] f, [2] R (diagApprox until impedance), [3] 1/AR_rr,
  // [4] AR_rr, [5] aref (K*imp*(pos-margin) until the solver), [6] B damping, [7] pos
  T *efc, *efc_margin, *efc_blk;
  T *Bm;
  int Bs;
  T *rk;  // RK4: X[0] positions [nq] then the dX velocity vector [nv]
  T *hess;  // Newton: nv x nv Hessian / its Cholesky factor (row-major, lower)
  int *con_geom, *con_pair, *act_list, *efc_type, *efc_id, *con_efcadr;
  int ncon, nefc, niter, overflow;
  int nw;    // waves per env: 1, or 2 (wave 0 + a Newton helper wave, team_begin)
  int* ctl;  // helper section command words (team_off)
  // dof-lane registers
  T qacc_ws, qfrc_applied, qfrc_smooth, qacc_smooth, qacc, qfrc_constraint, diaginv, time;
  int chainlen, madr;  // this lane's dof: chain length, dof_Madr
  uint64_t ancmask;
};

// GB: B rows in global scratch (gB = this env's slice) instead of LDS (Layout.gB); EG: the per-row
// constraint data as well (gb_efc_off: the wide kernels)
template <typename T, bool GB = false, bool EG = false>
__device__ __forceinline__ void env_bind(const DevModel<T>& m, Env<T>& e, char* smem, T* gB = nullptr) {
  T* R = reinterpret_cast<T*>(smem);
  const Layout& L = m.L;
  e.qpos = R + L.qpos; e.qvel = R + L.qvel; e.ctrl = R + L.ctrl; e.xfrc = R + L.xfrc;
  e.xpos = R + L.xpos; e.xquat = R + L.xquat; e.xmat = R + L.xmat; e.xipos = R + L.xipos;
  e.ximat = R + L.ximat; e.subtree_com = R + L.subtree_com; e.cinert = R + L.cinert; e.crb = R + L.crb;
  e.cvel = R + L.cvel; e.cfrc = R + L.cfrc; e.xaxis = R + L.xaxis; e.xanchor = R + L.xanchor;
  e.cdof = R + L.cdof; e.cdof_dot = R + L.cdof_dot; e.qLD = R + L.qLD; e.qMH = R + L.qMH;
  e.vec0 = R + L.vec0; e.vec1 = R + L.vec1; e.vec2 = R + L.vec2; e.vec3 = R + L.vec3; e.geom_xpos = R + L.geom_xpos;
  e.geom_xmat = R + L.geom_xmat; e.act_force = R + L.act_force; e.cacc = R + L.cacc; e.rowc = R + L.rowc; e.con_dist = R + L.con_dist;
  e.con_pos = R + L.con_pos; e.con_frame = R + L.con_frame; e.con_mu = R + L.con_mu; e.efc = R + L.efc;
  e.efc_margin = R + L.efc_margin; e.efc_blk = R + L.efc_blk; e.Bs = L.Bstride;
  if constexpr (EG) { e.efc = gB + gb_efc_off(L, sizeof(T)); e.efc_margin = gB + gb_efm_off(L, sizeof(T)); }
  if constexpr (GB) e.Bm = gB;
  else e.Bm = R + L.Bmat;
  e.rk = R + L.rk;
  e.hess = R + L.hess;
  int* I = reinterpret_cast<int*>(R + L.reals);
  e.con_geom = I + L.con_geom; e.con_pair = I + L.con_pair;
  e.act_list = L.act_union > 0 ? reinterpret_cast<int*>(R + L.act_union) : I + L.act_list;
  e.efc_type = I + L.efc_type; e.con_efcadr = I + L.con_efcadr;
#ifdef MGX_TEAM
  e.nw = blockDim.x >> 6;
  e.ctl = I + team_off(L);
#else
  e.nw = 1;  // one wave per workgroup (lane_id, mgx_common.h)
  e.ctl = nullptr;
#endif
  // the staged row builder lists only its joint-limit rows, after collision, in the broadphase list
  e.efc_id = L.staged ? e.act_list : I + L.efc_id;
  // the staged row builder's carry tail lives in global memory (bind_carry_tail)
  if (L.carry_lds < L.carry_reals) { e.xfrc = nullptr; e.qMH = nullptr; e.con_mu = nullptr; }
  if (L.gcon) e.con_pos = nullptr;
  int l = lane_id();
  e.chainlen = l < m.nv ? m.dof_chainlen[l] : 0;
  e.madr = l < m.nv ? m.dof_Madr[l] : 0;
  e.ancmask = l < m.nv ? m.dof_ancmask[l] : 0ull;
  e.overflow = 0;
}

// ---------------------------------------------------------------- state load / store / reset
template <typename T>
__device__ __forceinline__ void load_state(const DevModel<T>& m, Env<T>& e, const T* gqpos, const T* gqvel, const T* gqacc,
                           const T* gctrl, const T* gqfrc, const T* gxfrc, const T* gtime, int env) {
  int l = lane_id();
  for (int k = l; k < m.nq; k += 64) e.qpos[k] = gqpos[(size_t)env * m.nq + k];
  for (int k = l; k < m.nv; k += 64) e.qvel[k] = gqvel[(size_t)env * m.nv + k];
  for (int k = l; k < m.nu; k += 64) e.ctrl[k] = gctrl[(size_t)env * m.nu + k];
  for (int k = l; k < 6 * m.nbody; k += 64) e.xfrc[k] = gxfrc[(size_t)env * 6 * m.nbody + k];
  e.qacc_ws = l < m.nv ? gqacc[(size_t)env * m.nv + l] : (T)0;
  e.qfrc_applied = l < m.nv ? gqfrc[(size_t)env * m.nv + l] : (T)0;
  e.time = gtime[env];
  wsync();
}

template <typename T>
__device__ __forceinline__ void store_state(const DevModel<T>& m, Env<T>& e, T* gqpos, T* gqvel, T* gqacc, T* gctrl, T* gqfrc,
                            T* gxfrc, T* gtime, int env) {
  wsync();
  int l = lane_id();
  for (int k = l; k < m.nq; k += 64) gqpos[(size_t)env * m.nq + k] = e.qpos[k];
  for (int k = l; k < m.nv; k += 64) gqvel[(size_t)env * m.nv + k] = e.qvel[k];
  for (int k = l; k < m.nu; k += 64) gctrl[(size_t)env * m.nu + k] = e.ctrl[k];
  for (int k = l; k < 6 * m.nbody; k += 64) gxfrc[(size_t)env * 6 * m.nbody + k] = e.xfrc[k];
  if (l < m.nv) { gqacc[(size_t)env * m.nv + l] = e.qacc_ws; gqfrc[(size_t)env * m.nv + l] = e.qfrc_applied; }
  if (l == 0) gtime[env] = e.time;
}

// mj_resetData on the LDS copy (soccer_env.py:354 reaches it; also the bad-state reset)
template <typename T>
__device__ __forceinline__ void reset_env(const DevModel<T>& m, Env<T>& e) {
  int l = lane_id();
  wsync();
  for (int k = l; k < m.nq; k += 64) e.qpos[k] = m.qpos0[k];
  for (int k = l; k < m.nv; k += 64) e.qvel[k] = 0;
  for (int k = l; k < m.nu; k += 64) e.ctrl[k] = 0;
  for (int k = l; k < 6 * m.nbody; k += 64) e.xfrc[k] = 0;
  e.qacc_ws = 0;
  e.qfrc_applied = 0;
  e.time = 0;
  wsync();
}

template <typename T>
__device__ __forceinline__ bool any_bad(const T* x, int n) {
  bool b = false;
  for (int k = lane_id(); k < n; k += 64) b |= isbad(x[k]);
  return ballot(b) != 0ull;
}

// ---------------------------------------------------------------- kinematics (mj_kinematics)
// Lane b recomputes the chain root..b, so no level-by-level barriers are needed.
template <typename T>
__device__ __forceinline__ void body_pose_step(const DevModel<T>& m, Env<T>& e, int i, T* pos, T* quat, T* mat, bool store_joints) {
  int ja = m.body_jntadr[i], jn = m.body_jntnum[i];
  if (jn == 1 && m.jnt_type[ja] == JFREE) {
    int a = m.jnt_qposadr[ja];
    pos[0] = e.qpos[a]; pos[1] = e.qpos[a + 1]; pos[2] = e.qpos[a + 2];
    quat[0] = e.qpos[a + 3]; quat[1] = e.qpos[a + 4]; quat[2] = e.qpos[a + 5]; quat[3] = e.qpos[a + 6];
    normalize4(quat);
    if (store_joints) {
      for (int k = 0; k < 3; k++) { e.xanchor[3 * ja + k] = pos[k]; e.xaxis[3 * ja + k] = m.jnt_axis[3 * ja + k]; }
    }
  } else {
    T np[3], nq[4];
    mulmatvec3(np, mat, m.body_pos + 3 * i);
    for (int k = 0; k < 3; k++) np[k] += pos[k];
    mulquat(nq, quat, m.body_quat + 4 * i);
    for (int j = ja; j < ja + jn; j++) {
      int a = m.jnt_qposadr[j];
      T xaxis[3], xanchor[3];
      rotvecquat(xaxis, m.jnt_axis + 3 * j, nq);
      rotvecquat(xanchor, m.jnt_pos + 3 * j, nq);
      for (int k = 0; k < 3; k++) xanchor[k] += np[k];
      int t = m.jnt_type[j];
      if (t == JSLIDE) {
        T s = e.qpos[a] - m.qpos0[a];
        for (int k = 0; k < 3; k++) np[k] += xaxis[k] * s;
      } else if (t == JHINGE || t == JBALL) {
        T ql[4], v[3];
        if (t == JBALL) { ql[0] = e.qpos[a]; ql[1] = e.qpos[a + 1]; ql[2] = e.qpos[a + 2]; ql[3] = e.qpos[a + 3]; normalize4(ql); }
        else axisangle2quat(ql, m.jnt_axis + 3 * j, e.qpos[a] - m.qpos0[a]);
        mulquat(nq, nq, ql);
        rotvecquat(v, m.jnt_pos + 3 * j, nq);
        for (int k = 0; k < 3; k++) np[k] = xanchor[k] - v[k];
      }
      if (store_joints) for (int k = 0; k < 3; k++) { e.xaxis[3 * j + k] = xaxis[k]; e.xanchor[3 * j + k] = xanchor[k]; }
    }
    pos[0] = np[0]; pos[1] = np[1]; pos[2] = np[2];
    quat[0] = nq[0]; quat[1] = nq[1]; quat[2] = nq[2]; quat[3] = nq[3];
  }
  normalize4(quat);
  quat2mat(mat, quat);
}

template <typename T, bool FROMQ>
__device__ __forceinline__ void geom_poses(const DevModel<T>& m, Env<T>& e);

template <typename T>
__device__ __forceinline__ void kinematics(const DevModel<T>& m, Env<T>& e) {
  int l = lane_id();
  for (int b = l; b < m.nbody; b += 64) {
    T pos[3] = {0, 0, 0}, quat[4] = {1, 0, 0, 0}, mat[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    int depth = m.body_depth[b];
    for (int c = 0; c < depth; c++) {
      int i = m.body_chain[b * MGX_MAX_DEPTH + c];
      body_pose_step(m, e, i, pos, quat, mat, i == b);
    }
    for (int k = 0; k < 3; k++) e.xpos[3 * b + k] = pos[k];
    for (int k = 0; k < 4; k++) e.xquat[4 * b + k] = quat[k];
    for (int k = 0; k < 9; k++) e.xmat[9 * b + k] = mat[k];
    T q[4];
    T ip[3];
    mulmatvec3(ip, mat, m.body_ipos + 3 * b);
    for (int k = 0; k < 3; k++) e.xipos[3 * b + k] = ip[k] + pos[k];
    mulquat(q, quat, m.body_iquat + 4 * b);
    quat2mat(e.ximat + 9 * b, q);
  }
  wsync();
  if (!m.L.late_geom) geom_poses<T, false>(m, e);
}

// geom poses (mj_kinematics' geom loop). FROMQ (the staged row builder, Layout.late_geom): the body
// rotation is rebuilt from xquat — kinematics stores xmat = quat2mat(xquat), so this is the same
// matrix — and the poses are computed just before collision, over arrays dead by then.
template <typename T, bool FROMQ>
__device__ __forceinline__ void geom_poses(const DevModel<T>& m, Env<T>& e) {
  const int l = lane_id();
  for (int g = l; g < m.ngeom; g += 64) {
    int b = m.geom_bodyid[g];
    T q[4], gp[3];
    if constexpr (FROMQ) {
      T bm[9];
      quat2mat(bm, e.xquat + 4 * b);
      mulmatvec3(gp, bm, m.geom_pos + 3 * g);
    } else {
      mulmatvec3(gp, e.xmat + 9 * b, m.geom_pos + 3 * g);
    }
    for (int k = 0; k < 3; k++) e.geom_xpos[3 * g + k] = gp[k] + e.xpos[3 * b + k];
    mulquat(q, e.xquat + 4 * b, m.geom_quat + 4 * g);
    quat2mat(e.geom_xmat + 9 * g, q);
  }
  wsync();
}

// ---------------------------------------------------------------- comPos, CRB, M
template <typename T>
__device__ __forceinline__ void inertcom(T* res, const T* inert, const T* mat, const T* dif, T mass) {
  T tmp[9] = {mat[0] * inert[0], mat[3] * inert[0], mat[6] * inert[0],
              mat[1] * inert[1], mat[4] * inert[1], mat[7] * inert[1],
              mat[2] * inert[2], mat[5] * inert[2], mat[8] * inert[2]};
  res[0] = mat[0] * tmp[0] + mat[1] * tmp[3] + mat[2] * tmp[6];
  res[1] = mat[3] * tmp[1] + mat[4] * tmp[4] + mat[5] * tmp[7];
  res[2] = mat[6] * tmp[2] + mat[7] * tmp[5] + mat[8] * tmp[8];
  res[3] = mat[0] * tmp[1] + mat[1] * tmp[4] + mat[2] * tmp[7];
  res[4] = mat[0] * tmp[2] + mat[1] * tmp[5] + mat[2] * tmp[8];
  res[5] = mat[3] * tmp[2] + mat[4] * tmp[5] + mat[5] * tmp[8];
  res[0] += mass * (dif[1] * dif[1] + dif[2] * dif[2]);
  res[1] += mass * (dif[0] * dif[0] + dif[2] * dif[2]);
  res[2] += mass * (dif[0] * dif[0] + dif[1] * dif[1]);
  res[3] -= mass * dif[0] * dif[1];
  res[4] -= mass * dif[0] * dif[2];
  res[5] -= mass * dif[1] * dif[2];
  res[6] = mass * dif[0]; res[7] = mass * dif[1]; res[8] = mass * dif[2];
  res[9] = mass;
}

template <typename T>
__device__ __forceinline__ void com_crb(const DevModel<T>& m, Env<T>& e) {
  int l = lane_id();
  // subtree com: lane b sums its DFS-contiguous subtree
  for (int b = l; b < m.nbody; b += 64) {
    T s0 = 0, s1 = 0, s2 = 0, ms = 0;
    int end = m.body_subtree_end[b];
    for (int i = b; i < end; i++) {
      T mi = m.body_mass[i];
      s0 += e.xipos[3 * i] * mi; s1 += e.xipos[3 * i + 1] * mi; s2 += e.xipos[3 * i + 2] * mi;
      ms += mi;
    }
    if (ms < minval<T>()) { s0 = e.xipos[3 * b]; s1 = e.xipos[3 * b + 1]; s2 = e.xipos[3 * b + 2]; }
    else { T inv = (T)1 / ms; s0 *= inv; s1 *= inv; s2 *= inv; }
    e.subtree_com[3 * b] = s0; e.subtree_com[3 * b + 1] = s1; e.subtree_com[3 * b + 2] = s2;
  }
  wsync();
  for (int b = l; b < m.nbody; b += 64) {
    if (b == 0) { for (int k = 0; k < 10; k++) e.cinert[k] = 0; continue; }
    T off[3];
    int r = m.body_rootid[b];
    for (int k = 0; k < 3; k++) off[k] = e.xipos[3 * b + k] - e.subtree_com[3 * r + k];
    inertcom(e.cinert + 10 * b, m.body_inertia + 3 * b, e.ximat + 9 * b, off, m.body_mass[b]);
  }
  // cdof: lane = dof (dofs l, l + 64, ... when nv > 64)
  for (int d = l; d < m.nv; d += 64) {
    int b = m.dof_bodyid[d], j = m.dof_jntid[d], t = m.jnt_type[j], k = d - m.jnt_dofadr[j];
    T off[3];
    int r = m.body_rootid[b];
    for (int c = 0; c < 3; c++) off[c] = e.subtree_com[3 * r + c] - e.xanchor[3 * j + c];
    T* cd = e.cdof + 6 * d;
    if (t == JFREE && k < 3) {
      for (int c = 0; c < 6; c++) cd[c] = 0;
      cd[3 + k] = 1;
    } else if (t == JFREE || t == JBALL) {
      int kk = t == JFREE ? k - 3 : k;
      T ax[3] = {e.xmat[9 * b + kk], e.xmat[9 * b + kk + 3], e.xmat[9 * b + kk + 6]};
      cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
      cross3(cd + 3, ax, off);
    } else if (t == JSLIDE) {
      cd[0] = cd[1] = cd[2] = 0;
      cd[3] = e.xaxis[3 * j]; cd[4] = e.xaxis[3 * j + 1]; cd[5] = e.xaxis[3 * j + 2];
    } else {
      T ax[3] = {e.xaxis[3 * j], e.xaxis[3 * j + 1], e.xaxis[3 * j + 2]};
      cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
      cross3(cd + 3, ax, off);
    }
  }
  wsync();
  // composite inertia: lane b sums cinert over its subtree
  for (int b = l; b < m.nbody; b += 64) {
    if (b == 0) continue;
    T acc[10];
    for (int k = 0; k < 10; k++) acc[k] = 0;
    int end = m.body_subtree_end[b];
    for (int i = b; i < end; i++)
      for (int k = 0; k < 10; k++) acc[k] += e.cinert[10 * i + k];
    for (int k = 0; k < 10; k++) e.crb[10 * b + k] = acc[k];
  }
  wsync();
  // qM rows (tree-sparse, dof_Madr layout) and qMH = qM + h*diag(damping)
  for (int d = l; d < m.nv; d += 64) {
    T buf[6];
    mulinertvec(buf, e.crb + 10 * m.dof_bodyid[d], e.cdof + 6 * d);
    int adr = m.dof_Madr[d];
    int j = d;
    for (int t = 0; j >= 0; t++, j = m.dof_parentid[j]) {
      T v = dot6(e.cdof + 6 * j, buf);
      if (t == 0) v += m.dof_armature[d];
      e.qLD[adr + t] = v;
      e.qMH[adr + t] = t == 0 ? v + m.timestep * m.dof_damping[d] : v;
    }
  }
  wsync();
}

// mj_factorI on an LDS tree-sparse matrix: M = L' D L in place; returns diaginv in a register.
// Step k updates the (t, s) pairs of its ancestor block in parallel: lane -> t = (l & 15) + 1,
// s = s0 + (l >> 4), 4 values of s per pass; the ancestors' Madr come from the host table
// dof_ancadr, prefetched one step ahead.
// WIDE (nv > 64, mgx_wide.h): the pivot's Madr / chain length come from the model tables instead
// of the dof-lane registers (which only cover dofs 0..63); the returned diaginv is then unused.
template <typename T, bool WIDE = false>
__device__ __forceinline__ T factor_ld(const DevModel<T>& m, const Env<T>& e, T* LD) {
  int l = lane_id();
  const int t = (l & 15) + 1, sl = l >> 4;
  int ai_next = m.nv > 0 ? m.dof_ancadr[(m.nv - 1) * MGX_MAX_DEPTH + (t & 15)] : 0;
  for (int k = m.nv - 1; k >= 0; k--) {
    int akk = WIDE ? m.dof_Madr[k] : readlane(e.madr, k);
    int mk = (WIDE ? m.dof_chainlen[k] : readlane(e.chainlen, k)) - 1;  // number of ancestors
    int ai = ai_next;
    if (k > 0) ai_next = m.dof_ancadr[(k - 1) * MGX_MAX_DEPTH + (t & 15)];
    T dkk = LD[akk];
    if (dkk < minval<T>()) dkk = minval<T>();
    T tmp = t <= mk ? LD[akk + t] / dkk : (T)0;
    for (int s0 = 0; s0 < mk; s0 += 4) {
      int s = s0 + sl;
      if (t <= mk && s <= mk - t) LD[ai + s] -= LD[akk + t + s] * tmp;
    }
    T tmp_own = (l >= 1 && l <= mk) ? LD[akk + l] / dkk : (T)0;
    wsync();
    if (l >= 1 && l <= mk) LD[akk + l] = tmp_own;
    if (l == 0) LD[akk] = dkk;
    wsync();
  }
  return l < m.nv ? (T)1 / LD[e.madr] : (T)0;
}

// ---------------------------------------------------------------- row streaming helpers
// Row-major passes over B (lane = dof) load 8 rows at a time into registers before using any:
// with B in global scratch (Layout.gB) the loads would otherwise serialise behind the LDS row-
// scalar stores of the previous row (generic pointers may alias), one full memory latency each.
#define MGX_RB 8
template <typename T>
__device__ __forceinline__ void load_rows(T* x, const T* Bm, int Bs, int r0, int ne, int lc, bool dl) {
#pragma unroll
  for (int j = 0; j < MGX_RB; j++) x[j] = (r0 + j < ne && dl) ? Bm[(r0 + j) * Bs + lc] : (T)0;
}
// Prefetched row batches: the next MGX_RD batches' loads are in flight while one is reduced
// (a pass is otherwise one memory latency per batch; with B in global scratch, L2 misses).
// xn holds batches r0 + MGX_RB, ... r0 + MGX_RD MGX_RB; next_rows hands out batch r0 and
// issues r0 + (MGX_RD + 1) MGX_RB.
#define MGX_RD 2
#define MGX_HD 4  // Hessian passes: chunks of four rows in flight
// Batches r0, r0 + step, ... (step = MGX_RB, or MGX_RB * waves when a helper wave takes every
// other batch).
template <typename T>
__device__ __forceinline__ void first_rows(T (*xn)[MGX_RB], const T* Bm, int Bs, int ne, int lc, bool dl, int r0 = 0,
                                           int step = MGX_RB) {
#pragma unroll
  for (int d = 0; d < MGX_RD; d++) load_rows(xn[d], Bm, Bs, r0 + d * step, ne, lc, dl);
}
template <typename T>
__device__ __forceinline__ void next_rows(T* x, T (*xn)[MGX_RB], const T* Bm, int Bs, int r0, int ne, int lc, bool dl,
                                          int step = MGX_RB) {
#pragma unroll
  for (int j = 0; j < MGX_RB; j++) x[j] = xn[0][j];
#pragma unroll
  for (int d = 0; d + 1 < MGX_RD; d++)
#pragma unroll
    for (int j = 0; j < MGX_RB; j++) xn[d][j] = xn[d + 1][j];
  load_rows(xn[MGX_RD - 1], Bm, Bs, r0 + MGX_RD * step, ne, lc, dl);
}

// ---------------------------------------------------------------- helper waves
// The Newton kernels of assembly (narrow) and construction (mgx_wide.h) run two waves per env:
// wave 0 executes the step, wave 1 waits in a helper loop (team_helper_n / team_helper) and takes
// shares of the solver's row and tile passes. Every wsync() of wave 0 is a workgroup barrier the
// helper consumes; a section is: wave 0 posts the command in LDS -> barrier -> every wave runs its
// share (no barriers inside) -> barrier -> wave 0 clears the command. With one wave (nw = 1, every
// other kernel) the sections are plain wave barriers and wave 0 runs every share itself.
enum { TEAM_NONE = 0, TEAM_EXIT = 1, TEAM_HESS, TEAM_PANEL, TEAM_TRAIL, TEAM_JP, TEAM_GRAD, TEAM_XFORM, TEAM_SETUP,
       TEAM_FORCE, TEAM_CONTACT };

template <typename T>
__device__ __forceinline__ void team_begin(Env<T>& e, int cmd, int arg, int arg2 = 0) {
  if (e.nw > 1 && lane_id() == 0) { e.ctl[0] = cmd; e.ctl[1] = arg; e.ctl[2] = arg2; }
  wsync();
}
template <typename T>
__device__ __forceinline__ void team_end(Env<T>& e) {
  wsync();
  if (e.nw > 1 && lane_id() == 0) e.ctl[0] = TEAM_NONE;
}
// wave 0, before its first wsync: the helper reads the command word after every barrier
template <typename T>
__device__ __forceinline__ void team_init(Env<T>& e) {
  if (e.nw > 1 && lane_id() == 0) e.ctl[0] = TEAM_NONE;
}
// wave 0, at the end of the kernel (every path): releases the helper
template <typename T>
__device__ __forceinline__ void team_exit(Env<T>& e) {
  if (e.nw > 1) {
    if (lane_id() == 0) e.ctl[0] = TEAM_EXIT;
    wsync();
  }
}

template <typename T>
__device__ __forceinline__ T usum(T x) { return wave_sum_fast(x); }  // DPP, uniform result

// B_r = D^-1/2 L'^-1 J_r' for one row x (LDS, lane-private): for k = nv-1 .. 0 the ancestors
// of k get x[anc] -= L[k][anc] x[k]. The ancestors of one k are distinct, so all their loads
// are issued before any store (one LDS latency per k instead of one per ancestor).
template <typename T, bool WIDE = false>
__device__ __forceinline__ void transform_row(const DevModel<T>& m, const Env<T>& e, T* x, const T* dinv_sqrt) {
  for (int k = m.nv - 1; k >= 0; k--) {
    const int* ak = m.dof_anc + k * MGX_MAX_DEPTH;
    int mk = (WIDE ? m.dof_chainlen[k] : readlane(e.chainlen, k)) - 1;
    int a = (WIDE ? m.dof_Madr[k] : readlane(e.madr, k)) + 1;
    T xk = x[k];
    T xa[MGX_MAX_DEPTH], la[MGX_MAX_DEPTH];
#pragma unroll
    for (int t = 1; t < MGX_MAX_DEPTH; t++)
      if (t <= mk) { xa[t] = x[ak[t]]; la[t] = e.qLD[a + t - 1]; }
#pragma unroll
    for (int t = 1; t < MGX_MAX_DEPTH; t++)
      if (t <= mk) x[ak[t]] = xa[t] - la[t] * xk;
    x[k] = xk * dinv_sqrt[k];
  }
}

// x <- L'^-1 x (lane-distributed vector)
template <typename T>
__device__ __forceinline__ T solve_LT(const DevModel<T>& m, const Env<T>& e, const T* LD, T x) {
  int l = lane_id();
  for (int k = m.nv - 1; k >= 0; k--) {
    T xk = readlane(x, k);
    uint64_t am = readlane_u64(e.ancmask, k);
    int base = readlane(e.madr, k) + readlane(e.chainlen, k);
    if (l < m.nv && ((am >> l) & 1ull)) x -= LD[base - e.chainlen] * xk;
  }
  return x;
}
// x <- L^-1 x
template <typename T>
__device__ __forceinline__ T solve_L(const DevModel<T>& m, const Env<T>& e, const T* LD, T x) {
  int l = lane_id();
  const int base = e.madr + e.chainlen;
  for (int i = 0; i < m.nv; i++) {
    T xi = readlane(x, i);
    int ci = readlane(e.chainlen, i);
    if (l < m.nv && ((e.ancmask >> i) & 1ull)) x -= LD[base - ci] * xi;
  }
  return x;
}
// y = L x
template <typename T>
__device__ __forceinline__ T mul_L(const DevModel<T>& m, const Env<T>& e, const T* LD, T x) {
  int l = lane_id();
  const int base = e.madr + e.chainlen;
  T y = x;
  for (int i = 0; i < m.nv; i++) {
    T xi = readlane(x, i);
    int ci = readlane(e.chainlen, i);
    if (l < m.nv && ((e.ancmask >> i) & 1ull)) y += LD[base - ci] * xi;
  }
  return y;
}
// y = L' u
template <typename T>
__device__ __forceinline__ T mul_LT(const DevModel<T>& m, const Env<T>& e, const T* LD, T u) {
  int l = lane_id();
  T y = u;
  for (int k = 0; k < m.nv; k++) {
    T uk = readlane(u, k);
    uint64_t am = readlane_u64(e.ancmask, k);
    int base = readlane(e.madr, k) + readlane(e.chainlen, k);
    if (l < m.nv && ((am >> l) & 1ull)) y += LD[base - e.chainlen] * uk;
  }
  return y;
}
// x = M^-1 y
template <typename T>
__device__ __forceinline__ T solve_M(const DevModel<T>& m, const Env<T>& e, const T* LD, T diaginv, T y) {
  T x = solve_LT(m, e, LD, y);
  x *= diaginv;
  return solve_L(m, e, LD, x);
}

// ---------------------------------------------------------------- collision (mj_collision)
template <typename T>
__device__ __forceinline__ void collision(const DevModel<T>& m, Env<T>& e) {
  int l = lane_id();
  const Layout& L = m.L;
  // broadphase: bounding spheres (planes: the half-space test); compact survivors in pair order.
  // Each round reads its 64 pairs' records (DevModel.pair_bpi / pair_bpr) with the next round's
  // already in flight, so only the LDS pose reads depend on a load.
  int nact = 0;
  const int4* bpi = reinterpret_cast<const int4*>(m.pair_bpi);
  int4 nr = l < m.npair ? bpi[l] : make_int4(0, 0, -1, 0);
  T nreach = 0, nmargin = 0, nrbo = 0;
  if (l < m.npair) { nreach = m.pair_bpr[4 * l]; nmargin = m.pair_bpr[4 * l + 1]; nrbo = m.pair_bpr[4 * l + 2]; }
  for (int base = 0; base < m.npair; base += 64) {
    const int4 r = nr;
    const T reach = nreach, margin = nmargin, rbo = nrbo;
    const int pn = base + 64 + l;
    if (pn < m.npair) {
      nr = bpi[pn];
      nreach = m.pair_bpr[4 * pn]; nmargin = m.pair_bpr[4 * pn + 1]; nrbo = m.pair_bpr[4 * pn + 2];
    } else {
      nr = make_int4(0, 0, -1, 0);
    }
    const int p = base + l;
    bool act = false;
    if (r.z >= 0) {
      const int g1 = r.x, g2 = r.y;
      if (r.z & 1) {
        const T* pm = e.geom_xmat + 9 * g1;
        T n[3] = {pm[2], pm[5], pm[8]};
        T rel[3] = {e.geom_xpos[3 * g2] - e.geom_xpos[3 * g1], e.geom_xpos[3 * g2 + 1] - e.geom_xpos[3 * g1 + 1],
                    e.geom_xpos[3 * g2 + 2] - e.geom_xpos[3 * g1 + 2]};
        act = dot3(rel, n) <= reach;
      } else {
        T dv[3] = {e.geom_xpos[3 * g2] - e.geom_xpos[3 * g1], e.geom_xpos[3 * g2 + 1] - e.geom_xpos[3 * g1 + 1],
                   e.geom_xpos[3 * g2 + 2] - e.geom_xpos[3 * g1 + 2]};
        act = sqrt(dot3(dv, dv)) <= reach;
        // many-pair scenes (bipedal 3,185 candidate pairs, assembly 803, construction 1,202, soccer
        // 251): a pair that passes the bounding spheres must also pass a bounding-box test — the
        // two geoms' boxes (box, capsule, cylinder: DevModel.geom_obb) not separated along their
        // face axes, or a sphere within the margin of the other geom's box — so far fewer pairs
        // reach the divergent narrowphase; conservative, the contact list is unchanged
        if (act && L.tight_bp && (r.z & 14)) {
          const T tol = sizeof(T) == 8 ? (T)1e-9 : (T)1e-4;
          if (r.z & 2) {
            act = !box_box_separated(e.geom_xpos + 3 * g1, e.geom_xmat + 9 * g1, m.geom_obb + 3 * g1,
                                     e.geom_xpos + 3 * g2, e.geom_xmat + 9 * g2, m.geom_obb + 3 * g2, margin, tol);
          } else {
            const int gs = (r.z & 4) ? g1 : g2, gb = (r.z & 4) ? g2 : g1;
            act = !sphere_box_separated(e.geom_xpos + 3 * gs, rbo, e.geom_xpos + 3 * gb, e.geom_xmat + 9 * gb,
                                        m.geom_obb + 3 * gb, margin, tol);
          }
        }
      }
    }
    unsigned long long mask = ballot(act);
    int pos = nact + prefix_count(mask);
    if (act && pos < L.max_active) e.act_list[pos] = p;
    nact += popc64(mask);
  }
  if (nact > L.max_active) { nact = L.max_active; e.overflow |= 1; }
  wsync();
  // narrowphase: one active pair per lane, compaction by exclusive scan keeps pair order
  int ncon = 0;
  for (int base = 0; base < nact; base += 64) {
    int a = base + l;
    Con<T> rc[MGX_MAX_CONPAIR];
    int n = 0, p = -1;
    if (a < nact) {
      p = e.act_list[a];
      int g1 = m.pair_geom[2 * p], g2 = m.pair_geom[2 * p + 1];
      n = collide_pair(m.geom_type[g1], m.geom_type[g2], e.geom_xpos + 3 * g1, e.geom_xmat + 9 * g1,
                       m.geom_size + 3 * g1, e.geom_xpos + 3 * g2, e.geom_xmat + 9 * g2, m.geom_size + 3 * g2,
                       m.pair_margin[p], rc);
    }
    int total;
    int off = wave_excl_scan(n, &total);
    for (int c = 0; c < n; c++) {
      int k = ncon + off + c;
      if (k >= L.max_ncon) break;
      e.con_dist[k] = rc[c].dist;
      for (int q = 0; q < 3; q++) { e.con_pos[3 * k + q] = rc[c].pos[q]; e.con_frame[L.cfs * k + q] = rc[c].n[q]; }
      if (L.cfs == 9) make_frame(e.con_frame + 9 * k);  // else the normal only (Layout.cfs)
      e.con_pair[k] = p;
      e.con_mu[k] = sqrt(m.pair_friction[5 * p] * m.pair_friction[5 * p] + m.pair_friction[5 * p + 1] * m.pair_friction[5 * p + 1]);
      e.con_geom[2 * k] = m.pair_geom[2 * p];
      e.con_geom[2 * k + 1] = m.pair_geom[2 * p + 1];
    }
    ncon += total;
  }
  if (ncon > L.max_ncon) { ncon = L.max_ncon; e.overflow |= 2; }
  e.ncon = __builtin_amdgcn_readfirstlane(ncon);
  wsync();
}

// ---------------------------------------------------------------- constraints
template <typename T>
__device__ __forceinline__ bool body_has_dof(const DevModel<T>& m, int b, int d) {
  return (m.body_dofmask[b * m.nmaskword + (d >> 5)] >> (d & 31)) & 1u;
}

// dofs moving body b (its chain), nv <= 64
template <typename T>
__device__ __forceinline__ uint64_t body_mask64(const DevModel<T>& m, int b) {
  uint64_t lo = m.body_dofmask[b * m.nmaskword];
  uint64_t hi = m.nmaskword > 1 ? m.body_dofmask[b * m.nmaskword + 1] : 0u;
  return lo | (hi << 32);
}

template <typename T>
__device__ __forceinline__ T impedance(const T* solimp, T pos, T margin) {
  T d0 = clampv(solimp[0], (T)0.0001, (T)0.9999), d1 = clampv(solimp[1], (T)0.0001, (T)0.9999);
  T width = solimp[2], mid = solimp[3], power = solimp[4];
  if (d0 == d1 || width <= minval<T>()) return (T)0.5 * (d0 + d1);
  T x = (pos - margin) / width;
  if (x < 0) x = -x;
  if (x >= 1 || x <= 0) return x >= 1 ? d1 : d0;
  T y;
  if (power == 1) y = x;
  else if (x <= mid) y = pow(x, power) / pow(mid, power - 1);
  else y = 1 - pow(1 - x, power) / pow(1 - mid, power - 1);
  return d0 + y * (d1 - d0);
}

// The rows of contact c from row r0 (lane = dof): J_n +- mu_k J_k, then the rows' type / id /
// pos / margin / diagApprox (lane = row)
template <typename T>
__device__ __forceinline__ void contact_rows(const DevModel<T>& m, Env<T>& e, int c, int r0) {
  const int l = lane_id();
  int p = e.con_pair[c];
  int dim = m.pair_condim[p];
  int nrow = dim == 1 ? 1 : 2 * (dim - 1);
  int g1 = e.con_geom[2 * c], g2 = e.con_geom[2 * c + 1];
  int b1 = m.geom_bodyid[g1], b2 = m.geom_bodyid[g2];
  const T* fr = e.con_frame + 9 * c;
  const T* pos = e.con_pos + 3 * c;
  for (int d = l; d < m.nv; d += 64) {  // lane = dof (l, l + 64 when nv > 64)
    T j1[3] = {0, 0, 0}, j2[3] = {0, 0, 0};
    const T* cd = e.cdof + 6 * d;
    if (b2 > 0 && body_has_dof(m, b2, d)) {
      int r2 = m.body_rootid[b2];
      T off[3] = {pos[0] - e.subtree_com[3 * r2], pos[1] - e.subtree_com[3 * r2 + 1], pos[2] - e.subtree_com[3 * r2 + 2]}, t[3];
      cross3(t, cd, off);
      j2[0] = cd[3] + t[0]; j2[1] = cd[4] + t[1]; j2[2] = cd[5] + t[2];
    }
    if (b1 > 0 && body_has_dof(m, b1, d)) {
      int r1 = m.body_rootid[b1];
      T off[3] = {pos[0] - e.subtree_com[3 * r1], pos[1] - e.subtree_com[3 * r1 + 1], pos[2] - e.subtree_com[3 * r1 + 2]}, t[3];
      cross3(t, cd, off);
      j1[0] = cd[3] + t[0]; j1[1] = cd[4] + t[1]; j1[2] = cd[5] + t[2];
    }
    T jd[3] = {j2[0] - j1[0], j2[1] - j1[1], j2[2] - j1[2]};
    T cj0 = fr[0] * jd[0] + fr[1] * jd[1] + fr[2] * jd[2];
    if (dim == 1) {
      e.Bm[r0 * e.Bs + d] = cj0;
    } else {
      T cj[6];
      cj[1] = fr[3] * jd[0] + fr[4] * jd[1] + fr[5] * jd[2];
      cj[2] = fr[6] * jd[0] + fr[7] * jd[1] + fr[8] * jd[2];
      if (dim > 3) {
        // relative angular motion: the rotational parts of the dof's motion subspace
        T jr[3] = {0, 0, 0};
        if (b2 > 0 && body_has_dof(m, b2, d)) { jr[0] += cd[0]; jr[1] += cd[1]; jr[2] += cd[2]; }
        if (b1 > 0 && body_has_dof(m, b1, d)) { jr[0] -= cd[0]; jr[1] -= cd[1]; jr[2] -= cd[2]; }
        cj[3] = fr[0] * jr[0] + fr[1] * jr[1] + fr[2] * jr[2];
        cj[4] = fr[3] * jr[0] + fr[4] * jr[1] + fr[5] * jr[2];
        cj[5] = fr[6] * jr[0] + fr[7] * jr[1] + fr[8] * jr[2];
      }
      for (int k = 1; k < dim; k++) {
        T mu = m.pair_friction[5 * p + k - 1];
        e.Bm[(r0 + 2 * (k - 1)) * e.Bs + d] = cj0 + mu * cj[k];
        e.Bm[(r0 + 2 * (k - 1) + 1) * e.Bs + d] = cj0 - mu * cj[k];
      }
    }
  }
  if (l < nrow) {
    int r = r0 + l;
    T tran = m.body_invweight0[2 * b1] + m.body_invweight0[2 * b2];
    T rot = m.body_invweight0[2 * b1 + 1] + m.body_invweight0[2 * b2 + 1];
    T f = dim == 1 ? (T)0 : m.pair_friction[5 * p + (l >> 1)];
    e.efc_type[r] = dim == 1 ? C_CONTACT_FRICTIONLESS : C_CONTACT_PYRAMIDAL;
    e.efc_id[r] = c;
    e.efc[8 * r + 7] = e.con_dist[c];
    e.efc_margin[r] = m.pair_margin[p] - m.pair_gap[p];
    e.efc[8 * r + 2] = tran + f * f * ((l >> 1) < 2 ? tran : rot);  // mj_diagApprox [ext]
  }
}

// The contacts' rows over contacts w0, w0 + ws, ... (a helper wave takes every other contact):
// each contact's first row from a wave scan of the row counts, and the rows end at the first
// contact that does not fit (the serial loop's break). Returns the row count after the contacts
// (every wave computes the same) and flags an overflow.
template <typename T>
__device__ __forceinline__ int contact_rows_share(const DevModel<T>& m, Env<T>& e, int ncon, int nefc0, int w0, int ws,
                                                  bool& ovf) {
  const int l = lane_id();
  int total = nefc0;
  ovf = false;
  for (int cb = 0; cb < ncon; cb += 64) {
    const int c = cb + l;
    int nr = 0;
    if (c < ncon) {
      const int dim = m.pair_condim[e.con_pair[c]];
      nr = dim == 1 ? 1 : 2 * (dim - 1);
    }
    int bt;
    const int off = wave_excl_scan(nr, &bt);
    const int nb = ncon - cb < 64 ? ncon - cb : 64;
    const uint64_t valid = nb == 64 ? ~0ull : ((1ull << nb) - 1ull);
    const uint64_t fit = ballot(c < ncon && total + off + nr <= m.L.max_nefc);
    const uint64_t bad = valid & ~fit;
    const int kend = bad ? __builtin_ctzll(bad) : nb;
    for (int k = w0; k < kend; k += ws) contact_rows(m, e, cb + k, total + readlane(off, k));
    if (kend < nb) {
      ovf = true;
      total += readlane(off, kend);
      break;
    }
    total += bt;
  }
  return total;
}

// joint limits then pyramidal contacts; rows are written as J and transformed in place
template <typename T>
__device__ __forceinline__ void make_constraint(const DevModel<T>& m, Env<T>& e) {
  int l = lane_id();
  const Layout& L = m.L;
  int nefc = 0;
  // ---- joint limits (lane per joint), order (joint, lower, upper)
  for (int base = 0; base < m.njnt; base += 64) {
    int j = base + l;
    int cnt = 0;
    T dl = 0, du = 0;
    bool lo = false, hi = false;
    if (j < m.njnt && m.jnt_limited[j] && (m.jnt_type[j] == JHINGE || m.jnt_type[j] == JSLIDE)) {
      T val = e.qpos[m.jnt_qposadr[j]], margin = m.jnt_margin[j];
      dl = val - m.jnt_range[2 * j];
      du = m.jnt_range[2 * j + 1] - val;
      lo = dl < margin;
      hi = du < margin;
      cnt = (int)lo + (int)hi;
    }
    int total;
    int off = wave_excl_scan(cnt, &total);
    int r = nefc + off;
    for (int side = 0; side < 2; side++) {
      bool on = side == 0 ? lo : hi;
      if (!on) continue;
      if (r < L.max_nefc) {
        e.efc_type[r] = C_LIMIT_JOINT; e.efc_id[r] = j;
        e.efc[8 * r + 7] = side == 0 ? dl : du;
        e.efc_margin[r] = m.jnt_margin[j];
        e.efc[8 * r + 2] = m.dof_invweight0[m.jnt_dofadr[j]];
        e.efc[8 * r + 1] = side == 0 ? (T)1 : (T)-1;  // J entry, scattered below
      }
      r++;
    }
    nefc += total;
  }
  if (nefc > L.max_nefc) { nefc = L.max_nefc; e.overflow |= 4; }
  wsync();
  // zero-fill + set the single nonzero of each limit row (lane per row)
  for (int r = l; r < nefc; r += 64) {
    T* row = e.Bm + r * e.Bs;
    for (int k = 0; k < m.nv; k++) row[k] = 0;
    row[m.jnt_dofadr[e.efc_id[r]]] = e.efc[8 * r + 1];
  }
  // ---- contacts: 2*(condim-1) pyramid rows (condim 3, 4, 6) or 1 row (condim 1); lane = dof.
  // Edge k (k = 1 .. condim-1) is J_n +- mu_k J_k with J_1, J_2 the sliding directions
  // (translational Jacobian on the tangents), J_3 torsion (rotational on the normal), J_4, J_5
  // rolling (rotational on the tangents), in MuJoCo's order [ext]
  {
    bool ovf;
    team_begin(e, TEAM_CONTACT, e.ncon, nefc);
    nefc = contact_rows_share(m, e, e.ncon, nefc, 0, e.nw, ovf);
    team_end(e);
    if (ovf) e.overflow |= 4;
  }
  e.nefc = __builtin_amdgcn_readfirstlane(nefc);
  wsync();
  // impedance, K, B, R per row (lane per row)
  for (int r = l; r < nefc; r += 64) {
    const T *solref, *solimp;
    if (e.efc_type[r] == C_LIMIT_JOINT) {
      solref = m.jnt_solref + 2 * e.efc_id[r];
      solimp = m.jnt_solimp + 5 * e.efc_id[r];
    } else {
      int p = e.con_pair[e.efc_id[r]];
      solref = m.pair_solref + 2 * p;
      solimp = m.pair_solimp + 5 * p;
    }
    T pos = e.efc[8 * r + 7];
    T imp = impedance(solimp, pos, e.efc_margin[r]);
    T dmax = clampv(solimp[1], (T)0.0001, (T)0.9999), K, B;
    if (solref[0] > 0) {
      T tc = solref[0], dr = solref[1];
      if (tc < 2 * m.timestep) tc = 2 * m.timestep;
      K = (T)1 / (dmax * dmax * tc * tc * dr * dr);
      B = (T)2 / (dmax * tc);
    } else {
      K = -solref[0] / (dmax * dmax);
      B = -solref[1] / dmax;
    }
    T R = ((T)1 - imp) * e.efc[8 * r + 2] / imp;
    e.efc[8 * r + 6] = B;
    e.efc[8 * r + 5] = K * imp * (pos - e.efc_margin[r]);
    e.efc[8 * r + 2] = R > minval<T>() ? R : minval<T>();
  }
  wsync();
}

#ifndef MGX_TRANSFORM_LANE_ROW
#define MGX_TRANSFORM_LANE_ROW 0  // 1: the lane-per-row transform for narrow models too (A/B builds)
#endif
// B_r = D^-1/2 L'^-1 J_r' in place (lane per row), sqrtdi in vec0. Rows in global scratch
// (Layout.gB) are staged through LDS in chunks of L.tchunk rows (the phase-A union is dead once
// the rows exist): coalesced row copies in and out (lane = dof), the lane-per-row transform on
// LDS, instead of lane-strided global read-modify-writes along every row.
//
// Narrow models (nv <= 64) instead go four rows at a time, row-major (lane = dof): the rows are
// loaded coalesced (the next four in flight), and L'^-1 runs as a readlane sweep over the
// rows' dof support only — highest dof first, each dof's ancestors joining the support as it is
// reached — with x_anc -= L[k][anc] x_k as one FMA per row per step (the same operations in the
// same order as transform_row), then the D^-1/2 scale and one coalesced store per row. A
// contact row's support is two body chains (~10-20 of nv dofs), so a block costs tens of
// steps, where the lane-per-row walk visits all nv dofs of every row.
// Chunks of four rows c0, c0 + cs, ... (a helper wave takes every other chunk); the caller
// synchronises.
template <typename T>
__device__ __forceinline__ void transform_rows_rm(const DevModel<T>& m, Env<T>& e, int ne, int c0, int cs) {
  const int l = lane_id(), nv = m.nv;
  const bool dl = l < nv;
  const int lc = dl ? l : 0;
  T* Bm = e.Bm;
  const int Bs = e.Bs;
  const T dinvs = dl ? e.vec0[l] : (T)0;
  auto ld4 = [&](int r0, T& a, T& b, T& c, T& d) {
    a = (dl && r0 < ne) ? Bm[r0 * Bs + lc] : (T)0;
    b = (dl && r0 + 1 < ne) ? Bm[(r0 + 1) * Bs + lc] : (T)0;
    c = (dl && r0 + 2 < ne) ? Bm[(r0 + 2) * Bs + lc] : (T)0;
    d = (dl && r0 + 3 < ne) ? Bm[(r0 + 3) * Bs + lc] : (T)0;
  };
  T n0, n1, n2, n3;
  ld4(4 * c0, n0, n1, n2, n3);
  for (int r0 = 4 * c0; r0 < ne; r0 += 4 * cs) {
    T x0 = n0, x1 = n1, x2 = n2, x3 = n3;
    if (r0 + 4 * cs < ne) ld4(r0 + 4 * cs, n0, n1, n2, n3);
    uint64_t sp = ballot(x0 != (T)0 || x1 != (T)0 || x2 != (T)0 || x3 != (T)0);
    while (sp) {
      const int k = 63 - __clzll(sp);
      const uint64_t am = readlane_u64(e.ancmask, k);
      sp = (sp & ~(1ull << k)) | am;  // ancestors have lower indices: visited later in the sweep
      const int base = readlane(e.madr, k) + readlane(e.chainlen, k) - e.chainlen;
      const T coef = (dl && ((am >> l) & 1ull)) ? e.qLD[base > 0 ? base : 0] : (T)0;
      const T k0 = readlane(x0, k), k1 = readlane(x1, k), k2 = readlane(x2, k), k3 = readlane(x3, k);
      x0 -= coef * k0; x1 -= coef * k1; x2 -= coef * k2; x3 -= coef * k3;
    }
    if (dl) {
      if (r0 < ne) Bm[r0 * Bs + l] = x0 * dinvs;
      if (r0 + 1 < ne) Bm[(r0 + 1) * Bs + l] = x1 * dinvs;
      if (r0 + 2 < ne) Bm[(r0 + 2) * Bs + l] = x2 * dinvs;
      if (r0 + 3 < ne) Bm[(r0 + 3) * Bs + l] = x3 * dinvs;
    }
  }
}

template <typename T, bool WIDE = false>
__device__ __forceinline__ void transform_rows(const DevModel<T>& m, Env<T>& e) {
  int l = lane_id();
  if constexpr (!WIDE) {
    if (!(MGX_TRANSFORM_LANE_ROW)) {
      // four-row chunks, every other one on the helper wave when there is one
      const int ne = __builtin_amdgcn_readfirstlane(e.nefc);
      team_begin(e, TEAM_XFORM, ne);
      transform_rows_rm(m, e, ne, 0, e.nw);
      team_end(e);
      return;
    }
  }
  const int ne = __builtin_amdgcn_readfirstlane(e.nefc);
  const int C = m.L.tchunk;
  if (m.L.gB && C > 0) {
    T* S = e.xmat;  // start of the union region
    const int Bs = e.Bs, nv = m.nv;
    for (int r0 = 0; r0 < ne; r0 += C) {
      const int nr = ne - r0 < C ? ne - r0 : C;
      T* G = e.Bm + (size_t)r0 * Bs;
      for (int d0 = 0; d0 < (WIDE ? nv : 1); d0 += 64) {
        const int d = d0 + l;
        for (int q0 = 0; q0 < nr; q0 += MGX_RB) {
          T xb[MGX_RB];
          load_rows(xb, G, Bs, q0, nr, d < nv ? d : 0, d < nv);
#pragma unroll
          for (int j = 0; j < MGX_RB; j++)
            if (q0 + j < nr && d < nv) S[(q0 + j) * Bs + d] = xb[j];
        }
      }
      wsync();
      if (l < nr) transform_row<T, WIDE>(m, e, S + l * Bs, e.vec0);
      wsync();
      for (int d = l; d < nv; d += 64)
        for (int r = 0; r < nr; r++) G[r * Bs + d] = S[r * Bs + d];
      wsync();
    }
    return;
  }
  for (int r = l; r < ne; r += 64) transform_row<T, WIDE>(m, e, e.Bm + r * e.Bs, e.vec0);
  wsync();
}

// qfrc_smooth of dof d before the register store: passive (damping, springs) - bias (RNE,
// subtree sums in crb storage) + applied + actuation + J(xipos)' xfrc_applied; qfrc_applied comes
// from the dof's register (applied, passed by the caller)
template <typename T>
__device__ __forceinline__ T dof_force_applied(const DevModel<T>& m, const Env<T>& e, int d, T applied) {
  int b = m.dof_bodyid[d];
  T bias = dot6(e.cdof + 6 * d, e.crb + 10 * b);
  T passive = -m.dof_damping[d] * e.qvel[d];
  int j = m.dof_jntid[d];
  T st = m.jnt_stiffness[j];
  if (st != 0) {
    int t = m.jnt_type[j], a = m.jnt_qposadr[j], k = d - m.jnt_dofadr[j];
    if (t == JHINGE || t == JSLIDE) passive -= st * (e.qpos[a] - m.qpos_spring[a]);
    else if (t == JFREE && k < 3) passive -= st * (e.qpos[a + k] - m.qpos_spring[a + k]);
  }
  T act = 0;
  for (int u = 0; u < m.nu; u++)
    if (m.jnt_dofadr[m.actuator_trnid[u]] == d) act += m.actuator_gear[u] * e.act_force[u];
  // xfrc_applied: J(xipos)' f for every body with a nonzero wrench whose chain holds this dof
  T xf = 0;
  for (int i = 1; i < m.nbody; i++) {
    const T* f = e.xfrc + 6 * i;
    if (f[0] == 0 && f[1] == 0 && f[2] == 0 && f[3] == 0 && f[4] == 0 && f[5] == 0) continue;
    if (!body_has_dof(m, i, d)) continue;
    int r = m.body_rootid[i];
    const T* cd = e.cdof + 6 * d;
    T off[3] = {e.xipos[3 * i] - e.subtree_com[3 * r], e.xipos[3 * i + 1] - e.subtree_com[3 * r + 1],
                e.xipos[3 * i + 2] - e.subtree_com[3 * r + 2]}, t[3];
    cross3(t, cd, off);
    xf += (cd[3] + t[0]) * f[0] + (cd[4] + t[1]) * f[1] + (cd[5] + t[2]) * f[2] + cd[0] * f[3] + cd[1] * f[4] + cd[2] * f[5];
  }
  return passive - bias + applied + act + xf;
}
template <typename T>
__device__ __forceinline__ T dof_force(const DevModel<T>& m, const Env<T>& e, int d) {
  return dof_force_applied(m, e, d, e.qfrc_applied);
}

// ---------------------------------------------------------------- velocity stage
// comVel, actuator forces, RNE and its subtree sums (everything but the per-dof forces)
template <typename T>
__device__ __forceinline__ void velocity_bodies(const DevModel<T>& m, Env<T>& e) {
  int l = lane_id();
  // comVel: lane b walks its chain; cdof_dot for the body's own dofs
  for (int b = l; b < m.nbody; b += 64) {
    T cvel[6] = {0, 0, 0, 0, 0, 0};
    int depth = m.body_depth[b];
    for (int c = 0; c < depth; c++) {
      int i = m.body_chain[b * MGX_MAX_DEPTH + c];
      int bda = m.body_dofadr[i], nd = m.body_dofnum[i];
      bool own = i == b;
      for (int j = 0; j < nd; j++) {
        int dof = bda + j;
        int t = m.jnt_type[m.dof_jntid[dof]];
        if (t == JFREE) {
          if (own) for (int q = 0; q < 18; q++) e.cdof_dot[6 * dof + q] = 0;
          for (int q = 0; q < 3; q++)
            for (int k = 0; k < 6; k++) cvel[k] += e.cdof[6 * (dof + q) + k] * e.qvel[dof + q];
          if (own) for (int q = 3; q < 6; q++) crossmotion(e.cdof_dot + 6 * (dof + q), cvel, e.cdof + 6 * (dof + q));
          for (int q = 3; q < 6; q++)
            for (int k = 0; k < 6; k++) cvel[k] += e.cdof[6 * (dof + q) + k] * e.qvel[dof + q];
          j += 5;
        } else if (t == JBALL) {
          if (own) for (int q = 0; q < 3; q++) crossmotion(e.cdof_dot + 6 * (dof + q), cvel, e.cdof + 6 * (dof + q));
          for (int q = 0; q < 3; q++)
            for (int k = 0; k < 6; k++) cvel[k] += e.cdof[6 * (dof + q) + k] * e.qvel[dof + q];
          j += 2;
        } else {
          if (own) crossmotion(e.cdof_dot + 6 * dof, cvel, e.cdof + 6 * dof);
          for (int k = 0; k < 6; k++) cvel[k] += e.cdof[6 * dof + k] * e.qvel[dof];
        }
      }
    }
    for (int k = 0; k < 6; k++) e.cvel[6 * b + k] = cvel[k];
  }
  // actuator forces (lane per actuator)
  for (int u = l; u < m.nu; u += 64) {
    int j = m.actuator_trnid[u];
    T ctrl = e.ctrl[u];
    if (m.actuator_ctrllimited[u]) ctrl = clampv(ctrl, m.actuator_ctrlrange[2 * u], m.actuator_ctrlrange[2 * u + 1]);
    T g = m.actuator_gear[u];
    T len = g * e.qpos[m.jnt_qposadr[j]], vel = g * e.qvel[m.jnt_dofadr[j]];
    const T* gp = m.actuator_gainprm + 3 * u;
    const T* bp = m.actuator_biasprm + 3 * u;
    T f = gp[0] * ctrl + bp[0] + bp[1] * len + bp[2] * vel;
    if (m.actuator_forcelimited[u]) f = clampv(f, m.actuator_forcerange[2 * u], m.actuator_forcerange[2 * u + 1]);
    e.act_force[u] = f;
  }
  wsync();
  // RNE forward: cacc by chain walk, cfrc_body
  for (int b = l; b < m.nbody; b += 64) {
    if (b == 0) { for (int k = 0; k < 6; k++) e.cfrc[k] = 0; continue; }
    T cacc[6] = {0, 0, 0, -m.gravity[0], -m.gravity[1], -m.gravity[2]};
    int depth = m.body_depth[b];
    for (int c = 0; c < depth; c++) {
      int i = m.body_chain[b * MGX_MAX_DEPTH + c];
      int bda = m.body_dofadr[i], nd = m.body_dofnum[i];
      for (int j = 0; j < nd; j++)
        for (int k = 0; k < 6; k++) cacc[k] += e.cdof_dot[6 * (bda + j) + k] * e.qvel[bda + j];
    }
    T f[6], tmp[6], tmp1[6];
    mulinertvec(f, e.cinert + 10 * b, cacc);
    mulinertvec(tmp, e.cinert + 10 * b, e.cvel + 6 * b);
    crossforce(tmp1, e.cvel + 6 * b, tmp);
    for (int k = 0; k < 6; k++) e.cfrc[6 * b + k] = f[k] + tmp1[k];
  }
  wsync();
  // subtree sums of cfrc into crb storage (cfrc_total), lane per body
  for (int b = l; b < m.nbody; b += 64) {
    T acc[6] = {0, 0, 0, 0, 0, 0};
    if (b > 0) {
      int end = m.body_subtree_end[b];
      for (int i = b; i < end; i++)
        for (int k = 0; k < 6; k++) acc[k] += e.cfrc[6 * i + k];
    }
    for (int k = 0; k < 6; k++) e.crb[10 * b + k] = acc[k];  // crb no longer needed
  }
  wsync();
}

template <typename T>
__device__ __forceinline__ void velocity(const DevModel<T>& m, Env<T>& e) {
  velocity_bodies(m, e);
  // per-dof forces
  const int l = lane_id();
  e.qfrc_smooth = l < m.nv ? dof_force(m, e, l) : (T)0;
}

// ---------------------------------------------------------------- constraint solver (PGS)
// mj_fwdConstraint + mj_solPGS [ext]. Rows are swept in order (Gauss-Seidel, MuJoCo's order);
// per row: one LDS read of B_r (lane = dof), one wave reduction for B_r.v, scalar update,
// v += delta * B_r. Row scalars live in LDS and the next row is prefetched while the current
// reduction runs; 1/AR_rr is precomputed so the sweep has no division.
template <typename T>
__device__ __forceinline__ void pgs(const DevModel<T>& m, Env<T>& e) {
  int l = lane_id();
  const int ne = __builtin_amdgcn_readfirstlane(e.nefc);  // uniform: keeps the sweep a scalar loop
  const int nv = m.nv;
  const bool dl = l < nv;
  T sqrtD = dl ? sqrt(e.qLD[m.dof_Madr[l]]) : (T)0;
  if (ne == 0) {
    e.qacc = e.qacc_smooth;
    e.qfrc_constraint = 0;
    e.niter = 0;
    return;
  }
  // w vectors: D^1/2 L x for qvel, qacc_smooth, qacc_warmstart (lane = dof)
  T qv = dl ? e.qvel[l] : (T)0;
  const T wv = sqrtD * mul_L(m, e, e.qLD, qv);
  const T ws = sqrtD * mul_L(m, e, e.qLD, e.qacc_smooth);
  const T ww = dl ? sqrtD * mul_L(m, e, e.qLD, e.qacc_ws) : (T)0;
  T* efc = e.efc;
  const T* Bm = e.Bm;
  const int Bs = e.Bs;
  const int lc = dl ? l : 0;  // clamped column: every lane reads a valid address
  // per row (row-major, 8 rows per batch, wave reductions; lane 0 stores the scalars):
  // efc_vel -> aref (mj_referenceConstraint), b = J qacc_smooth - aref, warmstart force from
  // qacc_warmstart (mj_constraintUpdate), 1/AR_rr and AR_rr
  for (int r0 = 0; r0 < ne; r0 += MGX_RB) {
    T x[MGX_RB];
    load_rows(x, Bm, Bs, r0, ne, lc, dl);
#pragma unroll
    for (int j = 0; j < MGX_RB; j++) {
      const int r = r0 + j;
      if (r < ne) {
        T dv = x[j] * wv, ds = x[j] * ws, dw = x[j] * ww, nn = x[j] * x[j];
        wave_sum4(dv, ds, dw, nn);
        T* q = efc + 8 * r;
        const T aref = -q[6] * dv - q[5];
        const T Rr = q[2];
        const T jar = dw - aref;
        const T ad = nn + Rr;
        if (l == 0) {
          q[5] = aref;
          q[0] = ds - aref;
          q[1] = jar < 0 ? -jar / Rr : (T)0;
          q[4] = ad;
          q[3] = (T)1 / ad;
        }
      }
    }
  }
  wsync();
  // v = B' f (lane = dof), then the warmstart dual cost
  T v = 0;
  for (int r0 = 0; r0 < ne; r0 += MGX_RB) {
    T x[MGX_RB];
    load_rows(x, Bm, Bs, r0, ne, lc, dl);
#pragma unroll
    for (int j = 0; j < MGX_RB; j++)
      if (r0 + j < ne) v += efc[8 * (r0 + j) + 1] * x[j];
  }
  T cost = 0;
  for (int r0 = 0; r0 < ne; r0 += MGX_RB) {
    T x[MGX_RB];
    load_rows(x, Bm, Bs, r0, ne, lc, dl);
#pragma unroll
    for (int j = 0; j < MGX_RB; j++) {
      if (r0 + j < ne) {
        const T bv = usum(x[j] * v);
        const T* q = efc + 8 * (r0 + j);
        cost += q[1] * (q[0] + (T)0.5 * (bv + q[2] * q[1]));
      }
    }
  }
  if (cost > 0) {
    for (int r = l; r < ne; r += 64) efc[8 * r + 1] = 0;
    v = 0;
  }
  wsync();
  // Gauss-Seidel sweeps with early exit on scaled improvement < tolerance. Rows go in blocks of
  // 4: the four dots B_r.v use the pre-block v (4 interleaved reductions), and row i of the
  // block adds sum_{j<i} A_ij delta_j with A_ij = B_i.B_j precomputed -> the same sequential
  // Gauss-Seidel update as row-by-row, in a quarter of the reduction latency. Rows ne..ne4-1
  // are zero padding (B = 0, b = f = 0, R = AR = 1) and never change.
  const int ne4 = (ne + 3) & ~3;
  for (int r = ne + l; r < ne4; r += 64) {
    T* q = efc + 8 * r;
    q[0] = 0; q[1] = 0; q[2] = 1; q[3] = 1; q[4] = 1;
  }
  for (int r = ne; r < ne4; r++)
    if (dl) e.Bm[r * Bs + l] = 0;
  wsync();
  T* blk = e.efc_blk;  // [ne4/4][8]: A_10, A_20, A_21, A_30, A_31, A_32
  for (int b0 = 0; b0 < ne4; b0 += 4) {  // row-major: 4 coalesced row loads, 6 wave reductions
    const T x0 = dl ? Bm[b0 * Bs + lc] : (T)0, x1 = dl ? Bm[(b0 + 1) * Bs + lc] : (T)0;
    const T x2 = dl ? Bm[(b0 + 2) * Bs + lc] : (T)0, x3 = dl ? Bm[(b0 + 3) * Bs + lc] : (T)0;
    T a10 = x1 * x0, a20 = x2 * x0, a21 = x2 * x1, a30 = x3 * x0;
    T a31 = x3 * x1, a32 = x3 * x2, z0 = 0, z1 = 0;
    wave_sum4(a10, a20, a21, a30);
    wave_sum4(a31, a32, z0, z1);
    if (l == 0) {
      T* o = blk + 2 * b0;
      o[0] = a10; o[1] = a20; o[2] = a21; o[3] = a30; o[4] = a31; o[5] = a32;
    }
  }
  wsync();
  const T scale = (T)1 / (m.meaninertia * (T)(nv > 1 ? nv : 1));
  const T tol = m.tolerance;
  const int maxit = m.iterations;
  int iter = 0;
  while (iter < maxit) {
    T improvement = 0;
    // one block ahead: the next block's 4 rows load while this block is solved
    T nx0 = Bm[lc], nx1 = Bm[Bs + lc], nx2 = Bm[2 * Bs + lc], nx3 = Bm[3 * Bs + lc];
    for (int r0 = 0; r0 < ne4; r0 += 4) {
      const T bv0 = dl ? nx0 : (T)0, bv1 = dl ? nx1 : (T)0, bv2 = dl ? nx2 : (T)0, bv3 = dl ? nx3 : (T)0;
      const int rn = r0 + 4 < ne4 ? r0 + 4 : r0;  // the last block re-reads itself (in bounds)
      nx0 = Bm[rn * Bs + lc]; nx1 = Bm[(rn + 1) * Bs + lc];
      nx2 = Bm[(rn + 2) * Bs + lc]; nx3 = Bm[(rn + 3) * Bs + lc];
      T d0 = bv0 * v, d1 = bv1 * v, d2 = bv2 * v, d3 = bv3 * v;
      wave_sum4(d0, d1, d2, d3);
      const T* a = blk + 2 * r0;
      T a10 = a[0], a20 = a[1], a21 = a[2], a30 = a[3], a31 = a[4], a32 = a[5];
      T dl0, dl1, dl2, dl3;
#define MGX_ROW(i, DOT, DL)                                                        \
      {                                                                            \
        T* q = efc + 8 * (r0 + i);                                                 \
        T br = q[0], fr = q[1], Rr = q[2], ai = q[3], ad = q[4];                   \
        T res = br + (DOT) + Rr * fr;                                              \
        T fn = fr - res * ai;                                                      \
        fn = fn < 0 ? (T)0 : fn;                                                   \
        T delta = fn - fr;                                                         \
        T change = (T)0.5 * delta * delta * ad + delta * res;                      \
        bool keep = change > (T)1e-10;                                             \
        fn = keep ? fr : fn;                                                       \
        DL = keep ? (T)0 : delta;                                                  \
        improvement -= keep ? (T)0 : change;                                       \
        q[1] = fn;                                                                 \
      }
      MGX_ROW(0, d0, dl0)
      MGX_ROW(1, d1 + a10 * dl0, dl1)
      MGX_ROW(2, d2 + a20 * dl0 + a21 * dl1, dl2)
      MGX_ROW(3, d3 + a30 * dl0 + a31 * dl1 + a32 * dl2, dl3)
#undef MGX_ROW
      v += dl0 * bv0 + dl1 * bv1 + dl2 * bv2 + dl3 * bv3;
    }
    iter++;
    if (improvement * scale < tol) break;
  }
  e.niter = iter;
  // qacc = qacc_smooth + L^-1 D^-1/2 v ; qfrc_constraint = L' D^1/2 v
  T z = dl ? v * e.diaginv * sqrtD : (T)0;  // D^-1/2 = diaginv * sqrt(D)
  z = solve_L(m, e, e.qLD, z);
  e.qacc = e.qacc_smooth + z;
  e.qfrc_constraint = mul_LT(m, e, e.qLD, sqrtD * v);
  wsync();
}

// ---------------------------------------------------------------- Newton Hessian on MFMA
// H = I + sum_{x_r<0} D_r B_r B_r' (nv x nv, lower triangle into row-major LDS) as a sum of
// 16x16x4 MFMA products over chunks of 4 rows: tile (t, u) += A_t B_u with A_t[i][k] = s_k B[r0+k]
// [16t+i] (s_k = D of an active row, else 0) and B_u[k][j] = B[r0+k][16u+j]; 10 lower tiles for
// nv <= 64. Lane l holds A[l&15][l>>4] / B[l>>4][l&15] (one element each, 4 loads per chunk, 16
// consecutive columns of one row per 16 lanes); C/D: col = l&15, row = 4(l>>4)+v (f32) or
// (l>>4)+4v (f64) (cdna_hip_programming.md, fragment layout).
// GRAD (T1 = 4: every dof column is loaded): the same pass also returns sum_{x<0} D x B_r for this
// lane's dof (lane = dof): per lane the rows kq, kq + 4, ... of each tile column, then the four
// row groups added (xor 16, xor 32) — Newton's gradient off the Hessian's own row stream.
template <typename T>
__device__ __forceinline__ T xor_sum_kq(T x) {
  x += __shfl_xor(x, 16);
  x += __shfl_xor(x, 32);
  return x;
}
template <typename T, int T0 = 0, int T1 = 4, bool GRAD = false>
__device__ __forceinline__ T hessian_mfma(const T* Bm, int Bs, const T* efc, int ne, int nv, T* H) {
  typedef T V4 __attribute__((ext_vector_type(4)));
  const int l = lane_id(), i = l & 15, kq = l >> 4;
  const int nt = (nv + 15) >> 4;
  if (!GRAD && T0 >= nt) return (T)0;
  static_assert(!GRAD || T1 == 4, "the fused gradient needs every dof column");
  auto row_of = [&](int v) { return sizeof(T) == 8 ? kq + 4 * v : 4 * kq + v; };
  constexpr int NT = (T1 * (T1 + 1) - T0 * (T0 + 1)) / 2;  // tiles of tile rows [T0, T1)
  T gp[T1];
#pragma unroll
  for (int t = 0; t < T1; t++) gp[t] = 0;
  V4 acc[NT];
#pragma unroll
  for (int t = T0, q = 0; t < T1; t++)
#pragma unroll
    for (int u = 0; u <= t; u++, q++)
#pragma unroll
      for (int v = 0; v < 4; v++) acc[q][v] = (t == u && row_of(v) == i) ? (T)1 : (T)0;
  // rows with x >= 0 add nothing (s_k = 0): their B is not loaded (zeros instead), and a chunk
  // of four inactive rows skips its MFMAs — the same sums, without streaming inactive rows
  auto load = [&](int r0, T* b, T& sc, T& sg) {
    const int r = r0 + kq;
    sc = 0;
    sg = 0;
    if (r < ne) {
      const T x = efc[8 * r + 1];
      sc = x < 0 ? efc[8 * r + 4] : (T)0;
      sg = sc * x;
    }
#pragma unroll
    for (int t = 0; t < T1; t++) {
      const int c = 16 * t + i;
      b[t] = (sc != (T)0 && c < nv) ? Bm[r * Bs + c] : (T)0;
    }
  };
  // the next MGX_HD chunks are in flight during this chunk's MFMAs (B in global scratch: L2 misses)
  T bq[MGX_HD][T1], sq[MGX_HD], gq[MGX_HD];
#pragma unroll
  for (int d = 0; d < MGX_HD; d++) load(4 * d, bq[d], sq[d], gq[d]);
  for (int r0 = 0; r0 < ne; r0 += 4) {
    T b[T1];
#pragma unroll
    for (int t = 0; t < T1; t++) b[t] = bq[0][t];
    const T sc = sq[0], sg = gq[0];
#pragma unroll
    for (int d = 0; d + 1 < MGX_HD; d++) {
      sq[d] = sq[d + 1];
      gq[d] = gq[d + 1];
#pragma unroll
      for (int t = 0; t < T1; t++) bq[d][t] = bq[d + 1][t];
    }
    load(r0 + 4 * MGX_HD, bq[MGX_HD - 1], sq[MGX_HD - 1], gq[MGX_HD - 1]);
    if (__ballot(sc != (T)0) == 0ull) continue;
    if constexpr (GRAD) {
#pragma unroll
      for (int t = 0; t < T1; t++) gp[t] += sg * b[t];
    }
#pragma unroll
    for (int t = T0, q = 0; t < T1; t++)
#pragma unroll
      for (int u = 0; u <= t; u++, q++) {
        if (t < nt) {
          if constexpr (sizeof(T) == 8)
            acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(sc * b[t], b[u], acc[q], 0, 0, 0);
          else
            acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(sc * b[t], b[u], acc[q], 0, 0, 0);
        }
      }
  }
#pragma unroll
  for (int t = T0, q = 0; t < T1; t++)
#pragma unroll
    for (int u = 0; u <= t; u++, q++)
#pragma unroll
      for (int v = 0; v < 4; v++) {
        const int row = 16 * t + row_of(v), col = 16 * u + i;
        if (t < nt && row < nv && col <= row) H[row * nv + col] = acc[q][v];
      }
  if constexpr (GRAD) {
    // lane l = 16 kq + i holds dof 16 t + i of tile column t = kq after the row-group sums
    T g = 0;
#pragma unroll
    for (int t = 0; t < T1; t++) {
      const T s = xor_sum_kq(gp[t]);
      g = kq == t ? s : g;
    }
    return l < nv ? g : (T)0;
  }
  return (T)0;
}

// ---------------------------------------------------------------- blocked Cholesky
// H = L L' in place (lower triangle of the row-major nv x nv H, nv <= 128; the narrow Newton
// solver and the wide one), right-looking in
// 16-wide block columns: factor the diagonal block (lanes = its rows, one wave barrier per
// column, <= 15-term dots), solve the panel below it against L_kk' (lane = row, L_kk read as LDS
// broadcasts), then subtract L_I L_J' from every trailing lower tile on MFMA (16x16x4: four
// per tile, accumulators initialised from the tile). Entries past nv read as 0 and are never
// stored. Same pivot clamp as the unblocked factor (d = sqrt(max(dkk, minval))); the column
// below a pivot is scaled by 1 / d as mju_cholFactor [ext] does. PK: H is the
// packed lower triangle (entry (r, c), c <= r, at r (r + 1) / 2 + c; the wide solver, gb_efc_off).
template <bool PK>
__device__ __forceinline__ int hidx(int r, int c, int nv) {
  return PK ? (r * (r + 1) >> 1) + c : r * nv + c;
}

// 1. diagonal block kb in registers: lane i < bk holds row k0 + i of the block (16 entries), the
//    factor is right-looking over the block's columns with the column values broadcast by
//    readlane — no LDS round trip or wave barrier per column. Entry (i, c) receives the same
//    products in the same order as the left-looking dot s = a_ic - sum_{j<c} l_ij l_cj.
template <typename T, bool PK>
__device__ __forceinline__ void chol_diag(T* H, int nv, int kb) {
  const int l = lane_id();
  const int k0 = 16 * kb, bk = nv - k0 < 16 ? nv - k0 : 16;
  T x[16];
  const T* Lr = H + hidx<PK>(k0 + (l < bk ? l : 0), k0, nv);
#pragma unroll
  for (int j = 0; j < 16; j++) x[j] = (l < bk && j <= l) ? Lr[j] : (T)0;
#pragma unroll
  for (int c = 0; c < 16; c++) {
    if (c < bk) {
      const T dkk = readlane(x[c], c);
      const T d = sqrt(dkk > minval<T>() ? dkk : minval<T>());
      const T rd = (T)1 / d;  // mju_cholFactor: the column is scaled by 1 / L_cc
      x[c] = l == c ? d : (l > c ? x[c] * rd : x[c]);
      const T lic = x[c];
#pragma unroll
      for (int j = c + 1; j < 16; j++)
        if (j < bk && l >= j) x[j] -= lic * readlane(x[c], j);
    }
  }
  T* Hr = H + hidx<PK>(k0 + (l < bk ? l : 0), k0, nv);
  if (l < bk)
#pragma unroll
    for (int j = 0; j < 16; j++)
      if (j <= l) Hr[j] = x[j];
}

// 2. panel of block column kb: rows below the block, x = a L_kk^-T by forward substitution (lane =
//    row); row sets j = j0, j0 + js, ... of 64 rows each (one wave: all of them)
template <typename T, bool PK>
__device__ __forceinline__ void chol_panel(T* H, int nv, int kb, int j0, int js) {
  const int l = lane_id();
  const int k0 = 16 * kb, bk = nv - k0 < 16 ? nv - k0 : 16;
  if (k0 + bk + 64 * j0 >= nv) return;
  // 1 / L_cc of the block's columns, off the rows' dependent chains (mju_cholFactor's scaling)
  T rdg[16];
#pragma unroll
  for (int c = 0; c < 16; c++) rdg[c] = c < bk ? (T)1 / H[hidx<PK>(k0 + c, k0 + c, nv)] : (T)0;
  for (int rb = k0 + bk + 64 * j0; rb < nv; rb += 64 * js) {
    const int r = rb + l;
    if (r < nv) {
      T* Ar = H + hidx<PK>(r, k0, nv);
      T x[16];
#pragma unroll
      for (int c = 0; c < 16; c++) {
        if (c < bk) {
          T t = Ar[c];
#pragma unroll
          for (int j = 0; j < c; j++) t -= x[j] * H[hidx<PK>(k0 + c, k0 + j, nv)];
          x[c] = t * rdg[c];
        }
      }
#pragma unroll
      for (int c = 0; c < 16; c++)
        if (c < bk) Ar[c] = x[c];
    }
  }
}

// 3. trailing lower tiles (I, J), kb < J <= I < nb: A_IJ -= L_Ik L_Jk' on MFMA; tiles q0, q0 + qs,
//    ... in (I, J) order (one wave: all of them)
template <typename T, bool PK>
__device__ __forceinline__ void chol_trail(T* H, int nv, int kb, int q0, int qs) {
  typedef T V4 __attribute__((ext_vector_type(4)));
  const int l = lane_id();
  const int nb = (nv + 15) >> 4;
  const int k0 = 16 * kb, bk = nv - k0 < 16 ? nv - k0 : 16;
  const int i = l & 15, kq = l >> 4;
  auto row_of = [&](int v) { return sizeof(T) == 8 ? kq + 4 * v : 4 * kq + v; };
  int q = 0;
  for (int I = kb + 1; I < nb; I++) {
    for (int J = kb + 1; J <= I; J++, q++) {
      if (q < q0 || (q - q0) % qs) continue;
      V4 acc;
#pragma unroll
      for (int v = 0; v < 4; v++) {
        const int row = 16 * I + row_of(v), col = 16 * J + i;
        acc[v] = (row < nv && col <= row) ? H[hidx<PK>(row, col, nv)] : (T)0;
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int kk = k0 + 4 * u + kq;  // this lane's k in the 16-wide block column
        const int ra = 16 * I + i, rb = 16 * J + i;
        const T a = (ra < nv && kk < k0 + bk) ? -H[hidx<PK>(ra, kk, nv)] : (T)0;
        const T b = (rb < nv && kk < k0 + bk) ? H[hidx<PK>(rb, kk, nv)] : (T)0;
        if constexpr (sizeof(T) == 8)
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
        else
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
      }
#pragma unroll
      for (int v = 0; v < 4; v++) {
        const int row = 16 * I + row_of(v), col = 16 * J + i;
        if (row < nv && col <= row) H[hidx<PK>(row, col, nv)] = acc[v];
      }
    }
  }
}

template <typename T, bool PK = false>
__device__ __forceinline__ void chol_blocked(T* H, int nv) {
  const int nb = (nv + 15) >> 4;
  for (int kb = 0; kb < nb; kb++) {
    chol_diag<T, PK>(H, nv, kb);
    wsync();
    chol_panel<T, PK>(H, nv, kb, 0, 1);
    wsync();
    chol_trail<T, PK>(H, nv, kb, 0, 1);
    wsync();
  }
}

// ---------------------------------------------------------------- constraint solver (Newton)
// mj_solNewton [ext] (restated in oracle/mjref.c newton_solve), in the whitened coordinates of
// the PGS path: u = D^1/2 L (qacc - qacc_smooth), so 0.5 (a-a0)'M(a-a0) = 0.5 |u|^2 and
// J_r qacc - aref_r = B_r.u + b_r. Cost 0.5|u|^2 + sum_{x_r<0} 0.5 D_r x_r^2 (D = 1/R; limit and
// pyramid-edge rows are one-sided). Per iteration: gradient g = u + sum_{x<0} D x B_r (lane =
// dof); Hessian H = I + sum_{x<0} D B_r B_r' (row-major nv x nv in LDS, built lane = column);
// in-place Cholesky (lane = column, one wave barrier per column); p = -H^-1 g by two triangular
// sweeps on readlane; the exact line search along p on the convex piecewise-quadratic cost
// (safeguarded Newton on its piecewise-linear derivative, as the oracle); MuJoCo's stop rules
// (scaled dof-space gradient, scaled improvement). Row scalars: q[0] b, q[1] x (efc_force at
// exit), q[2] R, q[3] B_r.p, q[4] D.
//
// The improvement is the cost decrease along the accepted step evaluated term by term, al u.p +
// al^2 p.p / 2 + sum_r row_cost_change — algebraically MuJoCo's cost(old) - cost(new), without
// subtracting two totals: on construction states (steel beams deep in the floor) the cost is
// ~1e10 and the difference of totals rounds to 0 or a few ulps, so the stop test, the iteration
// count and qacc (at the 1e-3 level, along the weakly constrained light-block directions) would
// be decided by rounding. oracle/mjref.c newton_solve evaluates the same expression.
template <typename T>
__device__ __forceinline__ T row_cost_change(T x, T dx, T D) {
  // s(x + dx) - s(x) for s(x) = D x^2 / 2 on x < 0, 0 otherwise
  const T xn = x + dx;
  if (x < 0 && xn < 0) return (T)0.5 * D * dx * (x + xn);
  if (x < 0) return (T)-0.5 * D * x * x;
  if (xn < 0) return (T)0.5 * D * xn * xn;
  return 0;
}

// newton()'s row passes over the batches b0, b0 + bs, ... of MGX_RB rows (bs = the wave count:
// wave 0 takes the even batches, the helper wave the odd ones; one wave takes them all in order).
// setup: aref, b, x at u = 0 and at the warmstart, D per row; the two costs' partial sums, the
// even batches' in c0 / cw and the odd batches' in c0o / cwo whatever the wave count, so one wave
// and a wave pair add the same partial sums in the same order (c0 + c0o: ADVICE r05, the warmstart
// choice cw < c0 may not depend on the workgroup size)
template <typename T>
__device__ __forceinline__ void nt_setup_rows(const Env<T>& e, int ne, int nv, T wv, T ws, T wd, int b0, int bs, T& c0,
                                              T& cw, T& c0o, T& cwo) {
  const int l = lane_id();
  const bool dl = l < nv;
  const int lc = dl ? l : 0;
  T* efc = e.efc;
  const int step = MGX_RB * bs;
  T xn[MGX_RD][MGX_RB];
  first_rows(xn, e.Bm, e.Bs, ne, lc, dl, MGX_RB * b0, step);
  for (int r0 = MGX_RB * b0; r0 < ne; r0 += step) {
    T xb[MGX_RB];
    next_rows(xb, xn, e.Bm, e.Bs, r0, ne, lc, dl, step);
#pragma unroll
    for (int j = 0; j < MGX_RB; j++) {
      const int r = r0 + j;
      if (r < ne) {
        T dv = xb[j] * wv, ds = xb[j] * ws, dw = xb[j] * wd, z = 0;
        wave_sum4(dv, ds, dw, z);
        T* q = efc + 8 * r;
        const T aref = -q[6] * dv - q[5];
        const T b = ds - aref, D = (T)1 / q[2], xw = b + dw;
        const bool odd = ((r0 / MGX_RB) & 1) != 0;
        if (b < 0) (odd ? c0o : c0) += (T)0.5 * D * b * b;
        if (xw < 0) (odd ? cwo : cw) += (T)0.5 * D * xw * xw;
        if (l == 0) { q[5] = aref; q[0] = b; q[1] = b; q[3] = xw; q[4] = D; }
      }
    }
  }
}
// J p per row (wave reductions; lane 0 stores efc[8 r + 3])
template <typename T>
__device__ __forceinline__ void nt_jp_rows(const Env<T>& e, int ne, int nv, T p, int b0, int bs) {
  const int l = lane_id();
  const bool dl = l < nv;
  const int lc = dl ? l : 0;
  T* efc = e.efc;
  const int step = MGX_RB * bs;
  T xn[MGX_RD][MGX_RB];
  first_rows(xn, e.Bm, e.Bs, ne, lc, dl, MGX_RB * b0, step);
  for (int r0 = MGX_RB * b0; r0 < ne; r0 += step) {
    T xb[MGX_RB];
    next_rows(xb, xn, e.Bm, e.Bs, r0, ne, lc, dl, step);
#pragma unroll
    for (int j = 0; j < MGX_RB; j += 4) {
      T s0 = xb[j] * p, s1 = xb[j + 1] * p, s2 = xb[j + 2] * p, s3 = xb[j + 3] * p;
      wave_sum4(s0, s1, s2, s3);
      if (l == 0) {
        if (r0 + j < ne) efc[8 * (r0 + j) + 3] = s0;
        if (r0 + j + 1 < ne) efc[8 * (r0 + j + 1) + 3] = s1;
        if (r0 + j + 2 < ne) efc[8 * (r0 + j + 2) + 3] = s2;
        if (r0 + j + 3 < ne) efc[8 * (r0 + j + 3) + 3] = s3;
      }
    }
  }
}
template <typename T>
__device__ __forceinline__ void newton(const DevModel<T>& m, Env<T>& e) {
  const int l = lane_id();
  const int ne = __builtin_amdgcn_readfirstlane(e.nefc);
  const int nv = m.nv;
  const bool dl = l < nv;
  const int lc = dl ? l : 0;
  T sqrtD = dl ? sqrt(e.qLD[m.dof_Madr[l]]) : (T)0;
  if (ne == 0) {
    e.qacc = e.qacc_smooth;
    e.qfrc_constraint = 0;
    e.niter = 0;
    return;
  }
  MGX_STAMP_DECL
  T qv = dl ? e.qvel[l] : (T)0;
  const T wv = sqrtD * mul_L(m, e, e.qLD, qv);
  const T ws = sqrtD * mul_L(m, e, e.qLD, e.qacc_smooth);
  const T ww = sqrtD * mul_L(m, e, e.qLD, e.qacc_ws);
  const T wd = dl ? ww - ws : (T)0;
  T* efc = e.efc;
  const T* Bm = e.Bm;
  const int Bs = e.Bs;
  // per row: aref, b = J qacc_smooth - aref, D; x at u = 0 (q[1]) and at the warmstart (q[3]).
  // Rows are read row-major (lane = dof, one coalesced load per row, wave reductions), which is
  // what keeps the global-scratch rows (Layout.gB) off the latency path; the row scalars are
  // uniform and lane 0 stores them.
  T c0 = 0, cw = 0, c0o = 0, cwo = 0;
  const int nw = e.nw;
  if (nw > 1) {  // the helper's inputs
    if (dl) { e.vec0[l] = wv; e.vec1[l] = ws; e.vec2[l] = wd; }
  }
  team_begin(e, TEAM_SETUP, ne);
  nt_setup_rows(e, ne, nv, wv, ws, wd, 0, nw, c0, cw, c0o, cwo);
  team_end(e);
  if (nw > 1) {  // the helper's partial costs (odd batches), in vec3[0..1]
    c0 += e.vec3[0];
    cw += e.vec3[1];
  } else {
    c0 += c0o;
    cw += cwo;
  }
  const T uw = wd;
  cw += usum((T)0.5 * uw * uw);
  const bool warm = cw < c0;
  T u = warm ? uw : (T)0;
  if (warm) for (int r = l; r < ne; r += 64) efc[8 * r + 1] = efc[8 * r + 3];
  wsync();
  T* H = e.hess;
  const T scale = (T)1 / (m.meaninertia * (T)(nv > 1 ? nv : 1));
  const T tol = m.tolerance;
  const T eps = sizeof(T) == 4 ? (T)1e-7 : (T)1e-15;
  const int maxit = m.iterations;
  int iter = 0;
  // H = I + sum_{x<0} D B_r B_r' (MFMA, lower triangle) and the whitened gradient g = u + sum_{x<0}
  // D x B_r in one pass over the active rows, at the current point: before the first iteration and
  // after every update (the stop test's gradient; the Hessian of the next iteration, unused after the
  // last). Two waves: tile rows 0..2 on wave 0, tile row 3 and the gradient (every dof column) on
  // the helper, which hands the gradient over in vec1.
  auto hess_grad = [&]() {
    T gs = 0;
    team_begin(e, TEAM_HESS, ne);
    if (nw > 1) hessian_mfma<T, 0, 3>(Bm, Bs, efc, ne, nv, H);
    else gs = hessian_mfma<T, 0, 4, true>(Bm, Bs, efc, ne, nv, H);
    team_end(e);
    if (nw > 1) gs = e.vec1[lc];
    return dl ? u + gs : (T)0;
  };
  T g = hess_grad();
  MGX_STAMP(10);  // newton sub-stages (diagnostic build only): setup + the first Hessian
  // mj_solNewton's loop order [ext]: update first, then test the scaled improvement and the
  // scaled gradient at the new point, so at least one iteration runs
  while (iter < maxit) {
    MGX_STAMP(11);  // (the Hessian: hess_grad, stamped with the update)
    // Cholesky H = L L' in place: 16-wide block columns, trailing update on MFMA (chol_blocked)
    {
      const int nb = (nv + 15) >> 4;
      for (int kb = 0; kb < nb; kb++) {
        chol_diag<T, false>(H, nv, kb);
        wsync();
        chol_panel<T, false>(H, nv, kb, 0, 1);
        if (kb + 1 < nb) {
          team_begin(e, TEAM_TRAIL, kb);
          chol_trail<T, false>(H, nv, kb, 0, nw);
          team_end(e);
        } else {
          wsync();
        }
      }
    }
    MGX_STAMP(12);  // Cholesky
    // L y = -g, L' p = y (reciprocal pivots computed once, lane-parallel)
    const T rdiag = dl ? (T)1 / H[l * nv + l] : (T)0;
    T y = -g;
    for (int k = 0; k < nv; k++) {
      T yk = readlane(y, k) * readlane(rdiag, k);
      if (l == k) y = yk;
      else if (dl && l > k) y -= H[l * nv + k] * yk;
    }
    T p = y;
    for (int k = nv - 1; k >= 0; k--) {
      T pk = readlane(p, k) * readlane(rdiag, k);
      if (l == k) p = pk;
      else if (l < k) p -= H[k * nv + l] * pk;
    }
    p = dl ? p : (T)0;
    MGX_STAMP(13);  // triangular solves
    // J p per row, row-major (coalesced, 8 rows per batch) with wave reductions; lane 0 stores
    if (nw > 1 && dl) e.vec0[l] = p;  // the helper's input
    team_begin(e, TEAM_JP, ne);
    nt_jp_rows(e, ne, nv, p, 0, nw);
    team_end(e);
    MGX_STAMP(14);  // J p
    // line search along p (oracle/mjref.c newton_solve, MuJoCo's stop rule [ext]): f'(al) = u.p +
    // al p.p + sum_{x + al jp < 0} D (x + al jp) jp; first point the Newton step from al = 0, then
    // safeguarded Newton in the bracket until |f'| < gtol = tolerance * ls_tolerance * |s| *
    // meaninertia * max(1, nv) with s = L^-1 D^-1/2 p the dof-space direction, <= 50 evaluations
    const T g0 = usum(u * p), pp = usum(p * p);
    T sdof = dl ? p * e.diaginv * sqrtD : (T)0;  // D^-1/2 p
    sdof = solve_L(m, e, e.qLD, sdof);
    const T snorm = sqrt(usum(dl ? sdof * sdof : (T)0));
    auto ls_eval = [&](T al, T& d1, T& d2) {
      T d1p = 0, d2p = 0;
      for (int r = l; r < ne; r += 64) {
        const T* q = efc + 8 * r;
        T jp = q[3], xr = q[1] + al * jp;
        if (xr < 0) { d1p += q[4] * xr * jp; d2p += q[4] * jp * jp; }
      }
      d1 = g0 + al * pp + usum(d1p);
      d2 = pp + usum(d2p);
    };
    T al = 0;
    if (snorm >= minval<T>()) {
      const T gtol = tol * (T)0.01 * snorm * m.meaninertia * (T)(nv > 1 ? nv : 1);
      T d1, d2;
      ls_eval((T)0, d1, d2);
      al = -d1 / d2;
      T lo = 0, hi = (T)1e30;
      for (int ls = 0; ls < 50; ls++) {
        ls_eval(al, d1, d2);
        if (fabs(d1) < gtol) break;
        if (d1 < 0) lo = al; else hi = al;
        T nxt = d2 > 0 ? al - d1 / d2 : 2 * al;
        if (!(nxt > lo && nxt < hi)) nxt = hi < (T)1e30 ? (T)0.5 * (lo + hi) : 2 * al;
        const bool stall = fabs(nxt - al) <= eps * (1 + fabs(al));  // no change in floating point
        al = nxt;
        if (stall) break;
      }
    }
    MGX_STAMP(15);  // line search
    u += al * p;
    T dc = 0;
    for (int r = l; r < ne; r += 64) {
      T* q = efc + 8 * r;
      dc += row_cost_change(q[1], al * q[3], q[4]);
      q[1] += al * q[3];
    }
    // the cost decrease along the step, evaluated term by term (newton_step_decrease)
    const T improvement = -scale * (al * g0 + (T)0.5 * al * al * pp + usum(dc));
    iter++;
    wsync();
    g = hess_grad();
    // the gradient rule is on the dof-space gradient M(a - a0) - J'f = L' D^1/2 g
    T ga = mul_LT(m, e, e.qLD, sqrtD * g);
    const bool stop = improvement < tol || scale * sqrt(usum(dl ? ga * ga : (T)0)) < tol;
    MGX_STAMP(16);  // update, gradient, stop tests
    if (stop) break;
  }
  e.niter = iter;
  for (int r = l; r < ne; r += 64) {
    T* q = efc + 8 * r;
    q[1] = q[1] < 0 ? -q[4] * q[1] : (T)0;
  }
  wsync();
  // qacc = qacc_smooth + L^-1 D^-1/2 u ; qfrc_constraint = J'f = L' D^1/2 (sum f_r B_r)
  // sum_r f_r B_r with f_r = -D x_r on the active rows = u - g (g = u + sum_{x<0} D x B_r at the
  // final point, the last hess_grad): no pass over the rows
  T v = dl ? u - g : (T)0;
  T z = dl ? u * e.diaginv * sqrtD : (T)0;
  z = solve_L(m, e, e.qLD, z);
  e.qacc = e.qacc_smooth + z;
  e.qfrc_constraint = mul_LT(m, e, e.qLD, sqrtD * v);
  wsync();
}

// wave 1 of a two-wave narrow Newton env (k_assembly): one loop iteration per barrier of wave 0
// (TEAM_NONE), the odd batches / tile row 3 + the gradient / every other trailing tile of a section,
// until wave 0 posts TEAM_EXIT
template <typename T>
__device__ __forceinline__ void team_helper_n(const DevModel<T>& m, Env<T>& e) {
  const int l = lane_id(), nv = m.nv;
  const bool dl = l < nv;
  for (;;) {
    __syncthreads();
    const int cmd = __builtin_amdgcn_readfirstlane(e.ctl[0]);
    if (cmd == TEAM_NONE) continue;
    if (cmd == TEAM_EXIT) break;
    const int a = __builtin_amdgcn_readfirstlane(e.ctl[1]);
    if (cmd == TEAM_SETUP) {
      const T wv = dl ? e.vec0[l] : (T)0, ws = dl ? e.vec1[l] : (T)0, wd = dl ? e.vec2[l] : (T)0;
      T c0 = 0, cw = 0, c0o = 0, cwo = 0;  // odd batches only: c0o / cwo
      nt_setup_rows(e, a, nv, wv, ws, wd, 1, 2, c0, cw, c0o, cwo);
      if (l == 0) { e.vec3[0] = c0o; e.vec3[1] = cwo; }
    } else if (cmd == TEAM_HESS) {  // tile row 3 and the gradient (newton's hess_grad)
      e.vec1[l] = hessian_mfma<T, 3, 4, true>(e.Bm, e.Bs, e.efc, a, nv, e.hess);
    } else if (cmd == TEAM_TRAIL) {
      chol_trail<T, false>(e.hess, nv, a, 1, 2);
    } else if (cmd == TEAM_JP) {
      nt_jp_rows(e, a, nv, dl ? e.vec0[l] : (T)0, 1, 2);
    } else if (cmd == TEAM_XFORM) {
      transform_rows_rm(m, e, a, 1, 2);
    } else if (cmd == TEAM_CONTACT) {  // every other contact's rows (make_constraint)
      bool ovf;
      contact_rows_share(m, e, a, __builtin_amdgcn_readfirstlane(e.ctl[2]), 1, 2, ovf);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- integration
template <typename T>
__device__ __forceinline__ void quat_integrate(T* q, const T* w, T h) {
  T ax[3] = {w[0], w[1], w[2]}, qr[4];
  T ang = h * normalize3(ax);
  axisangle2quat(qr, ax, ang);
  normalize4(q);
  mulquat(q, q, qr);
}

// mj_integratePos [ext]: qpos <- qpos '+' h vel (free: position + quaternion, ball: quaternion)
template <typename T>
__device__ __forceinline__ void integrate_pos(const DevModel<T>& m, T* qpos, const T* vel, T h) {
  int l = lane_id();
  for (int j = l; j < m.njnt; j += 64) {
    int a = m.jnt_qposadr[j], da = m.jnt_dofadr[j], t = m.jnt_type[j];
    if (t == JFREE) {
      for (int k = 0; k < 3; k++) qpos[a + k] += h * vel[da + k];
      quat_integrate(qpos + a + 3, vel + da + 3, h);
    } else if (t == JBALL) {
      quat_integrate(qpos + a, vel + da, h);
    } else {
      qpos[a] += h * vel[da];
    }
  }
  wsync();
}

template <typename T, bool NT = false>
__device__ __forceinline__ void forward(const DevModel<T>& m, Env<T>& e);

// mj_RungeKutta(m, d, 4) [ext], after forward() at X[0] (oracle/mjref.c rk4): stage i runs the
// forward pass at X[i] = X[0] '+' h sum_j A_ij X'[j]; the final mj_advance uses
// dX = sum_j B_j X'[j]. Velocities and accelerations stay in dof-lane registers; X[0]
// positions and the dX velocity vector (integratePos input) sit in the rk LDS region. The
// frames left in LDS are those of the last stage, as MuJoCo leaves them in mjData.
template <typename T, bool NT = false>
__device__ __forceinline__ void rk4(const DevModel<T>& m, Env<T>& e) {
  const T A[9] = {(T)0.5, 0, 0, 0, (T)0.5, 0, 0, 0, (T)1};
  const T B[4] = {(T)(1.0 / 6.0), (T)(1.0 / 3.0), (T)(1.0 / 3.0), (T)(1.0 / 6.0)};
  const int l = lane_id(), nq = m.nq;
  const bool dl = l < m.nv;
  T* q0 = e.rk;
  T* dxv = e.rk + ((nq + 3) & ~3);
  const T h = m.timestep, t0 = e.time;
  for (int k = l; k < nq; k += 64) q0[k] = e.qpos[k];
  T v[4], f[4];
  v[0] = dl ? e.qvel[l] : (T)0;
  f[0] = dl ? e.qacc : (T)0;
  for (int i = 1; i < 4; i++) {
    T C = 0, dv = 0, da = 0;
    for (int j = 0; j < i; j++) {
      T a = A[(i - 1) * 3 + j];
      C += a;
      dv += a * v[j];
      da += a * f[j];
    }
    wsync();
    if (dl) dxv[l] = dv;
    for (int k = l; k < nq; k += 64) e.qpos[k] = q0[k];
    wsync();
    integrate_pos(m, e.qpos, dxv, h);
    v[i] = v[0] + h * da;
    if (dl) e.qvel[l] = v[i];
    e.time = t0 + C * h;
    wsync();
    forward<T, NT>(m, e);
    f[i] = dl ? e.qacc : (T)0;
  }
  T dv = 0, da = 0;
  for (int j = 0; j < 4; j++) { dv += B[j] * v[j]; da += B[j] * f[j]; }
  e.qacc_ws = e.qacc;  // mj_advance saves the last evaluation's qacc for the warmstart
  wsync();
  for (int k = l; k < nq; k += 64) e.qpos[k] = q0[k];
  if (dl) { dxv[l] = dv; e.qvel[l] = v[0] + h * da; }
  wsync();
  integrate_pos(m, e.qpos, dxv, h);
  e.time = t0 + h;
}

template <typename T>
__device__ __forceinline__ void euler(const DevModel<T>& m, Env<T>& e) {
  int l = lane_id();
  bool damp = false;
  for (int k = 0; k < m.nv; k++) damp |= m.dof_damping[k] > 0;
  T qa;
  if (!damp) qa = e.qacc;
  else {
    T di = factor_ld(m, e, e.qMH);
    qa = solve_M(m, e, e.qMH, di, e.qfrc_smooth + e.qfrc_constraint);
  }
  if (l < m.nv) e.qvel[l] += m.timestep * qa;
  wsync();
  integrate_pos(m, e.qpos, e.qvel, m.timestep);
  e.time += m.timestep;
}

// ---------------------------------------------------------------- forward + step
// NT: the model's solver is Newton (compile-time, so PGS kernels do not carry it)
template <typename T, bool NT>
__device__ __forceinline__ void forward(const DevModel<T>& m, Env<T>& e) {
  // phase A (kinematics .. velocity) uses the LDS union region; phase B (constraint rows)
  // overwrites it with the B matrix once collision has consumed the geom frames
  MGX_STAMP_DECL
  kinematics(m, e);
  MGX_STAMP(0);
  com_crb(m, e);
  MGX_STAMP(1);
  e.diaginv = factor_ld(m, e, e.qLD);
  MGX_STAMP(2);
  velocity(m, e);
  MGX_STAMP(3);
  e.qacc_smooth = solve_M(m, e, e.qLD, e.diaginv, e.qfrc_smooth);
  MGX_STAMP(4);
  collision(m, e);
  MGX_STAMP(5);
  make_constraint(m, e);
  MGX_STAMP(6);
  // D^-1/2 per dof for the row transform
  if (lane_id() < m.nv) e.vec0[lane_id()] = sqrt(e.diaginv);
  wsync();
  transform_rows(m, e);
  MGX_STAMP(7);
  if constexpr (NT) newton(m, e);
  else pgs(m, e);
  MGX_STAMP(8);
#ifdef MGX_PROFILE
  if (g_mgx_prof && lane_id() == 0) {
    g_mgx_prof[blockIdx.x * 32 + 20] += e.nefc;
    g_mgx_prof[blockIdx.x * 32 + 21] += e.niter;
    g_mgx_prof[blockIdx.x * 32 + 22] += e.ncon;
    g_mgx_prof[blockIdx.x * 32 + 23] += 1;
  }
#endif
}

// returns the number of bad-state resets performed (0..3). RK: the model's integrator is RK4
// (a compile-time choice so Euler kernels do not carry the RK4 stages).
template <typename T, bool RK = false, bool NT = false>
__device__ __forceinline__ int mj_step_env(const DevModel<T>& m, Env<T>& e) {
  int warn = 0;
  if (any_bad(e.qpos, m.nq)) { reset_env(m, e); warn++; }
  if (any_bad(e.qvel, m.nv)) { reset_env(m, e); warn++; }
  forward<T, NT>(m, e);
  if (ballot(lane_id() < m.nv && isbad(e.qacc)) != 0ull) {
    reset_env(m, e);
    warn++;
    forward<T, NT>(m, e);
  }
  if constexpr (RK) {
    rk4<T, NT>(m, e);
    return warn;
  }
  e.qacc_ws = e.qacc;
  MGX_STAMP_DECL
  euler(m, e);
  MGX_STAMP(9);
  return warn;
}

}  // namespace mgx
