// mgx_wide.h — one mj_step for one env with 64 < nv <= 128, executed by one wavefront.
//
// The execution model of mgx_physics.h with two dofs per lane: dof d lives on lane d % 64, in
// register word d / 64 (humanoid_construction: nv 99 = humanoid 36 + crane 3 + ten free blocks
// 60, construction_site.xml). Every stage that is lane-per-body / -geom / -pair / -row
// (kinematics, comPos, CRB, collision, makeConstraint, the row transform, the line search) is
// the mgx_physics.h code itself, which loops over dofs past 64; what changes is everything that
// keeps a dof-indexed vector in registers: the tree-sparse solves, the per-dof forces, the
// Newton solver (gradient, MFMA Hessian in tile-row passes, Cholesky with two rows per lane,
// triangular solves) and RK4's stage vectors. One wave per env keeps every cross-dof step a
// readlane (no cross-wave LDS barrier); the rows B live in per-env global scratch (Layout.gB)
// and the nv x nv Hessian overlays the dead phase-A LDS union (make_layout).
//
// Restates MuJoCo's mj_step [ext] for RK4 + Newton, the combination construction_site.xml:10
// selects (integrator="RK4", the default solver); oracle/mjref.c is the stage-level reference.
#pragma once
#include "mgx_physics.h"

namespace mgx {

template <typename T>
struct WEnv {
  Env<T> e;  // LDS views, contacts, rows; the dof-lane registers of Env are unused
  T qacc_ws[2], qfrc_applied[2], qfrc_smooth[2], qacc_smooth[2], qacc[2], qfrc_constraint[2], diaginv[2];
  int chainlen[2], madr[2];
  uint64_t anc_lo[2], anc_hi[2];  // strict ancestors of dof 64 w + lane among dofs 0..63 / 64..127
};

__device__ __forceinline__ int wdof(int w) { return 64 * w + lane_id(); }

// value of dof k (uniform) from a two-word lane vector
template <typename T>
__device__ __forceinline__ T wread(const T (&x)[2], int k) {
  return k < 64 ? readlane(x[0], k) : readlane(x[1], k - 64);
}
template <typename T>
__device__ __forceinline__ T wdot(const T (&a)[2], const T (&b)[2]) {
  return usum(a[0] * b[0] + a[1] * b[1]);
}

template <typename T>
__device__ __forceinline__ void wenv_bind(const DevModel<T>& m, WEnv<T>& w, char* smem, T* gB) {
  env_bind<T, true, true>(m, w.e, smem, gB);
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const int d = wdof(k);
    const bool ok = d < m.nv;
    w.chainlen[k] = ok ? m.dof_chainlen[d] : 0;
    w.madr[k] = ok ? m.dof_Madr[d] : 0;
    w.anc_lo[k] = ok ? m.dof_ancmask[d] : 0ull;
    w.anc_hi[k] = ok ? m.dof_ancmask_hi[d] : 0ull;
  }
}

template <typename T>
__device__ __forceinline__ void wload_state(const DevModel<T>& m, WEnv<T>& w, const T* gqpos, const T* gqvel,
                                            const T* gqacc, const T* gctrl, const T* gqfrc, const T* gxfrc, const T* gtime,
                                            int env) {
  Env<T>& e = w.e;
  const int l = lane_id();
  for (int k = l; k < m.nq; k += 64) e.qpos[k] = gqpos[(size_t)env * m.nq + k];
  for (int k = l; k < m.nv; k += 64) e.qvel[k] = gqvel[(size_t)env * m.nv + k];
  for (int k = l; k < m.nu; k += 64) e.ctrl[k] = gctrl[(size_t)env * m.nu + k];
  for (int k = l; k < 6 * m.nbody; k += 64) e.xfrc[k] = gxfrc[(size_t)env * 6 * m.nbody + k];
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const int d = wdof(k);
    w.qacc_ws[k] = d < m.nv ? gqacc[(size_t)env * m.nv + d] : (T)0;
    w.qfrc_applied[k] = d < m.nv ? gqfrc[(size_t)env * m.nv + d] : (T)0;
  }
  e.time = gtime[env];
  wsync();
}

template <typename T>
__device__ __forceinline__ void wstore_state(const DevModel<T>& m, WEnv<T>& w, T* gqpos, T* gqvel, T* gqacc, T* gctrl,
                                             T* gqfrc, T* gxfrc, T* gtime, int env) {
  Env<T>& e = w.e;
  wsync();
  const int l = lane_id();
  for (int k = l; k < m.nq; k += 64) gqpos[(size_t)env * m.nq + k] = e.qpos[k];
  for (int k = l; k < m.nv; k += 64) gqvel[(size_t)env * m.nv + k] = e.qvel[k];
  for (int k = l; k < m.nu; k += 64) gctrl[(size_t)env * m.nu + k] = e.ctrl[k];
  for (int k = l; k < 6 * m.nbody; k += 64) gxfrc[(size_t)env * 6 * m.nbody + k] = e.xfrc[k];
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const int d = wdof(k);
    if (d < m.nv) {
      gqacc[(size_t)env * m.nv + d] = w.qacc_ws[k];
      gqfrc[(size_t)env * m.nv + d] = w.qfrc_applied[k];
    }
  }
  if (l == 0) gtime[env] = e.time;
}

// mj_resetData on the LDS copy and the dof registers
template <typename T>
__device__ __forceinline__ void wreset_env(const DevModel<T>& m, WEnv<T>& w) {
  reset_env(m, w.e);
#pragma unroll
  for (int k = 0; k < 2; k++) { w.qacc_ws[k] = 0; w.qfrc_applied[k] = 0; }
}

// ---------------------------------------------------------------- tree-sparse solves
// x <- L'^-1 x: for k = nv-1 .. 0 the ancestors j of k get x[j] -= L[k][j] x[k]
template <typename T>
__device__ __forceinline__ void wsolve_LT(const DevModel<T>& m, const WEnv<T>& w, const T* LD, T (&x)[2]) {
  const int l = lane_id();
  const bool v0 = l < m.nv, v1 = 64 + l < m.nv;
  for (int k = m.nv - 1; k >= 0; k--) {
    const T xk = wread(x, k);
    const uint64_t alo = m.dof_ancmask[k], ahi = m.dof_ancmask_hi[k];
    const int base = m.dof_Madr[k] + m.dof_chainlen[k];
    if (v0 && ((alo >> l) & 1ull)) x[0] -= LD[base - w.chainlen[0]] * xk;
    if (v1 && ((ahi >> l) & 1ull)) x[1] -= LD[base - w.chainlen[1]] * xk;
  }
}
// x <- L^-1 x: for i = 0 .. nv-1 every descendant d of i gets x[d] -= L[d][i] x[i]
template <typename T>
__device__ __forceinline__ void wsolve_L(const DevModel<T>& m, const WEnv<T>& w, const T* LD, T (&x)[2]) {
  const int l = lane_id();
  const bool v0 = l < m.nv, v1 = 64 + l < m.nv;
  const int b0 = w.madr[0] + w.chainlen[0], b1 = w.madr[1] + w.chainlen[1];
  for (int i = 0; i < m.nv; i++) {
    const T xi = wread(x, i);
    const int ci = m.dof_chainlen[i];
    if (i < 64) {
      if (v0 && ((w.anc_lo[0] >> i) & 1ull)) x[0] -= LD[b0 - ci] * xi;
      if (v1 && ((w.anc_lo[1] >> i) & 1ull)) x[1] -= LD[b1 - ci] * xi;
    } else {
      if (v1 && ((w.anc_hi[1] >> (i - 64)) & 1ull)) x[1] -= LD[b1 - ci] * xi;
    }
  }
}
// y = L x
template <typename T>
__device__ __forceinline__ void wmul_L(const DevModel<T>& m, const WEnv<T>& w, const T* LD, const T (&x)[2], T (&y)[2]) {
  const int l = lane_id();
  const bool v0 = l < m.nv, v1 = 64 + l < m.nv;
  const int b0 = w.madr[0] + w.chainlen[0], b1 = w.madr[1] + w.chainlen[1];
  y[0] = x[0];
  y[1] = x[1];
  for (int i = 0; i < m.nv; i++) {
    const T xi = wread(x, i);
    const int ci = m.dof_chainlen[i];
    if (i < 64) {
      if (v0 && ((w.anc_lo[0] >> i) & 1ull)) y[0] += LD[b0 - ci] * xi;
      if (v1 && ((w.anc_lo[1] >> i) & 1ull)) y[1] += LD[b1 - ci] * xi;
    } else {
      if (v1 && ((w.anc_hi[1] >> (i - 64)) & 1ull)) y[1] += LD[b1 - ci] * xi;
    }
  }
}
// y = L' u
template <typename T>
__device__ __forceinline__ void wmul_LT(const DevModel<T>& m, const WEnv<T>& w, const T* LD, const T (&u)[2], T (&y)[2]) {
  const int l = lane_id();
  const bool v0 = l < m.nv, v1 = 64 + l < m.nv;
  y[0] = u[0];
  y[1] = u[1];
  for (int k = 0; k < m.nv; k++) {
    const T uk = wread(u, k);
    const uint64_t alo = m.dof_ancmask[k], ahi = m.dof_ancmask_hi[k];
    const int base = m.dof_Madr[k] + m.dof_chainlen[k];
    if (v0 && ((alo >> l) & 1ull)) y[0] += LD[base - w.chainlen[0]] * uk;
    if (v1 && ((ahi >> l) & 1ull)) y[1] += LD[base - w.chainlen[1]] * uk;
  }
}
// x = M^-1 y
template <typename T>
__device__ __forceinline__ void wsolve_M(const DevModel<T>& m, const WEnv<T>& w, const T* LD, const T (&y)[2], T (&x)[2]) {
  x[0] = y[0];
  x[1] = y[1];
  wsolve_LT(m, w, LD, x);
  x[0] *= w.diaginv[0];
  x[1] *= w.diaginv[1];
  wsolve_L(m, w, LD, x);
}

// ---------------------------------------------------------------- helper waves
// k_construction (step) and k_wide_step run two waves per env (the kernels use all 512 registers of
// a wave, so one wave per SIMD; two envs per CU by LDS): wave 0 executes the step (every stage of
// this file), wave 1 waits in team_helper and takes shares of the row- and tile-parallel
// passes of the Newton solver (MFMA Hessian tile-row passes, J p, gradient, Cholesky panel and
// trailing update) and of the row transform. Every wsync() of wave 0 is a workgroup barrier that
// the helpers consume; a section is: wave 0 posts the command in LDS -> barrier -> every wave runs
// its share (no barriers inside) -> barrier -> wave 0 clears the command. Shares split the same
// loops by chunk (chunk c to wave c mod nw), so a one-wave launch (nw = 1: the debug kernel, the
// reset) runs the identical code with every chunk on wave 0 and the same results.
// (team_begin / team_end / TEAM_* in mgx_physics.h)

// ---------------------------------------------------------------- Newton Hessian on MFMA
// H = I + sum_{x_r<0} D_r B_r B_r' for nv <= 128 (8 tile rows of 16): the lower tiles of tile
// rows [T0, T1) per pass, so the accumulators of one pass stay in registers (hessian_mfma's
// fragment layout, mgx_physics.h); passes over tile rows beyond the model's are skipped.
// GRAD (16 T1 >= nv): the pass also accumulates sum_{x<0} D x B_r over every dof column and returns
// it as the two-word lane vector (dof l, dof 64 + l) in g (hessian_mfma's fused gradient).
template <typename T, int T0, int T1, bool GRAD = false>
__device__ __forceinline__ void whess_pass(const T* Bm, int Bs, const T* efc, int ne, int nv, T* H, T* g = nullptr) {
  typedef T V4 __attribute__((ext_vector_type(4)));
  constexpr int NT = (T1 * (T1 + 1) - T0 * (T0 + 1)) / 2;
  const int l = lane_id(), i = l & 15, kq = l >> 4;
  const int nt = (nv + 15) >> 4;
  if (!GRAD && T0 >= nt) return;
  T gp[T1];
#pragma unroll
  for (int t = 0; t < T1; t++) gp[t] = 0;
  auto row_of = [&](int v) { return sizeof(T) == 8 ? kq + 4 * v : 4 * kq + v; };
  V4 acc[NT];
#pragma unroll
  for (int t = T0, q = 0; t < T1; t++)
#pragma unroll
    for (int u = 0; u <= t; u++, q++)
#pragma unroll
      for (int v = 0; v < 4; v++) acc[q][v] = (t == u && row_of(v) == i) ? (T)1 : (T)0;
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
      b[t] = (sc != (T)0 && c < nv) ? Bm[r * Bs + c] : (T)0;  // inactive rows: not streamed
    }
  };
  constexpr int HD = 2;  // chunks in flight (the register budget of the wide kernels)
  T bq[HD][T1], sq[HD], gq[HD];
#pragma unroll
  for (int d = 0; d < HD; d++) load(4 * d, bq[d], sq[d], gq[d]);
  for (int r0 = 0; r0 < ne; r0 += 4) {
    T b[T1];
#pragma unroll
    for (int t = 0; t < T1; t++) b[t] = bq[0][t];
    const T sc = sq[0], sg = gq[0];
#pragma unroll
    for (int d = 0; d + 1 < HD; d++) {
      sq[d] = sq[d + 1];
      gq[d] = gq[d + 1];
#pragma unroll
      for (int t = 0; t < T1; t++) bq[d][t] = bq[d + 1][t];
    }
    load(r0 + 4 * HD, bq[HD - 1], sq[HD - 1], gq[HD - 1]);
    if (__ballot(sc != (T)0) == 0ull) continue;  // four inactive rows: no MFMAs
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
        if (t < nt && row < nv && col <= row) H[hidx<true>(row, col, nv)] = acc[q][v];
      }
  if constexpr (GRAD) {
    // lane l = 16 kq + i: dof l is tile column kq, dof 64 + l tile column 4 + kq
    T g0 = 0, g1 = 0;
#pragma unroll
    for (int t = 0; t < T1; t++) {
      const T s = xor_sum_kq(gp[t]);
      g0 = kq == t ? s : g0;
      g1 = kq + 4 == t ? s : g1;
    }
    g[0] = l < nv ? g0 : (T)0;
    g[1] = 64 + l < nv ? g1 : (T)0;
  }
}

// pass q of the four to wave q mod nw; the gradient rides on pass 2 (dof columns 0..111, nv <= 112:
// construction, wave 0) or pass 3 (every column), into g (the owning wave's registers)
__device__ __forceinline__ int whess_grad_pass(int nv) { return nv <= 112 ? 2 : 3; }
template <typename T>
__device__ __forceinline__ void whess_share(const T* Bm, int Bs, const T* efc, int ne, int nv, T* H, int wv, int nw,
                                            T* g) {
  const int qg = whess_grad_pass(nv);
  for (int q = wv; q < 4; q += nw) {
    if (q == 0) whess_pass<T, 0, 4>(Bm, Bs, efc, ne, nv, H);       // 10 tiles
    else if (q == 1) whess_pass<T, 4, 6>(Bm, Bs, efc, ne, nv, H);  // 11 tiles
    else if (q == 2) {                                             // 7 tiles
      if (qg == 2) whess_pass<T, 6, 7, true>(Bm, Bs, efc, ne, nv, H, g);
      else whess_pass<T, 6, 7>(Bm, Bs, efc, ne, nv, H);
    } else {  // 8 tiles
      if (qg == 3) whess_pass<T, 7, 8, true>(Bm, Bs, efc, ne, nv, H, g);
      else whess_pass<T, 7, 8>(Bm, Bs, efc, ne, nv, H);
    }
  }
}

// blocked Cholesky of the packed H (chol_blocked's pieces): diagonal block on wave 0, the panel's
// 64-row sets and the trailing tiles shared
template <typename T>
__device__ __forceinline__ void wchol(WEnv<T>& w, T* H, int nv) {
  const int nb = (nv + 15) >> 4;
  for (int kb = 0; kb < nb; kb++) {
    chol_diag<T, true>(H, nv, kb);
    team_begin(w.e, TEAM_PANEL, kb);
    chol_panel<T, true>(H, nv, kb, 0, w.e.nw);
    team_end(w.e);
    if (kb + 1 < nb) {
      team_begin(w.e, TEAM_TRAIL, kb);
      chol_trail<T, true>(H, nv, kb, 0, w.e.nw);
      team_end(w.e);
    }
  }
}

// J p for the rows of chunks c0, c0 + cs, ... (MGX_RB rows each); lane 0 stores efc[8 r + 3]
template <typename T>
__device__ __forceinline__ void wjp_share(const Env<T>& e, int nv, int ne, const T (&p)[2], int c0, int cs) {
  const int l = lane_id();
  const bool dl[2] = {l < nv, 64 + l < nv};
  const int lc[2] = {dl[0] ? l : 0, dl[1] ? 64 + l : 0};
  T* efc = e.efc;
  T na[MGX_RB], nb[MGX_RB];  // the next chunk, in flight
  load_rows(na, e.Bm, e.Bs, MGX_RB * c0, ne, lc[0], dl[0]);
  load_rows(nb, e.Bm, e.Bs, MGX_RB * c0, ne, lc[1], dl[1]);
  for (int r0 = MGX_RB * c0; r0 < ne; r0 += MGX_RB * cs) {
    T xa[MGX_RB], xb[MGX_RB];
#pragma unroll
    for (int j = 0; j < MGX_RB; j++) { xa[j] = na[j]; xb[j] = nb[j]; }
    load_rows(na, e.Bm, e.Bs, r0 + MGX_RB * cs, ne, lc[0], dl[0]);
    load_rows(nb, e.Bm, e.Bs, r0 + MGX_RB * cs, ne, lc[1], dl[1]);
#pragma unroll
    for (int j = 0; j < MGX_RB; j += 4) {
      T s0 = xa[j] * p[0] + xb[j] * p[1], s1 = xa[j + 1] * p[0] + xb[j + 1] * p[1];
      T s2 = xa[j + 2] * p[0] + xb[j + 2] * p[1], s3 = xa[j + 3] * p[0] + xb[j + 3] * p[1];
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


// ---------------------------------------------------------------- Newton (mj_solNewton)
// newton() of mgx_physics.h with two-word dof vectors; same whitened coordinates, row scalars
// (q[0] b, q[1] x / force, q[2] R, q[3] B_r.p, q[4] D, q[5] aref, q[6] B damping), the same line
// search and stop rules.
template <typename T>
__device__ __forceinline__ void wnewton(const DevModel<T>& m, WEnv<T>& w) {
  Env<T>& e = w.e;
  const int l = lane_id();
  const int ne = __builtin_amdgcn_readfirstlane(e.nefc);
  const int nv = m.nv;
  const bool dl[2] = {l < nv, 64 + l < nv};
  const int lc[2] = {dl[0] ? l : 0, dl[1] ? 64 + l : 0};
  T sqrtD[2];
#pragma unroll
  for (int k = 0; k < 2; k++) sqrtD[k] = dl[k] ? sqrt(e.qLD[w.madr[k]]) : (T)0;
  if (ne == 0) {
#pragma unroll
    for (int k = 0; k < 2; k++) { w.qacc[k] = w.qacc_smooth[k]; w.qfrc_constraint[k] = 0; }
    e.niter = 0;
    return;
  }
  T qv[2] = {dl[0] ? e.qvel[l] : (T)0, dl[1] ? e.qvel[64 + l] : (T)0};
  T wv[2], ws[2], ww[2], wd[2];
  wmul_L(m, w, e.qLD, qv, wv);
  wmul_L(m, w, e.qLD, w.qacc_smooth, ws);
  wmul_L(m, w, e.qLD, w.qacc_ws, ww);
#pragma unroll
  for (int k = 0; k < 2; k++) {
    wv[k] *= sqrtD[k];
    ws[k] *= sqrtD[k];
    ww[k] *= sqrtD[k];
    wd[k] = dl[k] ? ww[k] - ws[k] : (T)0;
  }
  T* efc = e.efc;
  const T* Bm = e.Bm;
  const int Bs = e.Bs;
  // per row: aref, b = J qacc_smooth - aref, D; x at u = 0 (q[1]) and at the warmstart (q[3])
  T c0 = 0, cw = 0;
  T na[MGX_RD][MGX_RB], nb[MGX_RD][MGX_RB];  // the next batches, in flight
  first_rows(na, Bm, Bs, ne, lc[0], dl[0]);
  first_rows(nb, Bm, Bs, ne, lc[1], dl[1]);
  for (int r0 = 0; r0 < ne; r0 += MGX_RB) {
    T xa[MGX_RB], xb[MGX_RB];
    next_rows(xa, na, Bm, Bs, r0, ne, lc[0], dl[0]);
    next_rows(xb, nb, Bm, Bs, r0, ne, lc[1], dl[1]);
#pragma unroll
    for (int j = 0; j < MGX_RB; j++) {
      const int r = r0 + j;
      if (r < ne) {
        T dv = xa[j] * wv[0] + xb[j] * wv[1], ds = xa[j] * ws[0] + xb[j] * ws[1];
        T dw = xa[j] * wd[0] + xb[j] * wd[1], z = 0;
        wave_sum4(dv, ds, dw, z);
        T* q = efc + 8 * r;
        const T aref = -q[6] * dv - q[5];
        const T b = ds - aref, D = (T)1 / q[2], xw = b + dw;
        if (b < 0) c0 += (T)0.5 * D * b * b;
        if (xw < 0) cw += (T)0.5 * D * xw * xw;
        if (l == 0) { q[5] = aref; q[0] = b; q[1] = b; q[3] = xw; q[4] = D; }
      }
    }
  }
  wsync();
  cw += (T)0.5 * wdot(wd, wd);
  const bool warm = cw < c0;
  T u[2] = {warm ? wd[0] : (T)0, warm ? wd[1] : (T)0};
  if (warm) for (int r = l; r < ne; r += 64) efc[8 * r + 1] = efc[8 * r + 3];
  wsync();
  T* H = e.hess;
  const T scale = (T)1 / (m.meaninertia * (T)(nv > 1 ? nv : 1));
  const T tol = m.tolerance;
  const T eps = sizeof(T) == 4 ? (T)1e-7 : (T)1e-15;
  const int maxit = m.iterations;
  int iter = 0;
  // whitened gradient g = u + sum_{x<0} D x B_r as two partial sums over alternating row chunks
  // (even chunks on wave 0, odd chunks on the helper, its sum via vec1), added in that order with
  // one wave or two — the result does not depend on the launch's wave count
  // H and g = u + sum_{x<0} D x B_r in one set of passes over the active rows at the current point
  // (before the first iteration and after every update: the stop test's gradient, the next
  // iteration's Hessian); the gradient rides on one Hessian pass (whess_share), handed over in vec1
  // when the helper wave ran it
  auto hess_grad = [&](T (&gg)[2]) {
    T gs[2] = {0, 0};
    team_begin(w.e, TEAM_HESS, ne);
    whess_share(Bm, Bs, efc, ne, nv, H, 0, w.e.nw, gs);
    team_end(w.e);
    if (whess_grad_pass(nv) % w.e.nw != 0) {
      gs[0] = dl[0] ? e.vec1[l] : (T)0;
      gs[1] = dl[1] ? e.vec1[64 + l] : (T)0;
    }
    gg[0] = dl[0] ? u[0] + gs[0] : (T)0;
    gg[1] = dl[1] ? u[1] + gs[1] : (T)0;
  };
  T g[2];
  hess_grad(g);
  MGX_STAMP_DECL
  MGX_STAMP(10);  // setup + the first Hessian
  while (iter < maxit) {
    MGX_STAMP(11);  // (the Hessian: hess_grad, stamped with the update)
    wchol(w, H, nv);
    MGX_STAMP(12);  // Cholesky
    // L y = -g, L' p = y
    T rdiag[2];
#pragma unroll
    for (int k = 0; k < 2; k++) rdiag[k] = dl[k] ? (T)1 / H[hidx<true>(64 * k + l, 64 * k + l, nv)] : (T)0;
    T y[2] = {-g[0], -g[1]};
    for (int k = 0; k < nv; k++) {
      const T yk = wread(y, k) * wread(rdiag, k);
#pragma unroll
      for (int wd2 = 0; wd2 < 2; wd2++) {
        const int i = 64 * wd2 + l;
        if (i == k) y[wd2] = yk;
        else if (i < nv && i > k) y[wd2] -= H[hidx<true>(i, k, nv)] * yk;
      }
    }
    T p[2] = {y[0], y[1]};
    for (int k = nv - 1; k >= 0; k--) {
      const T pk = wread(p, k) * wread(rdiag, k);
#pragma unroll
      for (int wd2 = 0; wd2 < 2; wd2++) {
        const int i = 64 * wd2 + l;
        if (i == k) p[wd2] = pk;
        else if (i < k) p[wd2] -= H[hidx<true>(k, i, nv)] * pk;
      }
    }
    p[0] = dl[0] ? p[0] : (T)0;
    p[1] = dl[1] ? p[1] : (T)0;
    MGX_STAMP(13);  // triangular solves
    // J p per row (row-major, wave reductions; row chunks shared, p to the helpers in vec0)
    if (w.e.nw > 1) {
      if (dl[0]) e.vec0[l] = p[0];
      if (dl[1]) e.vec0[64 + l] = p[1];
    }
    team_begin(w.e, TEAM_JP, ne);
    wjp_share(e, nv, ne, p, 0, w.e.nw);
    team_end(w.e);
    MGX_STAMP(14);  // J p
    // line search (newton(), mgx_physics.h: MuJoCo's stop rule)
    const T g0 = wdot(u, p), pp = wdot(p, p);
    T sdof[2];
#pragma unroll
    for (int k = 0; k < 2; k++) sdof[k] = dl[k] ? p[k] * w.diaginv[k] * sqrtD[k] : (T)0;
    wsolve_L(m, w, e.qLD, sdof);
    const T snorm = sqrt(wdot(sdof, sdof));
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
        const bool stall = fabs(nxt - al) <= eps * (1 + fabs(al));
        al = nxt;
        if (stall) break;
      }
    }
    MGX_STAMP(15);  // line search
    u[0] += al * p[0];
    u[1] += al * p[1];
    T dc = 0;
    for (int r = l; r < ne; r += 64) {
      T* q = efc + 8 * r;
      dc += row_cost_change(q[1], al * q[3], q[4]);
      q[1] += al * q[3];
    }
    const T improvement = -scale * (al * g0 + (T)0.5 * al * al * pp + usum(dc));
    iter++;
    wsync();
    hess_grad(g);
    // the gradient rule is on the dof-space gradient L' D^1/2 g
    T sg[2] = {sqrtD[0] * g[0], sqrtD[1] * g[1]}, ga[2];
    wmul_LT(m, w, e.qLD, sg, ga);
    ga[0] = dl[0] ? ga[0] : (T)0;
    ga[1] = dl[1] ? ga[1] : (T)0;
    const bool stop = improvement < tol || scale * sqrt(wdot(ga, ga)) < tol;
    MGX_STAMP(16);  // update, gradient, stop tests
    if (stop) break;
  }
  e.niter = iter;
  for (int r = l; r < ne; r += 64) {
    T* q = efc + 8 * r;
    q[1] = q[1] < 0 ? -q[4] * q[1] : (T)0;
  }
  wsync();
  // qacc = qacc_smooth + L^-1 D^-1/2 u ; qfrc_constraint = L' D^1/2 (sum f_r B_r), with
  // sum f_r B_r = -sum_{x<0} D x B_r = u - g at the final point (the last hess_grad): no row pass
  T v[2] = {dl[0] ? u[0] - g[0] : (T)0, dl[1] ? u[1] - g[1] : (T)0};
  T z[2], sv[2];
#pragma unroll
  for (int k = 0; k < 2; k++) {
    z[k] = dl[k] ? u[k] * w.diaginv[k] * sqrtD[k] : (T)0;
    sv[k] = dl[k] ? sqrtD[k] * v[k] : (T)0;
  }
  wsolve_L(m, w, e.qLD, z);
#pragma unroll
  for (int k = 0; k < 2; k++) w.qacc[k] = w.qacc_smooth[k] + z[k];
  wmul_LT(m, w, e.qLD, sv, w.qfrc_constraint);
  wsync();
}

// ---------------------------------------------------------------- forward + step
// B_r = D^-1/2 L'^-1 J_r' in place, four rows at a time, row-major with two dofs per lane (the
// narrow transform_rows_rm with two-word rows): a readlane sweep over the rows' dof support
// (128-bit, ancestors joining as their descendants are reached), highest dof first.
// Chunks of four rows c0, c0 + cs, ... (the helper-wave share); the caller synchronises.
template <typename T>
__device__ __forceinline__ void wtransform_rows(const DevModel<T>& m, WEnv<T>& w, int ne, int c0, int cs) {
  Env<T>& e = w.e;
  const int l = lane_id(), nv = m.nv;
  const bool v0 = l < nv, v1 = 64 + l < nv;
  T* Bm = e.Bm;
  const int Bs = e.Bs;
  const T s0 = v0 ? e.vec0[l] : (T)0, s1 = v1 ? e.vec0[64 + l] : (T)0;
  for (int r0 = 4 * c0; r0 < ne; r0 += 4 * cs) {
    T x[4][2];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const bool ok = r0 + i < ne;
      x[i][0] = (ok && v0) ? Bm[(r0 + i) * Bs + l] : (T)0;
      x[i][1] = (ok && v1) ? Bm[(r0 + i) * Bs + 64 + l] : (T)0;
    }
    uint64_t sp_lo = ballot(x[0][0] != (T)0 || x[1][0] != (T)0 || x[2][0] != (T)0 || x[3][0] != (T)0);
    uint64_t sp_hi = ballot(x[0][1] != (T)0 || x[1][1] != (T)0 || x[2][1] != (T)0 || x[3][1] != (T)0);
    while (sp_lo | sp_hi) {
      const int k = sp_hi ? 127 - __clzll(sp_hi) : 63 - __clzll(sp_lo);
      if (k >= 64) sp_hi &= ~(1ull << (k - 64)); else sp_lo &= ~(1ull << k);
      const uint64_t alo = m.dof_ancmask[k], ahi = m.dof_ancmask_hi[k];
      sp_lo |= alo;  // ancestors have lower indices: visited later in the sweep
      sp_hi |= ahi;
      const int base = m.dof_Madr[k] + m.dof_chainlen[k];
      const T c0 = (v0 && ((alo >> l) & 1ull)) ? e.qLD[base - w.chainlen[0]] : (T)0;
      const T c1 = (v1 && ((ahi >> l) & 1ull)) ? e.qLD[base - w.chainlen[1]] : (T)0;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const T xk = wread(x[i], k);
        x[i][0] -= c0 * xk;
        x[i][1] -= c1 * xk;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if (r0 + i < ne) {
        if (v0) Bm[(r0 + i) * Bs + l] = x[i][0] * s0;
        if (v1) Bm[(r0 + i) * Bs + 64 + l] = x[i][1] * s1;
      }
    }
  }
}

template <typename T>
__device__ __forceinline__ void wforward(const DevModel<T>& m, WEnv<T>& w) {
  Env<T>& e = w.e;
  MGX_STAMP_DECL
  kinematics(m, e);
  MGX_STAMP(0);
  com_crb(m, e);
  MGX_STAMP(1);
  factor_ld<T, true>(m, e, e.qLD);
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const int d = wdof(k);
    w.diaginv[k] = d < m.nv ? (T)1 / e.qLD[m.dof_Madr[d]] : (T)0;
  }
  MGX_STAMP(2);
  velocity_bodies(m, e);
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const int d = wdof(k);
    w.qfrc_smooth[k] = d < m.nv ? dof_force_applied(m, e, d, w.qfrc_applied[k]) : (T)0;
  }
  MGX_STAMP(3);
  wsolve_M(m, w, e.qLD, w.qfrc_smooth, w.qacc_smooth);
  MGX_STAMP(4);
  collision(m, e);
  MGX_STAMP(5);
  make_constraint(m, e);
  MGX_STAMP(6);
  // D^-1/2 per dof for the row transform
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const int d = wdof(k);
    if (d < m.nv) e.vec0[d] = sqrt(w.diaginv[k]);
  }
  wsync();
  if (MGX_TRANSFORM_LANE_ROW) {
    transform_rows<T, true>(m, e);
  } else {
    const int ne = __builtin_amdgcn_readfirstlane(e.nefc);
    team_begin(w.e, TEAM_XFORM, ne);
    wtransform_rows(m, w, ne, 0, w.e.nw);
    team_end(w.e);
  }
  MGX_STAMP(7);
  wnewton(m, w);
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

// mj_RungeKutta(m, d, 4) [ext] (rk4() of mgx_physics.h with two-word stage vectors)
template <typename T>
__device__ __forceinline__ void wrk4(const DevModel<T>& m, WEnv<T>& w) {
  Env<T>& e = w.e;
  const T A[9] = {(T)0.5, 0, 0, 0, (T)0.5, 0, 0, 0, (T)1};
  const T B[4] = {(T)(1.0 / 6.0), (T)(1.0 / 3.0), (T)(1.0 / 3.0), (T)(1.0 / 6.0)};
  const int l = lane_id(), nq = m.nq, nv = m.nv;
  const bool dl[2] = {l < nv, 64 + l < nv};
  T* q0 = e.rk;
  T* dxv = e.rk + ((nq + 3) & ~3);
  const T h = m.timestep, t0 = e.time;
  for (int k = l; k < nq; k += 64) q0[k] = e.qpos[k];
  T v[4][2], f[4][2];
#pragma unroll
  for (int k = 0; k < 2; k++) {
    v[0][k] = dl[k] ? e.qvel[64 * k + l] : (T)0;
    f[0][k] = dl[k] ? w.qacc[k] : (T)0;
  }
  for (int i = 1; i < 4; i++) {
    T C = 0, dv[2] = {0, 0}, da[2] = {0, 0};
    for (int j = 0; j < i; j++) {
      const T a = A[(i - 1) * 3 + j];
      C += a;
#pragma unroll
      for (int k = 0; k < 2; k++) { dv[k] += a * v[j][k]; da[k] += a * f[j][k]; }
    }
    wsync();
#pragma unroll
    for (int k = 0; k < 2; k++)
      if (dl[k]) dxv[64 * k + l] = dv[k];
    for (int k = l; k < nq; k += 64) e.qpos[k] = q0[k];
    wsync();
    integrate_pos(m, e.qpos, dxv, h);
#pragma unroll
    for (int k = 0; k < 2; k++) {
      v[i][k] = v[0][k] + h * da[k];
      if (dl[k]) e.qvel[64 * k + l] = v[i][k];
    }
    e.time = t0 + C * h;
    wsync();
    wforward(m, w);
#pragma unroll
    for (int k = 0; k < 2; k++) f[i][k] = dl[k] ? w.qacc[k] : (T)0;
  }
  T dv[2] = {0, 0}, da[2] = {0, 0};
  for (int j = 0; j < 4; j++)
#pragma unroll
    for (int k = 0; k < 2; k++) { dv[k] += B[j] * v[j][k]; da[k] += B[j] * f[j][k]; }
#pragma unroll
  for (int k = 0; k < 2; k++) w.qacc_ws[k] = w.qacc[k];  // mj_advance keeps the last evaluation's qacc
  wsync();
  for (int k = l; k < nq; k += 64) e.qpos[k] = q0[k];
#pragma unroll
  for (int k = 0; k < 2; k++)
    if (dl[k]) { dxv[64 * k + l] = dv[k]; e.qvel[64 * k + l] = v[0][k] + h * da[k]; }
  wsync();
  integrate_pos(m, e.qpos, dxv, h);
  e.time = t0 + h;
}

// mj_step for RK4 + Newton; returns the number of bad-state resets (mj_checkPos / Vel / Acc)
template <typename T>
__device__ __forceinline__ int wmj_step(const DevModel<T>& m, WEnv<T>& w) {
  Env<T>& e = w.e;
  int warn = 0;
  if (any_bad(e.qpos, m.nq)) { wreset_env(m, w); warn++; }
  if (any_bad(e.qvel, m.nv)) { wreset_env(m, w); warn++; }
  wforward(m, w);
  const int l = lane_id();
  if (ballot((l < m.nv && isbad(w.qacc[0])) || (64 + l < m.nv && isbad(w.qacc[1]))) != 0ull) {
    wreset_env(m, w);
    warn++;
    wforward(m, w);
  }
  wrk4(m, w);
  return warn;
}

// wave 1 of a two-wave env: one loop iteration per barrier of wave 0 (TEAM_NONE), a share per
// posted section, until wave 0 posts TEAM_EXIT
template <typename T>
__device__ __forceinline__ void team_helper(const DevModel<T>& m, WEnv<T>& w) {
  Env<T>& e = w.e;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l = lane_id(), nv = m.nv;
  for (;;) {
    __syncthreads();
    const int cmd = __builtin_amdgcn_readfirstlane(w.e.ctl[0]);
    if (cmd == TEAM_NONE) continue;
    if (cmd == TEAM_EXIT) break;
    const int a = __builtin_amdgcn_readfirstlane(w.e.ctl[1]);
    if (cmd == TEAM_HESS) {
      T gs[2];
      whess_share(e.Bm, e.Bs, e.efc, a, nv, e.hess, wv, w.e.nw, gs);
      if (whess_grad_pass(nv) % w.e.nw == wv) {  // this wave ran the gradient's pass
        e.vec1[l] = gs[0];
        e.vec1[64 + l] = gs[1];
      }
    } else if (cmd == TEAM_PANEL) {
      chol_panel<T, true>(e.hess, nv, a, wv, w.e.nw);
    } else if (cmd == TEAM_TRAIL) {
      chol_trail<T, true>(e.hess, nv, a, wv, w.e.nw);
    } else if (cmd == TEAM_JP) {
      const T p[2] = {l < nv ? e.vec0[l] : (T)0, 64 + l < nv ? e.vec0[64 + l] : (T)0};
      wjp_share(e, nv, a, p, wv, w.e.nw);
    } else if (cmd == TEAM_XFORM) {
      wtransform_rows(m, w, a, wv, w.e.nw);
    } else if (cmd == TEAM_CONTACT) {  // every other contact's rows (make_constraint)
      bool ovf;
      contact_rows_share(m, e, a, __builtin_amdgcn_readfirstlane(w.e.ctl[2]), wv, w.e.nw, ovf);
    }
    __syncthreads();
  }
}

}  // namespace mgx
