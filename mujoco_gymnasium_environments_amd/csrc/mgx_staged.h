// mgx_staged.h — the staged soccer step: row builder -> lane-group PGS -> finisher.
//
// The monolithic kernel (mgx_soccer.h + mgx_physics.h, one wave per env for the whole step)
// holds the Delassus factor B in LDS for the PGS sweeps: 52 KB per env caps the chip at 3
// envs per CU and leaves the serial 50-sweep solve latency-bound. The staged step splits the
// same mj_step at the solver:
//
//   S1  k_soccer_rows   wave per slot   pre-logic, kinematics .. collision, constraint rows;
//                                       B rows + row scalars -> HBM, carry -> HBM (27 KB LDS)
//   S2  k_pgs_groups    16 lanes / slot PGS sweeps with B streamed from L2/MALL, v = B'f in
//                                       registers (lane j holds dofs j, j+16, ...), 4 slots/wave
//   S3  k_soccer_finish wave per env    qacc, checkAcc, Euler, post-logic, autoreset (7 KB LDS)
//   S4  k_soccer_fixup  wave per listed env, monolithic: reset whose bank was not ready
//
// Same-step autoreset without a serial 10-step settle on the critical path: a reset depends
// only on (seed, global env, episode) (Philox draws, zero controls), so each env keeps R
// "banks" — the post-settle states of its next R episodes — and every launch advances the
// unfinished banks by one settle step as extra slots of the same pipeline. A terminating env
// installs its ready bank (soccer_env.py:347-396 outcome: qpos/qvel/warmstart/time, obs,
// prev snapshots, wind) and that bank restarts for episode + R. A bank that is not ready
// falls back to the monolithic reset in S4 (deterministic per env either way).
#pragma once
#include "mgx_soccer.h"

namespace mgx {

#define MGX_PGS_LPE 16         // lanes per slot in the solver kernel
#define MGX_SCAL 8             // row scalars: b, f, R, 1/AR, AR/2, then 3 slots of the block's A_ij
#define MGX_BPAD 24            // B rows past max_nefc: the solver prefetches up to 3 blocks ahead
enum { FIX_RESET = 2 };

// Workspace layout (byte offsets from base), computed on the host (mgx_soccer_workspace_bytes)
struct Pipe {
  char* base;
  int N, R, S, maxE, dpl, nv;
  int carry_stride;    // reals per slot: carry_reals (64-aligned) + 5 * 64 registers
  int carryi_stride;   // ints per slot: carry_ints + 8
  int brow;            // reals per B row (16 * dpl)
  size_t o_carry, o_carryi, o_ne, o_niter, o_k2list, o_ctr, o_fix, o_scal, o_B, o_vout;
  size_t o_bq, o_bv, o_ba, o_btime, o_bobs, o_bprev, o_bwind, o_bk, o_bep, o_bwarn, o_bseed;
  // the checkAcc template: mj_step's outcome after mj_resetData (state + forward frames)
  size_t o_tq, o_tv, o_ta, o_tt, o_tx, o_txq, o_tsc, o_tn, o_tcg, o_tcd, o_tcm;
  int maxC;
  template <typename X> __device__ __forceinline__ X* at(size_t off) const { return reinterpret_cast<X*>(base + off); }
  __device__ __forceinline__ int* ctr() const { return at<int>(o_ctr); }  // [0] fixup count, [1] solver-list count
};

// ------------------------------------------------------------------ S1 helpers
// Row metadata (limits, then contacts in contact order) + impedance: the metadata half of
// make_constraint (mgx_physics.h), J rows are produced per chunk by build_chunk.
template <typename T>
__device__ __forceinline__ void rows_meta(const DevModel<T>& m, Env<T>& e) {
  int l = lane_id();
  const Layout& L = m.L;
  int nefc = 0;
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
        e.efc[8 * r + 1] = side == 0 ? (T)1 : (T)-1;
      }
      r++;
    }
    nefc += total;
  }
  if (nefc > L.max_nefc) { nefc = L.max_nefc; e.overflow |= 4; }
  // contacts: row offsets by a scan over contacts, lane per contact
  for (int base = 0; base < e.ncon; base += 64) {
    int c = base + l;
    int nrow = 0;
    if (c < e.ncon) nrow = m.pair_condim[e.con_pair[c]] == 1 ? 1 : 4;
    int total;
    int off = wave_excl_scan(nrow, &total);
    int adr = nefc + off;
    bool fits = adr + nrow <= L.max_nefc;
    if (c < e.ncon) {
      e.con_efcadr[c] = fits ? adr : -1;
      if (fits) {
        int p = e.con_pair[c];
        int g1 = e.con_geom[2 * c], g2 = e.con_geom[2 * c + 1];
        int b1 = m.geom_bodyid[g1], b2 = m.geom_bodyid[g2];
        T tran = m.body_invweight0[2 * b1] + m.body_invweight0[2 * b2];
        for (int i = 0; i < nrow; i++) {
          int r = adr + i;
          T f = nrow == 1 ? (T)0 : m.pair_friction[5 * p + (i >> 1)];
          e.efc_type[r] = nrow == 1 ? C_CONTACT_FRICTIONLESS : C_CONTACT_PYRAMIDAL;
          e.efc_id[r] = c;
          e.efc[8 * r + 7] = e.con_dist[c];
          e.efc_margin[r] = m.pair_margin[p] - m.pair_gap[p];
          e.efc[8 * r + 2] = tran + f * f * tran;
        }
      }
    }
    // MuJoCo stops adding rows at the first contact that does not fit; row offsets grow with
    // the contact index, so every later contact is dropped too
    unsigned long long bad = ballot(c < e.ncon && !fits);
    if (bad) {
      nefc = readlane(adr, __builtin_ctzll(bad));
      e.overflow |= 4;
      break;
    }
    nefc += total;
  }
  e.nefc = __builtin_amdgcn_readfirstlane(nefc);
  wsync();
  for (int r = l; r < e.nefc; r += 64) {
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

// J rows [c0, c1) into the chunk buffer (row r at Bm + (r - c0) * Bs)
template <typename T>
__device__ __forceinline__ void build_chunk(const DevModel<T>& m, Env<T>& e, int c0, int c1) {
  int l = lane_id();
  int r = c0 + l;
  if (r < c1) {
    T* row = e.Bm + (r - c0) * e.Bs;
    for (int k = 0; k < m.nv; k++) row[k] = 0;
    if (e.efc_type[r] == C_LIMIT_JOINT) row[m.jnt_dofadr[e.efc_id[r]]] = e.efc[8 * r + 1];
  }
  wsync();
  // contacts whose rows intersect the chunk, lane = dof
  int cfirst = e.efc_type[c0] == C_LIMIT_JOINT ? 0 : e.efc_id[c0];
  cfirst = __builtin_amdgcn_readfirstlane(cfirst);
  for (int c = cfirst; c < e.ncon; c++) {
    int adr = e.con_efcadr[c];
    if (adr < 0 || adr >= c1) break;
    int p = e.con_pair[c];
    int dim = m.pair_condim[p];
    int nrow = dim == 1 ? 1 : 4;
    if (adr + nrow <= c0) continue;
    int g1 = e.con_geom[2 * c], g2 = e.con_geom[2 * c + 1];
    int b1 = m.geom_bodyid[g1], b2 = m.geom_bodyid[g2];
    const T* fr = e.con_frame + 9 * c;
    const T* pos = e.con_pos + 3 * c;
    if (l < m.nv) {
      T j1[3] = {0, 0, 0}, j2[3] = {0, 0, 0};
      const T* cd = e.cdof + 6 * l;
      if (b2 > 0 && body_has_dof(m, b2, l)) {
        int r2 = m.body_rootid[b2];
        T off[3] = {pos[0] - e.subtree_com[3 * r2], pos[1] - e.subtree_com[3 * r2 + 1], pos[2] - e.subtree_com[3 * r2 + 2]}, t[3];
        cross3(t, cd, off);
        j2[0] = cd[3] + t[0]; j2[1] = cd[4] + t[1]; j2[2] = cd[5] + t[2];
      }
      if (b1 > 0 && body_has_dof(m, b1, l)) {
        int r1 = m.body_rootid[b1];
        T off[3] = {pos[0] - e.subtree_com[3 * r1], pos[1] - e.subtree_com[3 * r1 + 1], pos[2] - e.subtree_com[3 * r1 + 2]}, t[3];
        cross3(t, cd, off);
        j1[0] = cd[3] + t[0]; j1[1] = cd[4] + t[1]; j1[2] = cd[5] + t[2];
      }
      T jd[3] = {j2[0] - j1[0], j2[1] - j1[1], j2[2] - j1[2]};
      T cj0 = fr[0] * jd[0] + fr[1] * jd[1] + fr[2] * jd[2];
      T val[4];
      if (dim == 1) {
        val[0] = cj0;
      } else {
        T cj1 = fr[3] * jd[0] + fr[4] * jd[1] + fr[5] * jd[2];
        T cj2 = fr[6] * jd[0] + fr[7] * jd[1] + fr[8] * jd[2];
        T mu0 = m.pair_friction[5 * p], mu1 = m.pair_friction[5 * p + 1];
        val[0] = cj0 + mu0 * cj1; val[1] = cj0 - mu0 * cj1; val[2] = cj0 + mu1 * cj2; val[3] = cj0 - mu1 * cj2;
      }
      for (int i = 0; i < nrow; i++) {
        int rr = adr + i;
        if (rr >= c0 && rr < c1) e.Bm[(rr - c0) * e.Bs + l] = val[i];
      }
    }
  }
  wsync();
}

// S1 body: forward up to the constraint rows, rows -> pipe, carry -> pipe
template <typename T>
__device__ __forceinline__ void stage_rows(const DevModel<T>& m, Env<T>& e, const Pipe& P, int slot, int warn) {
  int l = lane_id();
  const int nv = m.nv;
  MGX_STAMP_DECL
  kinematics(m, e);
  MGX_STAMP(0);
  com_crb(m, e);
  MGX_STAMP(1);
  e.diaginv = factor_ld(m, e.qLD);
  MGX_STAMP(2);
  velocity(m, e);
  MGX_STAMP(3);
  e.qacc_smooth = solve_M(m, e, e.qLD, e.diaginv, e.qfrc_smooth);
  MGX_STAMP(4);
  collision(m, e);
  MGX_STAMP(5);
  rows_meta(m, e);
  MGX_STAMP(6);
  const int ne = e.nefc;
  const bool dl = l < nv;
  if (ne > 0) {
    T sqrtD = dl ? sqrt(e.qLD[m.dof_Madr[l]]) : (T)0;
    T qv = dl ? e.qvel[l] : (T)0;
    T wv = sqrtD * mul_L(m, e, e.qLD, qv);
    T ws = sqrtD * mul_L(m, e, e.qLD, e.qacc_smooth);
    T ww = sqrtD * mul_L(m, e, e.qLD, e.qacc_ws);
    wsync();
    if (dl) { e.vec0[l] = wv; e.vec1[l] = ws; e.vec2[l] = ww; e.vec3[l] = sqrt(e.diaginv); }
    wsync();
    T* scal = P.at<T>(P.o_scal) + (size_t)slot * P.maxE * MGX_SCAL;
    T* Bo = P.at<T>(P.o_B) + (size_t)slot * (P.maxE + MGX_BPAD) * P.brow;
    const int CH = m.L.chunk_rows;
    for (int c0 = 0; c0 < ne; c0 += CH) {
      int c1 = c0 + CH < ne ? c0 + CH : ne;
      build_chunk(m, e, c0, c1);
      int r = c0 + l;
      if (r < c1) {
        // B_r = D^-1/2 L'^-1 J_r' in place (transform_rows), then the row scalars of pgs()
        T* x = e.Bm + (r - c0) * e.Bs;
        for (int k = nv - 1; k >= 0; k--) {
          T xk = x[k];
          int a = m.dof_Madr[k] + 1;
          int mk = m.dof_chainlen[k] - 1;
          for (int t = 1; t <= mk; t++) x[m.dof_anc[k * MGX_MAX_DEPTH + t]] -= e.qLD[a + t - 1] * xk;
          x[k] = xk * e.vec3[k];
        }
        T dv = 0, ds = 0, dw = 0, nn = 0;
        for (int k = 0; k < nv; k++) {
          T xx = x[k];
          dv += xx * e.vec0[k]; ds += xx * e.vec1[k]; dw += xx * e.vec2[k]; nn += xx * xx;
        }
        const T* q = e.efc + 8 * r;
        T aref = -q[6] * dv - q[5];
        T Rr = q[2];
        T jar = dw - aref;
        T ad = nn + Rr;
        T* o = scal + r * MGX_SCAL;
        o[0] = ds - aref;
        o[1] = jar < 0 ? -jar / Rr : (T)0;
        o[2] = Rr;
        o[3] = (T)1 / ad;
        o[4] = (T)0.5 * ad;  // the solver's cost change is delta * (delta * AR / 2 + res)
      }
      wsync();
      // block Gauss-Seidel couplings A_ij = B_i.B_j (j < i) of each 4-row block in the chunk:
      // row 4b holds A10 A20 A21 in slots 5..7, row 4b+1 holds A30 A31 A32
      if (4 * l < c1 - c0) {
        int rb0 = 4 * l;
        const T* x0 = e.Bm + rb0 * e.Bs;
        bool h1 = c0 + rb0 + 1 < c1, h2 = c0 + rb0 + 2 < c1, h3 = c0 + rb0 + 3 < c1;
        T a10 = 0, a20 = 0, a21 = 0, a30 = 0, a31 = 0, a32 = 0;
        for (int k = 0; k < nv; k++) {
          T y0 = x0[k];
          T y1 = h1 ? x0[e.Bs + k] : (T)0, y2 = h2 ? x0[2 * e.Bs + k] : (T)0, y3 = h3 ? x0[3 * e.Bs + k] : (T)0;
          a10 += y1 * y0; a20 += y2 * y0; a21 += y2 * y1; a30 += y3 * y0; a31 += y3 * y1; a32 += y3 * y2;
        }
        T* o = scal + (c0 + rb0) * MGX_SCAL;
        o[5] = a10; o[6] = a20; o[7] = a21;
        if (h1) { o[MGX_SCAL + 5] = a30; o[MGX_SCAL + 6] = a31; o[MGX_SCAL + 7] = a32; }
        else { o[MGX_SCAL + 5] = 0; o[MGX_SCAL + 6] = 0; o[MGX_SCAL + 7] = 0; }
      }
      wsync();
      // B rows out, lane = dof, zero padded to brow
      if (l < P.brow)
        for (int rr = c0; rr < c1; rr++) Bo[(size_t)rr * P.brow + l] = dl ? e.Bm[(rr - c0) * e.Bs + l] : (T)0;
      wsync();
    }
  }
  MGX_STAMP(7);
  // carry + registers + ints
  T* cr = P.at<T>(P.o_carry) + (size_t)slot * P.carry_stride;
  for (int k = l; k < m.L.carry_reals; k += 64) cr[k] = reinterpret_cast<T*>(e.qpos)[k - m.L.qpos];
  T* rg = cr + ((m.L.carry_reals + 63) & ~63);
  rg[l] = e.qacc_ws; rg[64 + l] = e.qfrc_applied; rg[128 + l] = e.qfrc_smooth; rg[192 + l] = e.qacc_smooth;
  if (l == 0) rg[256] = e.time;
  int* ci = P.at<int>(P.o_carryi) + (size_t)slot * P.carryi_stride;
  for (int k = l; k < 2 * e.ncon; k += 64) ci[k] = e.con_geom[k];
  int* cx = ci + m.L.carry_ints;
  if (l == 0) {
    cx[0] = e.ncon; cx[1] = ne; cx[2] = e.overflow; cx[3] = warn;
    P.at<int>(P.o_ne)[slot] = ne;
#ifdef MGX_PROFILE
    if (g_mgx_prof && slot < (int)gridDim.x) {
      g_mgx_prof[slot * 32 + 20] += ne;
      g_mgx_prof[slot * 32 + 22] += e.ncon;
      g_mgx_prof[slot * 32 + 23] += 1;
      if ((unsigned long long)ne > g_mgx_prof[slot * 32 + 24]) g_mgx_prof[slot * 32 + 24] = ne;
      g_mgx_prof[slot * 32 + 25] += e.overflow != 0;
    }
#endif
    if (ne > 0) {
      int idx = atomicAdd(P.ctr() + 1, 1);
      P.at<int>(P.o_k2list)[idx] = slot;
    }
  }
}

// ------------------------------------------------------------------ S2: lane-group PGS
template <int CTRL>
__device__ __forceinline__ float dpp_row(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
// sum over the 16 lanes of a DPP row; every lane of the row gets the identical total
__device__ __forceinline__ float row16_sum(float x) {
  x += dpp_row<0xB1>(x);   // quad_perm 1,0,3,2
  x += dpp_row<0x4E>(x);   // quad_perm 2,3,0,1
  x += dpp_row<0x141>(x);  // row_half_mirror
  x += dpp_row<0x140>(x);  // row_mirror
  return x;
}
// four independent 16-lane sums, DPP steps interleaved to fill each other's hazard slots
__device__ __forceinline__ void row16_sum4(float& a, float& b, float& c, float& d) {
#define MGX_R4(CTRL) a += dpp_row<CTRL>(a); b += dpp_row<CTRL>(b); c += dpp_row<CTRL>(c); d += dpp_row<CTRL>(d);
  MGX_R4(0xB1)
  MGX_R4(0x4E)
  MGX_R4(0x141)
  MGX_R4(0x140)
#undef MGX_R4
}
__device__ __forceinline__ void row16_sum4(double& a, double& b, double& c, double& d);
__device__ __forceinline__ double row16_sum(double x) {
  x += __shfl_xor(x, 1);
  x += __shfl_xor(x, 2);
  x += __shfl_xor(x, 4);
  x += __shfl_xor(x, 8);
  return x;
}
__device__ __forceinline__ void row16_sum4(double& a, double& b, double& c, double& d) {
  a = row16_sum(a); b = row16_sum(b); c = row16_sum(c); d = row16_sum(d);
}

// Gauss-Seidel sweeps of mj_solPGS [ext] for 4 slots per wave, 16 lanes per slot. Row
// scalars live in LDS (8 per row); B rows stream from the pipe (row-major, 16*DPL reals, lane j
// reads dofs j + 16d) through a 4-block register ring, 3 blocks (12 rows) ahead of use. Rows
// go in blocks of 4: the four B_r.v use the pre-block v (interleaved reductions) and row i adds
// sum_{j<i} A_ij delta_j with A_ij = B_i.B_j from the row builder -> the sequential
// Gauss-Seidel update in a quarter of the reduction latency. Results per slot do not depend
// on which slots share the wave (other slots only add masked no-op rows / sweeps).
template <typename T, int DPL>
__device__ __forceinline__ void pgs_load_block(T (&dst)[4][DPL], const T* Bs, int r0, int brow) {
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int d = 0; d < DPL; d++) dst[i][d] = Bs[(size_t)(r0 + i) * brow + 16 * d];
  __builtin_amdgcn_sched_barrier(0);  // keep the prefetch where it is issued
}

template <typename T, int DPL>
__device__ __forceinline__ void pgs_block(T (&bb)[4][DPL], T (&v)[DPL], T* sc, int r0, int ne, bool act, T& impr) {
  const bool ok0 = act && r0 < ne, ok1 = act && r0 + 1 < ne, ok2 = act && r0 + 2 < ne, ok3 = act && r0 + 3 < ne;
  T d0 = 0, d1 = 0, d2 = 0, d3 = 0;
#pragma unroll
  for (int d = 0; d < DPL; d++) {
    bb[0][d] = ok0 ? bb[0][d] : (T)0;
    bb[1][d] = ok1 ? bb[1][d] : (T)0;
    bb[2][d] = ok2 ? bb[2][d] : (T)0;
    bb[3][d] = ok3 ? bb[3][d] : (T)0;
    d0 += bb[0][d] * v[d]; d1 += bb[1][d] * v[d]; d2 += bb[2][d] * v[d]; d3 += bb[3][d] * v[d];
  }
  row16_sum4(d0, d1, d2, d3);
  T* q0 = sc + r0 * MGX_SCAL;
  const T a10 = q0[5], a20 = q0[6], a21 = q0[7], a30 = q0[MGX_SCAL + 5], a31 = q0[MGX_SCAL + 6], a32 = q0[MGX_SCAL + 7];
  T dl0, dl1, dl2, dl3;
#define MGX_PGS_ROW(I, OK, DOT, DL)                                      \
  {                                                                      \
    T* q = q0 + (I) * MGX_SCAL;                                          \
    T br = q[0], fr = q[1], Rr = q[2], ai = q[3], hd = q[4];             \
    T res = br + (DOT) + Rr * fr;                                        \
    T fn = fr - res * ai;                                                \
    fn = fn < 0 ? (T)0 : fn;                                             \
    T delta = fn - fr;                                                   \
    T change = delta * (delta * hd + res);                               \
    bool keep = !(OK) || change > (T)1e-10;                              \
    DL = keep ? (T)0 : delta;                                            \
    impr -= keep ? (T)0 : change;                                        \
    q[1] = keep ? fr : fn;                                               \
  }
  MGX_PGS_ROW(0, ok0, d0, dl0)
  MGX_PGS_ROW(1, ok1, d1 + a10 * dl0, dl1)
  MGX_PGS_ROW(2, ok2, d2 + a20 * dl0 + a21 * dl1, dl2)
  MGX_PGS_ROW(3, ok3, d3 + a30 * dl0 + a31 * dl1 + a32 * dl2, dl3)
#undef MGX_PGS_ROW
#pragma unroll
  for (int d = 0; d < DPL; d++) v[d] += dl0 * bb[0][d] + dl1 * bb[1][d] + dl2 * bb[2][d] + dl3 * bb[3][d];
}

template <typename T, int DPL>
__global__ void __launch_bounds__(64) k_pgs_groups(Pipe P, int maxit, T tol, T scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int l = threadIdx.x, s = l >> 4, j = l & 15;
  if (blockIdx.x == 0 && l == 0) P.ctr()[0] = 0;  // fixup list count, filled by the finisher
  const int cnt = P.ctr()[1];
  const int base = blockIdx.x * 4;
  if (base >= cnt) return;
  const int idx = base + s;
  const int slot = idx < cnt ? P.at<int>(P.o_k2list)[idx] : -1;
  const int ne = slot >= 0 ? P.at<int>(P.o_ne)[slot] : 0;
  const int sstride = MGX_SCAL * P.maxE + 4;
  T* sc = reinterpret_cast<T*>(smem) + s * sstride;
  const T* gsc = P.at<T>(P.o_scal) + (size_t)(slot >= 0 ? slot : 0) * P.maxE * MGX_SCAL;
  for (int q = j; q < ne * MGX_SCAL; q += 16) sc[q] = gsc[q];
  int nm = ne;
  nm = max(nm, __shfl_xor(nm, 16));
  nm = max(nm, __shfl_xor(nm, 32));
  const int neMax = __builtin_amdgcn_readfirstlane(nm);
  const int ne4 = (neMax + 3) & ~3;
  const int brow = 16 * DPL;
  const T* Bs = P.at<T>(P.o_B) + (size_t)(slot >= 0 ? slot : 0) * (P.maxE + MGX_BPAD) * brow + j;
  __syncthreads();
  // warmstart: v = B' f, dual cost, reset to zero if the cost is positive
  T v[DPL];
#pragma unroll
  for (int d = 0; d < DPL; d++) v[d] = 0;
  for (int r = 0; r < neMax; r++) {
    bool ok = r < ne;
    T f = ok ? sc[r * MGX_SCAL + 1] : (T)0;
#pragma unroll
    for (int d = 0; d < DPL; d++) {
      T b = Bs[(size_t)r * brow + 16 * d];
      v[d] += f * (ok ? b : (T)0);
    }
  }
  T cpart = 0;
  for (int r = 0; r < neMax; r++) {
    bool ok = r < ne;
    T dot = 0;
#pragma unroll
    for (int d = 0; d < DPL; d++) {
      T b = Bs[(size_t)r * brow + 16 * d];
      dot += (ok ? b : (T)0) * v[d];
    }
    dot = row16_sum(dot);
    const T* q = sc + r * MGX_SCAL;
    if (ok) cpart += q[1] * (q[0] + (T)0.5 * (dot + q[2] * q[1]));
  }
  if (cpart > 0) {
    for (int r = j; r < ne; r += 16) sc[r * MGX_SCAL + 1] = 0;
#pragma unroll
    for (int d = 0; d < DPL; d++) v[d] = 0;
  }
  __syncthreads();
  bool act = ne > 0;
  int it = 0;
  for (int iter = 0; iter < maxit; iter++) {
    if (__ballot(act) == 0ull) break;
    T impr = 0;
    T R0[4][DPL], R1[4][DPL], R2[4][DPL], R3[4][DPL];
    pgs_load_block<T, DPL>(R0, Bs, 0, brow);
    pgs_load_block<T, DPL>(R1, Bs, 4, brow);
    pgs_load_block<T, DPL>(R2, Bs, 8, brow);
    // full groups of 4 blocks: no early exit inside, so every prefetch is consumed on every
    // path and the compiler cannot sink the loads next to their use
    int r0 = 0;
    for (; r0 + 16 <= ne4; r0 += 16) {
      pgs_load_block<T, DPL>(R3, Bs, r0 + 12, brow);
      pgs_block<T, DPL>(R0, v, sc, r0, ne, act, impr);
      pgs_load_block<T, DPL>(R0, Bs, r0 + 16, brow);
      pgs_block<T, DPL>(R1, v, sc, r0 + 4, ne, act, impr);
      pgs_load_block<T, DPL>(R1, Bs, r0 + 20, brow);
      pgs_block<T, DPL>(R2, v, sc, r0 + 8, ne, act, impr);
      pgs_load_block<T, DPL>(R2, Bs, r0 + 24, brow);
      pgs_block<T, DPL>(R3, v, sc, r0 + 12, ne, act, impr);
    }
    // 0..3 remaining blocks, already in the ring
    if (r0 < ne4) pgs_block<T, DPL>(R0, v, sc, r0, ne, act, impr);
    if (r0 + 4 < ne4) pgs_block<T, DPL>(R1, v, sc, r0 + 4, ne, act, impr);
    if (r0 + 8 < ne4) pgs_block<T, DPL>(R2, v, sc, r0 + 8, ne, act, impr);
    if (act) {
      it++;
      if (impr * scale < tol) act = false;
    }
  }
  if (slot >= 0) {
    T* vo = P.at<T>(P.o_vout) + (size_t)slot * 64;
#pragma unroll
    for (int d = 0; d < DPL; d++)
      if (j + 16 * d < P.nv) vo[j + 16 * d] = v[d];
    if (j == 0) P.at<int>(P.o_niter)[slot] = it;
  }
}

// ------------------------------------------------------------------ S3 helpers
template <typename T>
__device__ __forceinline__ int load_carry(const DevModel<T>& m, Env<T>& e, const Pipe& P, int slot) {
  int l = lane_id();
  const T* cr = P.at<T>(P.o_carry) + (size_t)slot * P.carry_stride;
  for (int k = l; k < m.L.carry_reals; k += 64) reinterpret_cast<T*>(e.qpos)[k - m.L.qpos] = cr[k];
  const T* rg = cr + ((m.L.carry_reals + 63) & ~63);
  e.qacc_ws = rg[l]; e.qfrc_applied = rg[64 + l]; e.qfrc_smooth = rg[128 + l]; e.qacc_smooth = rg[192 + l];
  e.time = rg[256];
  const int* ci = P.at<int>(P.o_carryi) + (size_t)slot * P.carryi_stride;
  const int* cx = ci + m.L.carry_ints;
  e.ncon = cx[0];
  e.nefc = cx[1];
  e.overflow = cx[2];
  for (int k = l; k < 2 * e.ncon; k += 64) e.con_geom[k] = ci[k];
  wsync();
  return cx[3];
}

// mj_checkAcc's outcome. A bad qacc makes mj_step reset the data (qpos0, zero velocities,
// controls and applied forces), run mj_forward again and integrate: a result that does not
// depend on the env, so it is computed once (k_soccer_template) and loaded here.
template <typename T>
__device__ __forceinline__ void load_template(const DevModel<T>& m, Env<T>& e, const Pipe& P) {
  int l = lane_id();
  wsync();
  for (int k = l; k < m.nq; k += 64) e.qpos[k] = P.at<T>(P.o_tq)[k];
  for (int k = l; k < m.nv; k += 64) e.qvel[k] = P.at<T>(P.o_tv)[k];
  for (int k = l; k < m.nu; k += 64) e.ctrl[k] = 0;
  for (int k = l; k < 6 * m.nbody; k += 64) e.xfrc[k] = 0;
  for (int k = l; k < 3 * m.nbody; k += 64) {
    e.xpos[k] = P.at<T>(P.o_tx)[k];
    e.subtree_com[k] = P.at<T>(P.o_tsc)[k];
  }
  for (int k = l; k < 4 * m.nbody; k += 64) e.xquat[k] = P.at<T>(P.o_txq)[k];
  int nc = P.at<int>(P.o_tn)[0];
  e.ncon = nc;
  for (int k = l; k < nc; k += 64) {
    e.con_geom[2 * k] = P.at<int>(P.o_tcg)[2 * k];
    e.con_geom[2 * k + 1] = P.at<int>(P.o_tcg)[2 * k + 1];
    e.con_dist[k] = P.at<T>(P.o_tcd)[k];
    e.con_mu[k] = P.at<T>(P.o_tcm)[k];
  }
  e.qacc_ws = l < m.nv ? P.at<T>(P.o_ta)[l] : (T)0;
  e.qfrc_applied = 0;
  e.time = P.at<T>(P.o_tt)[0];
  wsync();
}

// qacc from the solver's v, checkAcc, warmstart, Euler. Returns false on a bad qacc (the
// state is then left untouched; the caller loads the template).
template <typename T>
__device__ __forceinline__ bool finish_physics(const DevModel<T>& m, Env<T>& e, const Pipe& P, int slot) {
  int l = lane_id();
  const bool dl = l < m.nv;
  if (e.nefc > 0) {
    T v = dl ? P.at<T>(P.o_vout)[(size_t)slot * 64 + l] : (T)0;
    T D = dl ? e.qLD[m.dof_Madr[l]] : (T)1;
    T sqrtD = sqrt(D);
    T z = dl ? v / sqrtD : (T)0;  // D^-1/2 v
    z = solve_L(m, e, e.qLD, z);
    e.qacc = e.qacc_smooth + z;
    e.qfrc_constraint = mul_LT(m, e, e.qLD, dl ? sqrtD * v : (T)0);
  } else {
    e.qacc = e.qacc_smooth;
    e.qfrc_constraint = 0;
  }
  if (ballot(dl && isbad(e.qacc)) != 0ull) return false;
  e.qacc_ws = e.qacc;
  euler(m, e);
  return true;
}

template <typename T>
__device__ __forceinline__ void copy_g(T* dst, const T* src, int n) {
  for (int k = lane_id(); k < n; k += 64) dst[k] = src[k];
}

// bank (env, b) restarts for `episode`: Philox draws -> mj_resetData + randomised qpos
// (soccer_apply_reset), settle counter 0. Clobbers the Env's state arrays.
template <typename T>
__device__ __forceinline__ void bank_init(const DevModel<T>& m, Env<T>& e, const SoccerIds<T>& ids, const Pipe& P, int env,
                                          int b, int episode, uint64_t seed, int env_offset) {
  int l = lane_id();
  int bi = env * P.R + b;
  soccer_philox_draws(seed, (uint32_t)(env_offset + env), (uint32_t)episode, ids.n_noise, e.vec1);
  wsync();
  soccer_apply_reset(m, e, ids, e.vec1, P.at<T>(P.o_bwind) + 3 * (size_t)bi);
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

// settle finished: the reset's observation and prev snapshots (soccer_env.py:381-396)
template <typename T>
__device__ __forceinline__ void bank_finalize(const DevModel<T>& m, Env<T>& e, const SoccerIds<T>& ids, const Pipe& P, int bi) {
  soccer_obs(m, e, ids, 0, P.at<float>(P.o_bobs) + (size_t)bi * 80);
  int l = lane_id();
  T* pv = P.at<T>(P.o_bprev) + (size_t)bi * 6;
  if (l < 3) { pv[l] = e.xpos[3 * ids.ball + l]; pv[3 + l] = e.xpos[3 * ids.torso + l]; }
}

template <typename T>
__device__ __forceinline__ void bank_store_state(const DevModel<T>& m, Env<T>& e, const Pipe& P, int bi, int warn) {
  wsync();
  int l = lane_id();
  copy_g(P.at<T>(P.o_bq) + (size_t)bi * m.nq, e.qpos, m.nq);
  if (l < m.nv) {
    P.at<T>(P.o_bv)[(size_t)bi * m.nv + l] = e.qvel[l];
    P.at<T>(P.o_ba)[(size_t)bi * m.nv + l] = e.qacc_ws;
  }
  if (l == 0) {
    P.at<T>(P.o_btime)[bi] = e.time;
    P.at<int>(P.o_bwarn)[bi] += warn;
  }
}

// load bank state as an mj_resetData'd MjData (zero controls and applied forces)
template <typename T>
__device__ __forceinline__ void bank_load_state(const DevModel<T>& m, Env<T>& e, const Pipe& P, int bi) {
  int l = lane_id();
  const T* q = P.at<T>(P.o_bq) + (size_t)bi * m.nq;
  for (int k = l; k < m.nq; k += 64) e.qpos[k] = q[k];
  for (int k = l; k < m.nv; k += 64) e.qvel[k] = P.at<T>(P.o_bv)[(size_t)bi * m.nv + k];
  for (int k = l; k < m.nu; k += 64) e.ctrl[k] = 0;
  for (int k = l; k < 6 * m.nbody; k += 64) e.xfrc[k] = 0;
  e.qacc_ws = l < m.nv ? P.at<T>(P.o_ba)[(size_t)bi * m.nv + l] : (T)0;
  e.qfrc_applied = 0;
  e.time = P.at<T>(P.o_btime)[bi];
  wsync();
}

// Install the ready bank of env `env` into its live state and restart the bank for
// episode + R. Returns false if the bank is not ready (caller falls back).
template <typename T>
__device__ __forceinline__ bool bank_install(const DevModel<T>& m, Env<T>& e, const SoccerIds<T>& ids, const Pipe& P,
                                             mgx_state s, mgx_soccer_env ev, float* obs, uint64_t seed, int env_offset,
                                             int env) {
  int l = lane_id();
  int E = ev.episode[env];
  int b = E % P.R;
  int bi = env * P.R + b;
  bool ready = P.at<int>(P.o_bk)[bi] == 10 && P.at<int>(P.o_bep)[bi] == E && P.at<uint64_t>(P.o_bseed)[bi] == seed;
  if (!ready) return false;
  copy_g((T*)s.qpos + (size_t)env * m.nq, P.at<T>(P.o_bq) + (size_t)bi * m.nq, m.nq);
  copy_g((T*)s.qvel + (size_t)env * m.nv, P.at<T>(P.o_bv) + (size_t)bi * m.nv, m.nv);
  copy_g((T*)s.qacc_warmstart + (size_t)env * m.nv, P.at<T>(P.o_ba) + (size_t)bi * m.nv, m.nv);
  for (int k = l; k < m.nv; k += 64) ((T*)s.qfrc_applied)[(size_t)env * m.nv + k] = 0;
  for (int k = l; k < m.nu; k += 64) ((T*)s.ctrl)[(size_t)env * m.nu + k] = 0;
  for (int k = l; k < 6 * m.nbody; k += 64) ((T*)s.xfrc_applied)[(size_t)env * 6 * m.nbody + k] = 0;
  copy_g(obs + (size_t)env * 80, P.at<float>(P.o_bobs) + (size_t)bi * 80, 80);
  const T* pv = P.at<T>(P.o_bprev) + (size_t)bi * 6;
  if (l < 3) {
    ((T*)ev.prev_ball_pos)[3 * (size_t)env + l] = pv[l];
    ((T*)ev.prev_robot_pos)[3 * (size_t)env + l] = pv[3 + l];
    ((T*)ev.wind)[3 * (size_t)env + l] = P.at<T>(P.o_bwind)[3 * (size_t)bi + l];
  }
  if (l < 5) ((T*)ev.stats)[5 * (size_t)env + l] = 0;
  if (l == 0) {
    ((T*)s.time)[env] = P.at<T>(P.o_btime)[bi];
    if (s.warning) s.warning[env] += P.at<int>(P.o_bwarn)[bi];
    ev.step[env] = 0;
    ev.goal_scored[env] = 0;
    ev.episode[env] = E + 1;
  }
  wsync();
  bank_init(m, e, ids, P, env, b, E + P.R, seed, env_offset);
  return true;
}

}  // namespace mgx
