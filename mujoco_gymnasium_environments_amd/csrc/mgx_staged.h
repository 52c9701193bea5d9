// mgx_staged.h — the staged soccer step: row builder -> lane-group PGS -> finisher.
//
// The monolithic kernel (mgx_soccer.h + mgx_physics.h, one wave per env for the whole step)
// holds the Delassus factor B in LDS for the PGS sweeps: 52 KB per env caps the chip at 3
// envs per CU and leaves the serial 50-sweep solve latency-bound. The staged step splits the
// same mj_step at the solver:
//
//   S1  k_soccer_rows   wave per slot   pre-logic, kinematics .. collision, constraint rows;
//                                       B rows + row scalars -> HBM, carry -> HBM (27 KB LDS)
//   S2  k_pgs_groups    16 lanes / slot PGS sweeps, 4 slots / wave, with the slots' B copied
//                                       once into an LDS arena (global-B launch for waves whose
//                                       slots do not fit), v = B'f in registers
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

#define MGX_SCAL 5             // row scalars: b, f, R, 1/AR, AR/2
// scalar layout per 4-row block (20 reals, 16-byte aligned): [b x4][f x4][R x4][1/AR x4][AR/2 x4],
// so the solver reads each quantity of a block with one 16-byte LDS load
#define MGX_SQ(k, i) (4 * (k) + (i))
// Two B layouts per 4-row block (16 bytes of block table each in the pipe), template flag DOFB:
//  * 8-dof groups (DOFB = false; soccer, parkour): [A 8][per touched group: 8 dofs x 4 rows], table
//    of 8 uint16 — the A offset, then one offset per group (0 = the slot's zero group). The solver
//    reads its lane's offsets straight from the table (widened to 8 words in LDS).
//  * dof-granular (DOFB = true; the RK4 bipedal pipeline): [A 8][per support dof: 4 rows], table
//    [B offset, support lo, support hi, 0] (4 uint32). Half the B bytes of the group layout (a
//    contact's support is ~8 dofs, its groups ~2.6 x 8), at ~25 more VALU ops per block to decode
//    a lane's rank: the bipedal solver streams B from HBM and gains, the soccer solver (one wave
//    per SIMD, B from L2 / MALL) measured 3% slower with it.
#define MGX_TW 4  // table words per block in the pipe (16 bytes)
__host__ __device__ constexpr int mgx_twl(bool dofb) { return dofb ? 4 : 8; }  // table words per block in LDS
#define MGX_PGS_LPS 16         // solver: lanes per slot (16 or 64; MGX_PGS_LPS env overrides per process)
#define MGX_PGS_LDS_B 0        // main solver launch: 1 = B in an LDS arena, 0 = B from global memory
#define MGX_PGS_RING 2         // global-B solver: register ring of 4-row blocks (RING - 1 in flight; 3 and 4 measured no faster)
#define MGX_PGS_RING_LDS 2     // LDS-B solver: one block in flight covers the LDS latency
#define MGX_PGS_LDS_ROWS 192   // rows per slot the main solver launch keeps in LDS (2 waves / CU in fp64)
#define MGX_PGS_WIDE_GRID 256  // waves of the global-B launch (slots over MGX_PGS_LDS_ROWS, waves over their arena)
#define MGX_PGS_WIDE_LDS_GRID 32  // waves of the wide launch with LDS-resident B (one slot per wave)
#define MGX_PGS_ARENA_F64 49152  // LDS arena per main-launch solver wave of 4 slots, fp64 (tools/pgs_census.py)
#define MGX_PGS_ARENA_F32 32768  //                                                    fp32
enum { FIX_RESET = 2 };

// Workspace layout (byte offsets from base), computed on the host (mgx_soccer_workspace_bytes)
struct Pipe {
  char* base;
  int N, R, S, maxE, dpl, nv;
  int carry_stride;    // reals per slot: carry_reals (64-aligned) + 5 * 64 registers
  int carryi_stride;   // ints per slot: carry_ints + 8
  int bcap;            // reals per slot of group-compressed B: 32 + (max_nefc / 4) * (8 + 32 * ceil(nv / 8))
  int capE;            // rows the main solver launch holds in LDS per slot; slots with more rows (up
                       // to maxE) go to the second, wide-LDS launch (o_k2big)
  int arena;           // LDS bytes of one main-launch solver wave (scalars + block table + B of its slots)
  int sqg;             // soccer main launch: row scalars read from the pipe, forces only in LDS (capE > 192)
  int prio_rows;       // main launch: a wave whose slots reach more rows than this raises its wave
                       // priority (s_setprio 3): the launch's longest chains issue first on a
                       // shared SIMD (default: capE, i.e. the hmain waves; MGX_PGS_PRIO_ROWS)
  int hmain;           // 1: slots over capE rows stay in the main launch's heaviest-first list; a wave
                       // holding one runs with its row scalars read from the pipe (SQG), whose LDS
                       // (forces + table for maxE rows) fits the wave's capE-row allocation
  int warena;          // > 0: LDS bytes of the wide launch's one-slot waves, which solve a slot of
                       // more than capE rows with its B, scalars and table copied into LDS (the
                       // latency-bound chain of a heavy slot reads LDS instead of L2 / MALL)
  size_t o_cpos;        // contact points of the row builder, 3 * maxC reals per slot (Layout.gcon)
  size_t o_carry, o_carryi, o_ne, o_blen, o_niter, o_k2list, o_k2big, o_ctr, o_fix, o_scal, o_blk, o_B, o_vout;
  // the main solver launch's slots by block count: o_hist[b] slots with b blocks (b = 1 .. nbk - 1),
  // listed in o_blist[b * S ..]; the launch takes them heaviest first (sorted_slot), so a wave's
  // four slots have (nearly) equal sweeps and the longest chains start first. The finisher
  // clears the histogram.
  int nbk;
  size_t o_hist, o_blist;
  size_t o_bq, o_bv, o_ba, o_btime, o_bobs, o_bprev, o_bwind, o_bk, o_bep, o_bwarn, o_bseed;
  // the checkAcc template: mj_step's outcome after mj_resetData (state + forward frames)
  size_t o_tq, o_tv, o_ta, o_tt, o_tx, o_txq, o_tsc, o_tn, o_tcg, o_tcd, o_tcm;
  int maxC;
  int tw;              // block-table words per 4-row block (MGX_TW: B offset, 64-bit dof support)
  int nobs;            // floats of a bank's reset observation
  // RK4 staged step (mgx_rk_staged.h): per slot the stage carry (rk_stride reals: X0 positions,
  // the stage's positions, stage velocities / accelerations, t0 / t_k), its state in the step
  // (o_rks) and the warnings / overflow gathered over its stages (o_rkw); o_tscr: the template
  // kernel's row scratch (monolithic layout with rows in global memory)
  int rk_stride;
  size_t o_rk, o_rks, o_rkw, o_tscr;
  template <typename X> __device__ __forceinline__ X* at(size_t off) const { return reinterpret_cast<X*>(base + off); }
  // [0] fixup count, [1] solver-list count, [2] wide-solver-list count, [3] / [4] the last
  // step's list sizes, [5] RK4 step: fixup count (k_pgs_groups clears [0] at every launch)
  __device__ __forceinline__ int* ctr() const { return at<int>(o_ctr); }
};

// The row builder's carry tail (Layout.carry_lds): con_mu, xfrc_applied and qMH of `slot` are read
// and written in its pipe carry (global memory), where the finisher's load_carry picks them up;
// the contact points (Layout.gcon) in the slot's o_cpos storage, read back by the row blocks.
// Every Env bound with the row-builder layout binds its tail before first use (env_bind leaves
// those pointers null).
template <typename T>
__device__ __forceinline__ void bind_carry_tail(const DevModel<T>& m, Env<T>& e, const Pipe& P, int slot) {
  if (m.L.carry_lds < m.L.carry_reals) {
    T* cr = P.at<T>(P.o_carry) + (size_t)slot * P.carry_stride;
    e.xfrc = cr + (m.L.xfrc - m.L.qpos);
    e.qMH = cr + (m.L.qMH - m.L.qpos);
    e.con_mu = cr + (m.L.con_mu - m.L.qpos);
  }
  if (m.L.gcon) e.con_pos = P.at<T>(P.o_cpos) + (size_t)slot * 3 * P.maxC;
}

// ------------------------------------------------------------------ S1 helpers
// Row plan (mj_makeConstraint order [ext]): joint limits (joint order, lower then upper),
// padded with dummy rows to a multiple of 4, then one 4-row block per contact (the 4 pyramid
// rows; a condim-1 contact uses row 0 and 3 dummies). Dummy rows have B = 0, b = f = 0 and
// never change in the sweeps, so the Gauss-Seidel sequence over the real rows is MuJoCo's.
// The limit list goes to efc_id (code 2*joint + side). Returns nefc (padded).
template <typename T>
__device__ __forceinline__ int rows_plan(const DevModel<T>& m, Env<T>& e, int* nlim_out, int* ncon_out) {
  int l = lane_id();
  const int maxE = m.L.max_nefc;
  int nlim = 0;
  for (int base = 0; base < m.njnt; base += 64) {
    int j = base + l;
    bool lo = false, hi = false;
    if (j < m.njnt && m.jnt_limited[j] && (m.jnt_type[j] == JHINGE || m.jnt_type[j] == JSLIDE)) {
      T val = e.qpos[m.jnt_qposadr[j]], margin = m.jnt_margin[j];
      lo = val - m.jnt_range[2 * j] < margin;
      hi = m.jnt_range[2 * j + 1] - val < margin;
    }
    int total;
    int off = wave_excl_scan((int)lo + (int)hi, &total);
    int r = nlim + off;
    if (lo) { if (r < maxE) e.efc_id[r] = 2 * j; r++; }
    if (hi) { if (r < maxE) e.efc_id[r] = 2 * j + 1; }
    nlim += total;
  }
  if (nlim > maxE) { nlim = maxE; e.overflow |= 4; }
  int nlim4 = (nlim + 3) & ~3;
  int ncf = e.ncon;
  if (nlim4 + 4 * ncf > maxE) { ncf = (maxE - nlim4) / 4; e.overflow |= 4; }
  *nlim_out = nlim;
  *ncon_out = ncf;
  wsync();
  return nlim4 + 4 * ncf;
}

// Per-row constants of mj_makeImpedance [ext], lane per row: R, B (damping of aref),
// K*imp*(pos - margin), 1 for a real row / 0 for padding. They go to the slot's own row-scalar
// area in the pipe (the b, f, R, 1/AR places of the row, overwritten by build_block with the
// final scalars), not to LDS: 4 reals per row would cost the row builder 12 KB of LDS at full
// capacity (384 rows, fp64).
template <typename T>
__device__ __forceinline__ void rows_impedance(const DevModel<T>& m, Env<T>& e, int ne, int nlim, int nlim4, T* scal) {
  const int l = lane_id();
  for (int r = l; r < ne; r += 64) {
    const T *solref = nullptr, *solimp = nullptr;
    T pos = 0, margin = 0, diag = 0;
    if (r < nlim) {
      int code = e.efc_id[r];
      int jn = code >> 1, side = code & 1;
      T val = e.qpos[m.jnt_qposadr[jn]];
      pos = side ? m.jnt_range[2 * jn + 1] - val : val - m.jnt_range[2 * jn];
      margin = m.jnt_margin[jn];
      diag = m.dof_invweight0[m.jnt_dofadr[jn]];
      solref = m.jnt_solref + 2 * jn;
      solimp = m.jnt_solimp + 5 * jn;
    } else if (r >= nlim4) {
      int c = (r - nlim4) >> 2, i = (r - nlim4) & 3;
      int p = e.con_pair[c];
      int dim = m.pair_condim[p];
      if (dim != 1 || i == 0) {
        int b1 = m.geom_bodyid[e.con_geom[2 * c]], b2 = m.geom_bodyid[e.con_geom[2 * c + 1]];
        T tran = m.body_invweight0[2 * b1] + m.body_invweight0[2 * b2];
        T f = dim == 1 ? (T)0 : m.pair_friction[5 * p + (i >> 1)];
        pos = e.con_dist[c];
        margin = m.pair_margin[p] - m.pair_gap[p];
        diag = tran + f * f * tran;
        solref = m.pair_solref + 2 * p;
        solimp = m.pair_solimp + 5 * p;
      }
    }
    T* o = scal + (size_t)(r >> 2) * (4 * MGX_SCAL) + (r & 3);
    if (!solref) {
      o[MGX_SQ(0, 0)] = 1; o[MGX_SQ(1, 0)] = 0; o[MGX_SQ(2, 0)] = 0; o[MGX_SQ(3, 0)] = 0;
      continue;
    }
    T imp = impedance(solimp, pos, margin);
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
    T R = ((T)1 - imp) * diag / imp;
    o[MGX_SQ(0, 0)] = R > minval<T>() ? R : minval<T>();
    o[MGX_SQ(1, 0)] = B;
    o[MGX_SQ(2, 0)] = K * imp * (pos - margin);
    o[MGX_SQ(3, 0)] = 1;
  }
}

// Contact constants of the J build, lane per contact (c < 64), read back with readlane
template <typename T>
struct ContactMeta {
  int dim, b1, b2, rt1, rt2;
  uint64_t m1, m2;
  T mu0, mu1;
};
template <typename T>
__device__ __forceinline__ void contact_meta(const DevModel<T>& m, const Env<T>& e, int ncf, ContactMeta<T>& cm,
                                             int c0 = 0) {
  const int c = c0 + lane_id();
  cm.dim = 3; cm.b1 = 0; cm.b2 = 0; cm.rt1 = 0; cm.rt2 = 0; cm.m1 = 0; cm.m2 = 0; cm.mu0 = 0; cm.mu1 = 0;
  if (c < ncf) {
    int p = e.con_pair[c];
    cm.dim = m.pair_condim[p];
    cm.b1 = m.geom_bodyid[e.con_geom[2 * c]];
    cm.b2 = m.geom_bodyid[e.con_geom[2 * c + 1]];
    cm.rt1 = m.body_rootid[cm.b1];
    cm.rt2 = m.body_rootid[cm.b2];
    cm.m1 = cm.b1 > 0 ? body_mask64(m, cm.b1) : 0ull;
    cm.m2 = cm.b2 > 0 ? body_mask64(m, cm.b2) : 0ull;
    cm.mu0 = m.pair_friction[5 * p];
    cm.mu1 = m.pair_friction[5 * p + 1];
  }
}

#ifdef MGX_PROFILE
#define MGX_BSTAMP(slot)                                                                \
  do {                                                                                  \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    unsigned long long _t = __builtin_amdgcn_s_memtime();                               \
    if (g_mgx_prof && threadIdx.x == 0) g_mgx_prof[blockIdx.x * 32 + (slot)] += _t - _bt; \
    _bt = _t;                                                                           \
    __builtin_amdgcn_sched_barrier(0);                                                  \
  } while (0)
#else
#define MGX_BSTAMP(slot) do {} while (0)
#endif

__device__ __forceinline__ float readlane_t(float x, int l) { return readlane(x, l); }
__device__ __forceinline__ double readlane_t(double x, int l) { return readlane(x, l); }

// One 4-row block, lane = dof: J rows in registers; J.qvel, J.qacc_smooth, J.qacc_warmstart
// (= B.(D^1/2 L x) of the monolithic path) per row in lane i without a reduction (limit
// rows: the dof's entry; contacts: the bodies' chain sums cvel / cacc at the contact point);
// B = D^-1/2 L'^-1 J' by a readlane sweep over the block's dof support only (the two bodies'
// chains, closed under ancestors, highest dof first); then B.B and the block couplings A_ij,
// the row scalars and B -> pipe.
// NCS: contact-metadata lane sets (contact c reads set c / 64, lane c % 64): 1 for up to 64
// contacts, 3 for up to 192 (bipedal_rescue).
template <typename T, int NCS = 1, bool DOFB = false>
__device__ __forceinline__ void build_block(const DevModel<T>& m, Env<T>& e, const Pipe& P, int r0, int nlim, int nlim4,
                                            const ContactMeta<T>& cm, const ContactMeta<T>& cm2,
                                            const ContactMeta<T>& cm3, T dinvs, T* scal, uint32_t* blk, T* Bo,
                                            int& boff) {
  const int l = lane_id();
  const int nv = m.nv;
  const bool dl = l < nv;
#ifdef MGX_PROFILE
  unsigned long long _bt = __builtin_amdgcn_s_memtime();
#endif
  // the block's row constants (rows_impedance), lane i < 4 row r0 + i, loaded now and used last
  T rc0 = 0, rc1 = 0, rc2 = 0, rc3 = 0;
  if (l < 4) {
    const T* q = scal + (size_t)(r0 >> 2) * (4 * MGX_SCAL) + l;
    rc0 = q[MGX_SQ(0, 0)]; rc1 = q[MGX_SQ(1, 0)]; rc2 = q[MGX_SQ(2, 0)]; rc3 = q[MGX_SQ(3, 0)];
  }
  T j0 = 0, j1 = 0, j2 = 0, j3 = 0;
  uint64_t sup = 0;
  T dv = 0, ds = 0, dw = 0;
  if (r0 < nlim4) {
    T* jj[4] = {&j0, &j1, &j2, &j3};
#pragma unroll
    for (int i = 0; i < 4; i++) {
      int r = r0 + i;
      if (r < nlim) {
        int code = e.efc_id[r];
        int d = m.jnt_dofadr[code >> 1];
        T sg = (code & 1) ? (T)-1 : (T)1;
        *jj[i] = l == d ? sg : (T)0;
        sup |= readlane_u64(e.ancmask, d) | (1ull << d);
        if (l == i) { dv = sg * e.qvel[d]; ds = sg * e.vec1[d]; dw = sg * e.vec2[d]; }
      }
    }
  } else {
    const int c = (r0 - nlim4) >> 2;
    const ContactMeta<T>& cs = (NCS > 2 && c >= 128) ? cm3 : (NCS > 1 && c >= 64) ? cm2 : cm;
    const int cl = c & 63;
    const int dim = readlane(cs.dim, cl), b1 = readlane(cs.b1, cl), b2 = readlane(cs.b2, cl);
    const int rt1 = readlane(cs.rt1, cl), rt2 = readlane(cs.rt2, cl);
    const uint64_t m1 = readlane_u64(cs.m1, cl), m2 = readlane_u64(cs.m2, cl);
    const T mu0 = readlane_t(cs.mu0, cl), mu1 = readlane_t(cs.mu1, cl);
    // the contact frame from its normal (make_frame, as collision builds it for the
    // monolithic layout: the same arithmetic on the same normal)
    T fr[9];
    fr[0] = e.con_frame[3 * c]; fr[1] = e.con_frame[3 * c + 1]; fr[2] = e.con_frame[3 * c + 2];
    make_frame(fr);
    const T* cp = e.con_pos + 3 * c;
    sup = m1 | m2;
    T o1[3] = {cp[0] - e.subtree_com[3 * rt1], cp[1] - e.subtree_com[3 * rt1 + 1], cp[2] - e.subtree_com[3 * rt1 + 2]};
    T o2[3] = {cp[0] - e.subtree_com[3 * rt2], cp[1] - e.subtree_com[3 * rt2 + 1], cp[2] - e.subtree_com[3 * rt2 + 2]};
    if (dl) {
      T jd[3] = {0, 0, 0};
      const T* cd = e.cdof + 6 * l;
      if ((m2 >> l) & 1ull) {
        T t[3];
        cross3(t, cd, o2);
        jd[0] += cd[3] + t[0]; jd[1] += cd[4] + t[1]; jd[2] += cd[5] + t[2];
      }
      if ((m1 >> l) & 1ull) {
        T t[3];
        cross3(t, cd, o1);
        jd[0] -= cd[3] + t[0]; jd[1] -= cd[4] + t[1]; jd[2] -= cd[5] + t[2];
      }
      T cj0 = fr[0] * jd[0] + fr[1] * jd[1] + fr[2] * jd[2];
      if (dim == 1) {
        j0 = cj0;
      } else {
        T cj1 = fr[3] * jd[0] + fr[4] * jd[1] + fr[5] * jd[2];
        T cj2 = fr[6] * jd[0] + fr[7] * jd[1] + fr[8] * jd[2];
        j0 = cj0 + mu0 * cj1; j1 = cj0 - mu0 * cj1; j2 = cj0 + mu1 * cj2; j3 = cj0 - mu1 * cj2;
      }
    }
    if (l < 4) {
      // relative point motion of body 2 vs body 1 in the contact frame, for x = qvel,
      // qacc_smooth, qacc_warmstart (vel = cvel, the others = cacc[0:6] / cacc[6:12])
      T out[3];
#pragma unroll
      for (int q = 0; q < 3; q++) {
        const T* s2 = q == 0 ? e.cvel + 6 * b2 : e.cacc + 12 * b2 + 6 * (q - 1);
        const T* s1 = q == 0 ? e.cvel + 6 * b1 : e.cacc + 12 * b1 + 6 * (q - 1);
        T t2[3], t1[3];
        cross3(t2, s2, o2);
        cross3(t1, s1, o1);
        T dd[3] = {s2[3] + t2[0] - s1[3] - t1[0], s2[4] + t2[1] - s1[4] - t1[1], s2[5] + t2[2] - s1[5] - t1[2]};
        T cn = fr[0] * dd[0] + fr[1] * dd[1] + fr[2] * dd[2];
        T ct = (l >> 1) == 0 ? fr[3] * dd[0] + fr[4] * dd[1] + fr[5] * dd[2] : fr[6] * dd[0] + fr[7] * dd[1] + fr[8] * dd[2];
        T mu = (l >> 1) == 0 ? mu0 : mu1;
        out[q] = dim == 1 ? cn : ((l & 1) ? cn - mu * ct : cn + mu * ct);
      }
      dv = out[0]; ds = out[1]; dw = out[2];
    }
  }
  MGX_BSTAMP(8);
  // L'^-1 over the support, highest dof first (the rows of a dof's descendants are final);
  // the next step's L column is loaded before this step's updates
  uint64_t sp = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)sup) |
                ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(sup >> 32)) << 32);
  if (sp) {
    int k = 63 - __clzll(sp);
    int base = readlane(e.madr, k) + readlane(e.chainlen, k) - e.chainlen;
    T ld = e.qLD[base > 0 ? base : 0];
    while (true) {
      sp &= ~(1ull << k);
      uint64_t am = readlane_u64(e.ancmask, k);
      T x0 = readlane(j0, k), x1 = readlane(j1, k), x2 = readlane(j2, k), x3 = readlane(j3, k);
      int kn = sp ? 63 - __clzll(sp) : k;
      int basen = readlane(e.madr, kn) + readlane(e.chainlen, kn) - e.chainlen;
      T ldn = e.qLD[basen > 0 ? basen : 0];
      T coef = (dl && ((am >> l) & 1ull)) ? ld : (T)0;
      j0 -= coef * x0; j1 -= coef * x1; j2 -= coef * x2; j3 -= coef * x3;
      if (!sp) break;
      k = kn;
      ld = ldn;
    }
  }
  j0 *= dinvs; j1 *= dinvs; j2 *= dinvs; j3 *= dinvs;
  MGX_BSTAMP(9);
  // B.B and the couplings (10 sums; the last two slots of the third call are unused)
  T n0 = j0 * j0, n1 = j1 * j1, n2 = j2 * j2, n3 = j3 * j3;
  T a10 = j1 * j0, a20 = j2 * j0, a21 = j2 * j1, a30 = j3 * j0, a31 = j3 * j1, a32 = j3 * j2;
  wave_sum4(n0, n1, n2, n3);
  wave_sum4(a10, a20, a21, a30);
  T z0 = 0, z1 = 0;
  wave_sum4(a31, a32, z0, z1);
  MGX_BSTAMP(10);
  if (l < 4) {
    T* o = scal + (size_t)(r0 >> 2) * (4 * MGX_SCAL) + l;
    T nn = l == 0 ? n0 : l == 1 ? n1 : l == 2 ? n2 : n3;
    if (rc3 != 0) {
      T R = rc0;
      T aref = -rc1 * dv - rc2;   // mj_referenceConstraint
      T jar = dw - aref;
      T ad = nn + R;
      o[MGX_SQ(0, 0)] = ds - aref;                 // b = J qacc_smooth - aref
      o[MGX_SQ(1, 0)] = jar < 0 ? -jar / R : (T)0; // warmstart force (mj_constraintUpdate, pyramidal)
      o[MGX_SQ(2, 0)] = R;
      o[MGX_SQ(3, 0)] = (T)1 / ad;
      o[MGX_SQ(4, 0)] = (T)0.5 * ad;               // the solver's cost change is delta * (delta * AR / 2 + res)
    } else {
      o[MGX_SQ(0, 0)] = 0; o[MGX_SQ(1, 0)] = 0; o[MGX_SQ(2, 0)] = 1; o[MGX_SQ(3, 0)] = 1; o[MGX_SQ(4, 0)] = (T)0.5;
    }
  }
  // the block for the solver: [A10 A20 A21 A30 A31 A32 0 0], then its B entries (DOFB: per support
  // dof ascending, the dof's 4 rows; else per touched 8-dof group ascending, [8 dofs][4 rows]) — a
  // lane's 4 rows of one dof are one 16-byte load in the solver. A dof outside the support has B = 0
  // exactly (the J build and the L'^-1 sweep touch the support only); every lane of a touched group
  // stores, so a group running past nv (bipedal's phantom dof 63) carries zeros, not stale data.
  {
    T* o = Bo + boff;
    if (l < 8) o[l] = l == 0 ? a10 : l == 1 ? a20 : l == 2 ? a21 : l == 3 ? a30 : l == 4 ? a31 : l == 5 ? a32 : (T)0;
    if constexpr (DOFB) {
      if ((sup >> l) & 1ull) {
        T* od = o + 8 + 4 * __popcll(sup & ((1ull << l) - 1ull));
        od[0] = j0; od[1] = j1; od[2] = j2; od[3] = j3;
      }
      if (l < MGX_TW) {
        uint32_t* bt = blk + MGX_TW * (r0 >> 2);
        bt[l] = l == 0 ? (uint32_t)boff : l == 1 ? (uint32_t)sup : l == 2 ? (uint32_t)(sup >> 32) : 0u;
      }
      boff += 8 + 4 * __popcll(sup);
    } else {
      uint32_t gm = 0;
#pragma unroll
      for (int g = 0; g < 8; g++) gm |= ((sup >> (8 * g)) & 0xffull) ? (1u << g) : 0u;
      const int g = l >> 3, jj = l & 7;
      if ((gm >> g) & 1u) {
        T* og = o + 8 + 32 * __popc(gm & ((1u << g) - 1u)) + 4 * jj;
        og[0] = j0; og[1] = j1; og[2] = j2; og[3] = j3;
      }
      if (l < 8) {  // 8 uint16: the A offset, then per group g < 7 its data offset or 0 (the zero group)
        uint16_t* bt = reinterpret_cast<uint16_t*>(blk + MGX_TW * (r0 >> 2));
        const int v = l == 0 ? boff : (((gm >> (l - 1)) & 1u) ? boff + 8 + 32 * __popc(gm & ((1u << (l - 1)) - 1u)) : 0);
        bt[l] = (uint16_t)v;
      }
      boff += 8 + 32 * __popc(gm);
    }
  }
  MGX_BSTAMP(11);
}

// S1 body: forward up to the constraint rows, rows -> pipe, carry -> pipe
// list_slot: enter the slot in the solver launches' lists (the pipeline); the one-wave settle
// (settle_step) solves the slot itself.
template <typename T, int NCS = 1, bool DOFB = false>
__device__ __forceinline__ void stage_rows(const DevModel<T>& m, Env<T>& e, const Pipe& P, int slot, int warn,
                                           bool list_slot = true) {
  int l = lane_id();
  const int nv = m.nv;
  MGX_STAMP_DECL
  kinematics(m, e);
  MGX_STAMP(0);
  com_crb(m, e);
  MGX_STAMP(1);
  e.diaginv = factor_ld(m, e, e.qLD);
  MGX_STAMP(2);
  {
    // the velocity stage reads xfrc_applied from an LDS copy (the carry tail is in global memory)
    T* const xg = e.xfrc;
    T* const xl = e.cdof + (m.L.xfrc_lds - m.L.cdof);
    for (int k = l; k < 6 * m.nbody; k += 64) xl[k] = xg[k];
    wsync();
    e.xfrc = xl;
    velocity(m, e);
    e.xfrc = xg;
  }
  MGX_STAMP(3);
  e.qacc_smooth = solve_M(m, e, e.qLD, e.diaginv, e.qfrc_smooth);
  MGX_STAMP(4);
  if (m.L.late_geom) geom_poses<T, true>(m, e);
  collision(m, e);
  MGX_STAMP(5);
  int nlim, ncf;
  const int ne = rows_plan(m, e, &nlim, &ncf);
  e.nefc = ne;
  MGX_STAMP(6);
  const bool dl = l < nv;
  int boff = 32;  // B reals of the slot; [0, 32): the zero area (A and B of absent entries)
  if (ne > 0) {
    const T dinvs = dl ? sqrt(e.diaginv) : (T)0;
    T* scal = P.at<T>(P.o_scal) + (size_t)slot * P.maxE * MGX_SCAL;
    T* Bo = P.at<T>(P.o_B) + (size_t)slot * P.bcap;
    uint32_t* blk = P.at<uint32_t>(P.o_blk) + (size_t)slot * (P.maxE / 4) * MGX_TW;
    const int nlim4 = (nlim + 3) & ~3;
    // qacc_smooth / qacc_warmstart into LDS (limit rows) and their per-body chain sums
    if (dl) { e.vec1[l] = e.qacc_smooth; e.vec2[l] = e.qacc_ws; }
    wsync();
    if (ncf > 0) {
      for (int b = l; b < m.nbody; b += 64) {
        T a[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        int depth = m.body_depth[b];
        for (int c = 0; c < depth; c++) {
          int i = m.body_chain[b * MGX_MAX_DEPTH + c];
          int bda = m.body_dofadr[i], nd = m.body_dofnum[i];
          for (int jd = bda; jd < bda + nd; jd++) {
            T xs = e.vec1[jd], xw = e.vec2[jd];
            const T* cd = e.cdof + 6 * jd;
            for (int q = 0; q < 6; q++) { a[q] += cd[q] * xs; a[6 + q] += cd[q] * xw; }
          }
        }
        for (int q = 0; q < 12; q++) e.cacc[12 * b + q] = a[q];
      }
      wsync();
    }
    rows_impedance(m, e, ne, nlim, nlim4, scal);
    ContactMeta<T> cm, cm2, cm3;
    contact_meta(m, e, ncf, cm);
    if constexpr (NCS > 1) contact_meta(m, e, ncf, cm2, 64);
    if constexpr (NCS > 2) contact_meta(m, e, ncf, cm3, 128);
    __threadfence();  // the row constants are read back by other lanes of this wave (build_block)
    wsync();
    for (int r0 = 0; r0 < ne; r0 += 4)
      build_block<T, NCS, DOFB>(m, e, P, r0, nlim, nlim4, cm, cm2, cm3, dinvs, scal, blk, Bo, boff);
  }
  MGX_STAMP(7);
  // carry + registers + ints
  T* cr = P.at<T>(P.o_carry) + (size_t)slot * P.carry_stride;
  for (int k = l; k < m.L.carry_lds; k += 64) cr[k] = reinterpret_cast<T*>(e.qpos)[k - m.L.qpos];
  T* rg = cr + ((m.L.carry_reals + 63) & ~63);
  rg[l] = e.qacc_ws; rg[64 + l] = e.qfrc_applied; rg[128 + l] = e.qfrc_smooth; rg[192 + l] = e.qacc_smooth;
  if (l == 0) rg[256] = e.time;
  int* ci = P.at<int>(P.o_carryi) + (size_t)slot * P.carryi_stride;
  for (int k = l; k < 2 * e.ncon; k += 64) ci[k] = e.con_geom[k];
  int* cx = ci + m.L.carry_ints;
  if (l == 0) {
    cx[0] = e.ncon; cx[1] = ne; cx[2] = e.overflow; cx[3] = warn;
    P.at<int>(P.o_ne)[slot] = ne;
    P.at<int>(P.o_blen)[slot] = boff;
#ifdef MGX_PROFILE
    if (g_mgx_prof && slot < (int)gridDim.x) {
      g_mgx_prof[slot * 32 + 20] += ne;
      g_mgx_prof[slot * 32 + 22] += e.ncon;
      g_mgx_prof[slot * 32 + 23] += 1;
      if ((unsigned long long)ne > g_mgx_prof[slot * 32 + 24]) g_mgx_prof[slot * 32 + 24] = ne;
      g_mgx_prof[slot * 32 + 25] += e.overflow != 0;
    }
#endif
    if (!list_slot) {
    } else if (ne > P.capE && !P.hmain) {  // rare: more rows than the main solver launch keeps in LDS
      int idx = atomicAdd(P.ctr() + 2, 1);
      P.at<int>(P.o_k2big)[idx] = slot;
    } else if (ne > 0) {
      int idx = atomicAdd(P.ctr() + 1, 1);
      P.at<int>(P.o_k2list)[idx] = slot;  // arrival order (diagnostics: tools/pgs_census.py)
      const int nb = ne >> 2;
      const int r = atomicAdd(P.at<int>(P.o_hist) + nb, 1);
      P.at<int>(P.o_blist)[(size_t)nb * P.S + r] = slot;
    }
  }
}

// ------------------------------------------------------------------ S2: lane-group PGS
// Gauss-Seidel sweeps of mj_solPGS [ext], 64 / LPS slots per wave, LPS lanes per slot (16: four
// slots per wave; 64: one slot per wave, lane = dof). Row scalars (b, f, R, 1/AR, AR/2), the block
// table and the slot's B live in LDS; v = B'f lives in registers. Each 4-row block's B comes
// compressed to the 8-dof groups its support touches, with its couplings A_ij; lane j holds
// dof 8 gi + (j & 7) of group gi. A register ring keeps the next block in flight ahead of use
// (RING - 1 blocks: 1 from LDS, 2 from global memory). Per block the four B_r.v use the
// pre-block v (interleaved DPP reductions) and row i adds sum_{j<i} A_ij delta_j: the
// sequential Gauss-Seidel update. Per-slot results do not depend on which slots share the wave
// (other slots only add masked no-op blocks / sweeps) nor on the launch that solves the slot.
template <int CTRL>
__device__ __forceinline__ float dpp_row(float v) {
  // bound_ctrl: every source lane of these patterns is valid, so the mov folds into its add
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, true));
}
// four independent 8-lane sums (quad_perm 1,0,3,2 / 2,3,0,1, row_half_mirror); every lane of
// the 8-lane group ends with the identical total
// With 16 lanes per slot a row_mirror step adds the two 8-lane halves (lane i and 15 - i).
template <int LPS>
__device__ __forceinline__ void oct_sum4(float& a, float& b, float& c, float& d) {
#define MGX_R4(CTRL) a += dpp_row<CTRL>(a); b += dpp_row<CTRL>(b); c += dpp_row<CTRL>(c); d += dpp_row<CTRL>(d);
  MGX_R4(0xB1)
  MGX_R4(0x4E)
  MGX_R4(0x141)
  if constexpr (LPS == 16) { MGX_R4(0x140) }
#undef MGX_R4
}
template <int LPS>
__device__ __forceinline__ double oct_sum(double x) {
  x += dpp_d<0xB1>(x);
  x += dpp_d<0x4E>(x);
  x += dpp_d<0x141>(x);
  if constexpr (LPS == 16) x += dpp_d<0x140>(x);
  return x;
}
template <int LPS>
__device__ __forceinline__ void oct_sum4(double& a, double& b, double& c, double& d) {
  a = oct_sum<LPS>(a); b = oct_sum<LPS>(b); c = oct_sum<LPS>(c); d = oct_sum<LPS>(d);
}
// the slot's four row dots: 8 / 16 lanes in-row DPP butterflies; a whole wave (one slot per
// wave) the full-wave DPP reduction, totals uniform
template <int LPS, typename T>
__device__ __forceinline__ void slot_sum4(T& a, T& b, T& c, T& d) {
  if constexpr (LPS == 64) wave_sum4(a, b, c, d);
  else oct_sum4<LPS>(a, b, c, d);
}

template <typename T>
struct Vec4T;
template <>
struct Vec4T<float> { typedef float type __attribute__((ext_vector_type(4))); };
template <>
struct Vec4T<double> { typedef double type __attribute__((ext_vector_type(4))); };

template <typename T, int EPL>
struct PgsBlk {
  typename Vec4T<T>::type b[EPL];  // B of the block's 4 rows at this lane's dof j + 8d
  typename Vec4T<T>::type a0, a1;  // A10 A20 A21 A30 | A31 A32 - -
  typename Vec4T<T>::type qb, qf, qR, qi, qh;  // the rows' b, f, R, 1/AR, AR/2
};
// a block's table entry for this lane: the A offset and the offsets of its EPL dof groups,
// loaded one ring step before the data they address
template <int EPL>
struct PgsTab {
  uint32_t a, g[EPL];
};

template <int EPL, int LPS, bool DOFB>
__device__ __forceinline__ void pgs_load_tab(PgsTab<EPL>& t, const uint32_t* bt, int blk, int j) {
  if constexpr (DOFB) {
    // one 16-byte LDS load: [B offset, support lo, support hi, 0]; this lane's dof of each register
    // entry is at rank popc(support below it) of the block's dof list, or absent (zero area)
    const uint4 e = *reinterpret_cast<const uint4*>(bt + 4 * blk);
    t.a = e.x;
    const uint64_t sup = (uint64_t)e.y | ((uint64_t)e.z << 32);
#pragma unroll
    for (int d = 0; d < EPL; d++) {
      const int dof = 8 * (d * (LPS / 8) + (j >> 3)) + (j & 7);
      const uint64_t below = dof >= 64 ? sup : sup & ((1ull << dof) - 1ull);
      const bool in = dof < 64 && ((sup >> (dof & 63)) & 1ull);
      t.g[d] = in ? e.x + 8u + 4u * (uint32_t)__popcll(below) : 0u;
    }
  } else {
    // the A offset and the offsets of the lane's EPL dof groups (widened in LDS: no 16-bit extracts
    // on the address path); absent groups point at the zero group
    const uint32_t* e = bt + 8 * blk;
    t.a = e[0];
#pragma unroll
    for (int d = 0; d < EPL; d++) {
      const int gi = d * (LPS / 8) + (j >> 3);
      t.g[d] = (gi < 7 ? e[1 + gi] : 0u) + 4u * (uint32_t)(j & 7);
    }
  }
}

// f32: two values per v_pk_fma_f32
typedef float mgx_f2 __attribute__((ext_vector_type(2)));

// One block's data at its (prefetched) table entry: A, the lane's B entries and the row scalars.
// The forces travel with the prefetch: a block's f changes only when the block itself is solved,
// and the look-ahead never crosses a sweep boundary (each sweep restarts the ring), so the value
// loaded here is the latest one.
// sq: the row scalars ([b][f][R][1/AR][AR/2] x 4 per block; LDS arena or the pipe in global
// memory), fb: the forces, FS reals per block (the LDS copy the sweeps update)
template <typename T, int EPL, int LPS, int FS>
__device__ __forceinline__ void pgs_load_block(PgsBlk<T, EPL>& k, const T* Bsl, const T* sq, const T* fb,
                                               const PgsTab<EPL>& t, int blk, int sblk, int j) {
  // the table entry of a block past the slot's end points at the zero group (A included);
  // every load is one 16-byte vector load at a table offset (Bsl: the slot's B in the LDS
  // arena, or in global memory for the global-B launch)
  typedef typename Vec4T<T>::type V4;
  const V4* pa = reinterpret_cast<const V4*>(Bsl + t.a);
  k.a0 = pa[0];
  k.a1 = pa[1];
#pragma unroll
  for (int d = 0; d < EPL; d++) k.b[d] = *reinterpret_cast<const V4*>(Bsl + t.g[d]);
  const V4* q = reinterpret_cast<const V4*>(sq + 4 * MGX_SCAL * sblk);
  k.qb = q[0];
  k.qf = *reinterpret_cast<const V4*>(fb + FS * blk);
  k.qR = q[2];
  k.qi = q[3];
  k.qh = q[4];
  __builtin_amdgcn_sched_barrier(0);  // keep the prefetch where it is issued
}
template <typename T, int EPL, int LPS, int FS, bool DOFB>
__device__ __forceinline__ void pgs_load_block(PgsBlk<T, EPL>& k, const T* Bsl, const T* sq, const T* fb,
                                               const uint32_t* bt, int blk, int sblk, int j) {
  PgsTab<EPL> t;
  pgs_load_tab<EPL, LPS, DOFB>(t, bt, blk, j);
  pgs_load_block<T, EPL, LPS, FS>(k, Bsl, sq, fb, t, blk, sblk, j);
}

template <typename T, int EPL>
__device__ __forceinline__ void pgs_dots(const PgsBlk<T, EPL>& k, const T (&v)[EPL], T& d0, T& d1, T& d2, T& d3) {
  d0 = d1 = d2 = d3 = 0;
#pragma unroll
  for (int d = 0; d < EPL; d++) {
    d0 += k.b[d].x * v[d]; d1 += k.b[d].y * v[d]; d2 += k.b[d].z * v[d]; d3 += k.b[d].w * v[d];
  }
}
template <int EPL>
__device__ __forceinline__ void pgs_dots(const PgsBlk<float, EPL>& k, const float (&v)[EPL], float& d0, float& d1,
                                         float& d2, float& d3) {
  mgx_f2 p01 = {0.f, 0.f}, p23 = {0.f, 0.f};
#pragma unroll
  for (int d = 0; d < EPL; d++) {
    mgx_f2 vv = {v[d], v[d]};
    p01 = __builtin_elementwise_fma(k.b[d].xy, vv, p01);
    p23 = __builtin_elementwise_fma(k.b[d].zw, vv, p23);
  }
  d0 = p01.x; d1 = p01.y; d2 = p23.x; d3 = p23.y;
}

template <typename T, int EPL>
__device__ __forceinline__ void pgs_update(const PgsBlk<T, EPL>& k, T (&v)[EPL], T dl0, T dl1, T dl2, T dl3) {
  // v += B' dl as four FMA chains per entry (one v_fmac each)
#pragma unroll
  for (int d = 0; d < EPL; d++) {
    T x = fma(dl0, k.b[d].x, v[d]);
    x = fma(dl1, k.b[d].y, x);
    x = fma(dl2, k.b[d].z, x);
    v[d] = fma(dl3, k.b[d].w, x);
  }
}

template <typename T, int EPL, int LPS>
__device__ __forceinline__ void pgs_block(const PgsBlk<T, EPL>& k, T (&v)[EPL], T* fblk, bool ok0, T& impr) {
  typedef typename Vec4T<T>::type V4;
  V4* qf = reinterpret_cast<V4*>(fblk);
  const V4 qb = k.qb, f = k.qf, qR = k.qR, qi = k.qi, qh = k.qh;
  T d0, d1, d2, d3;
  pgs_dots(k, v, d0, d1, d2, d3);
  // b + R f off the dependent chain
  const T t0 = qb.x + qR.x * f.x, t1 = qb.y + qR.y * f.y;
  const T t2 = qb.z + qR.z * f.z, t3 = qb.w + qR.w * f.w;
  slot_sum4<LPS>(d0, d1, d2, d3);
  T dl0, dl1, dl2, dl3;
  V4 nfv;
#define MGX_PGS_ROW(C, I, DOT, DL)                                \
  {                                                               \
    const T fr = f.C, ai = qi.C, hd = qh.C;                       \
    T res = (DOT) + t##I;                                         \
    T fn = fmax(fr - res * ai, (T)0);                             \
    T delta = fn - fr;                                            \
    T change = delta * (delta * hd + res);                        \
    bool keep = !ok0 || change > (T)1e-10;                        \
    DL = keep ? (T)0 : delta;                                     \
    impr -= keep ? (T)0 : change;                                 \
    nfv.C = keep ? fr : fn;                                       \
  }
  MGX_PGS_ROW(x, 0, d0, dl0)
  MGX_PGS_ROW(y, 1, d1 + k.a0.x * dl0, dl1)
  MGX_PGS_ROW(z, 2, d2 + k.a0.y * dl0 + k.a0.z * dl1, dl2)
  MGX_PGS_ROW(w, 3, d3 + k.a0.w * dl0 + k.a1.x * dl1 + k.a1.y * dl2, dl3)
#undef MGX_PGS_ROW
  // one lane per slot stores the forces: the slot's lanes hold identical values, and a
  // same-address LDS store from every lane serialises
  if ((lane_id() & (LPS - 1)) == 0) *qf = nfv;
  pgs_update(k, v, dl0, dl1, dl2, dl3);
}

// One group of up to 64 / LPS slots (one wave).
// BLDS (main launch): the wave's slots get an LDS arena of P.arena bytes laid out by their
// actual sizes — per slot the row scalars and block table for the wave's block count, then the
// slot's compressed B (P.o_blen reals), copied from global memory once. A wave whose slots do
// not fit lists them for the global-B launch and returns before touching anything.
// !BLDS (global-B launch): fixed per-slot capacity of capE rows of scalars and table in LDS, B
// read from global memory (L2 / MALL) with a register ring RING - 1 blocks ahead.
// Both run the identical arithmetic on every slot, so which launch solves a slot is invisible.
// SQG (global-B only): the row scalars b / R / 1/AR / AR/2 are read from the pipe with the B
// prefetch and only the forces live in LDS. The RK4 pipeline uses it (its 256-row slots would
// otherwise hold the launch to two waves per CU; bipedal 175.0k -> 186.6k env-steps/s); the
// soccer launch keeps all scalars in LDS at four waves per CU, which measured faster than the
// global scalars at any occupancy (MGX_PGS_LDS_PAD sweep).
template <typename T, int EPL, int LPS, bool BLDS, bool SQG = false, bool DOFB = false>
__device__ __forceinline__ void pgs_group(const Pipe& P, char* smem, int slot, int capE, int maxit, T tol, T scale,
                                          int spw, int arena = -1) {
  constexpr int RING = BLDS ? MGX_PGS_RING_LDS : MGX_PGS_RING;
  typedef typename Vec4T<T>::type V4;
  constexpr int SPW = 64 / LPS;
  const int l = threadIdx.x, s = l / LPS, j = l % LPS;
  (void)spw;
  const int ne = slot >= 0 ? P.at<int>(P.o_ne)[slot] : 0;  // a multiple of 4
  const int nblk = ne >> 2;
  int nm = nblk;
  nm = max(nm, __shfl_xor(nm, 8));
  nm = max(nm, __shfl_xor(nm, 16));
  nm = max(nm, __shfl_xor(nm, 32));
  int nbMax = __builtin_amdgcn_readfirstlane(nm);
  if (spw < 0) nbMax = capE / 4;  // debug: sweep every block slot
  // whole ring turns: the sweep has no remainder path; the padding blocks are zero-table
  // blocks whose rows are masked (their LDS scalars zero-filled below)
  const int nbRun = (nbMax + RING - 1) / RING * RING;
  const size_t sl = (size_t)(slot >= 0 ? slot : 0);
  const T* gsc = P.at<T>(P.o_scal) + sl * P.maxE * MGX_SCAL;
  constexpr int TWL = mgx_twl(DOFB);  // table words per block in LDS
  const uint32_t* gbt = P.at<uint32_t>(P.o_blk) + sl * (P.maxE / 4) * MGX_TW;
  const uint16_t* gbt16 = reinterpret_cast<const uint16_t*>(gbt);
  const T* gB = P.at<T>(P.o_B) + sl * P.bcap;
  int nbA;  // blocks of scalars / table entries per slot (the look-ahead stays inside)
  T* sc;
  uint32_t* bt;
  const T* Bsl;
  // all row scalars in LDS with the forces in place (FS = 20 reals per block), or (SQG) only the
  // forces in LDS (FS = 4)
  constexpr bool SG = SQG && !BLDS;
  constexpr int FS = SG ? 4 : 4 * MGX_SCAL;
  const T* sq;
  T* fb;
  if constexpr (BLDS) {
    nbA = nbRun + RING - 1;
    const int blen = slot >= 0 ? (P.at<int>(P.o_blen)[slot] + 3) & ~3 : 0;
    const int bytes = nbA * (4 * MGX_SCAL * (int)sizeof(T) + 4 * TWL) + blen * (int)sizeof(T);  // 16-byte multiple
    int off = 0, tot = 0;
    if (arena < 0) {
      // main launch: the wave's slots side by side
#pragma unroll
      for (int q = 0; q < SPW; q++) {
        const int bq = __shfl(bytes, q * LPS);
        off += q < s ? bq : 0;
        tot += bq;
      }
    } else {
      // wide launch: every lane group of the wave runs the wave's one slot on one shared copy
      // (identical values to identical addresses; the slot's arithmetic is the lane group's)
      tot = bytes;
    }
    if (__builtin_amdgcn_readfirstlane(tot) > (arena < 0 ? P.arena : arena)) {
      // main launch: the wide launch takes the wave's slots. The wide launch's own arena
      // (arena >= 0, P.warena) holds any one slot by construction (make_staged_pipe), so it never
      // lands here
      if (arena < 0 && j == 0 && slot >= 0) P.at<int>(P.o_k2big)[atomicAdd(P.ctr() + 2, 1)] = slot;
      return;
    }
    sc = reinterpret_cast<T*>(smem + off);
    bt = reinterpret_cast<uint32_t*>(sc + 4 * MGX_SCAL * nbA);
    T* Bs = reinterpret_cast<T*>(bt + TWL * nbA);
    for (int q = 4 * j; q < blen; q += 4 * LPS)
      *reinterpret_cast<V4*>(Bs + q) = *reinterpret_cast<const V4*>(gB + q);
    Bsl = Bs;
    sq = sc;
    fb = sc + MGX_SQ(1, 0);
    for (int q = j; q < MGX_SCAL * 4 * nbA; q += LPS) sc[q] = q < ne * MGX_SCAL ? gsc[q] : (T)0;
  } else {
    // LDS capacity in whole ring turns: nbA = capE / 4 rounded up to a multiple of the ring
    const int nbcap = capE / 4;
    nbA = (nbcap + RING - 1) / RING * RING;
    const int sstride = (SG ? 4 : 4 * MGX_SCAL) * nbA + 4;  // 16-byte aligned per slot
    sc = reinterpret_cast<T*>(smem) + s * sstride;
    bt = reinterpret_cast<uint32_t*>(reinterpret_cast<T*>(smem) + SPW * sstride) + s * TWL * nbA;
    Bsl = gB;
    if constexpr (SG) {
      sq = gsc;
      fb = sc;
      for (int q = j; q < 4 * nbA; q += LPS) sc[q] = q < ne ? gsc[(q >> 2) * (4 * MGX_SCAL) + MGX_SQ(1, q & 3)] : (T)0;
    } else {
      sq = sc;
      fb = sc + MGX_SQ(1, 0);
      for (int q = j; q < MGX_SCAL * 4 * nbA; q += LPS) sc[q] = q < ne * MGX_SCAL ? gsc[q] : (T)0;
    }
  }
  // scalar blocks past the slot's capacity are never real (masked); their loads stay inside it
  const int sbmax = P.maxE / 4 - 1;
  // block table: the slot's blocks, then zero-group entries up to the capacity
  for (int q = j; q < TWL * nbA; q += LPS) bt[q] = q < TWL * nblk ? (DOFB ? gbt[q] : (uint32_t)gbt16[q]) : 0u;
  __syncthreads();
  // warmstart: v = B' f, dual cost, reset to zero if the cost is positive
  T v[EPL];
#pragma unroll
  for (int d = 0; d < EPL; d++) v[d] = 0;
  for (int b = 0; b < nbMax; b++) {
    PgsBlk<T, EPL> k;
    pgs_load_block<T, EPL, LPS, FS, DOFB>(k, Bsl, sq, fb, bt, b, min(b, sbmax), j);
    const T* qf = fb + FS * b;
    bool ok = b < nblk;
    T f0 = ok ? qf[0] : (T)0, f1 = ok ? qf[1] : (T)0, f2 = ok ? qf[2] : (T)0, f3 = ok ? qf[3] : (T)0;
    pgs_update(k, v, f0, f1, f2, f3);
  }
  T cpart = 0;
  for (int b = 0; b < nbMax; b++) {
    PgsBlk<T, EPL> k;
    pgs_load_block<T, EPL, LPS, FS, DOFB>(k, Bsl, sq, fb, bt, b, min(b, sbmax), j);
    T d0, d1, d2, d3;
    pgs_dots(k, v, d0, d1, d2, d3);
    slot_sum4<LPS>(d0, d1, d2, d3);
    if (b < nblk) {
      T dd[4] = {d0, d1, d2, d3};
      const T* qq = sq + 4 * b * MGX_SCAL;
      const T* qf = fb + FS * b;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const T fi = qf[i];
        cpart += fi * (qq[MGX_SQ(0, i)] + (T)0.5 * (dd[i] + qq[MGX_SQ(2, i)] * fi));
      }
    }
  }
  if (cpart > 0) {
    for (int r = j; r < ne; r += LPS) fb[(r >> 2) * FS + (r & 3)] = 0;
#pragma unroll
    for (int d = 0; d < EPL; d++) v[d] = 0;
  }
  __syncthreads();
  bool act = ne > 0;
  int it = 0;
#ifdef MGX_PROFILE
  unsigned long long t_sweep0 = __builtin_amdgcn_s_memtime();
  unsigned long long r_sweep0 = __builtin_amdgcn_s_memrealtime();
  int nsweep = 0;
#endif
  for (int iter = 0; iter < maxit; iter++) {
    if (__ballot(act) == 0ull) break;
#ifdef MGX_PROFILE
    nsweep++;
#endif
    T impr = 0;
    PgsBlk<T, EPL> R[RING];
    PgsTab<EPL> tn;  // the table entry of the next block to load (one ring step ahead of its data)
    pgs_load_tab<EPL, LPS, DOFB>(tn, bt, 0, j);
#pragma unroll
    for (int k = 0; k < RING - 1; k++) {
      pgs_load_block<T, EPL, LPS, FS>(R[k], Bsl, sq, fb, tn, k, min(k, sbmax), j);
      pgs_load_tab<EPL, LPS, DOFB>(tn, bt, k + 1, j);
    }
    // full ring turns, no early exit inside, so every prefetch is consumed on every path and
    // the compiler cannot sink the loads next to their use. The table has zero entries up to
    // nbA, so the look-ahead past nbMax reads zeros.
    for (int b0 = 0; b0 < nbRun; b0 += RING) {
#pragma unroll
      for (int k = 0; k < RING; k++) {
        // the slot consumed last lands the block RING - 1 ahead, then block b0 + k is solved
        const int bn = min(b0 + k + RING - 1, nbA - 1);
        pgs_load_block<T, EPL, LPS, FS>(R[(k + RING - 1) % RING], Bsl, sq, fb, tn, bn, min(bn, sbmax), j);
        pgs_load_tab<EPL, LPS, DOFB>(tn, bt, min(bn + 1, nbA - 1), j);
        pgs_block<T, EPL, LPS>(R[k], v, fb + FS * (b0 + k), act && b0 + k < nblk, impr);
      }
    }
    if (act) {
      it++;
      if (impr * scale < tol) act = false;
    }
  }
#ifdef MGX_PROFILE
  if (g_mgx_prof && l == 0) {
    // solver diagnostics, one record per wave in slots 26..30 of the wave's profile row
    unsigned long long* pr = g_mgx_prof + (size_t)blockIdx.x * 32;
    pr[26] += __builtin_amdgcn_s_memtime() - t_sweep0;
    pr[27] += (unsigned long long)nsweep * nbMax;
    pr[28] += 1;
    pr[29] += __builtin_amdgcn_s_memrealtime() - r_sweep0;
    if ((unsigned long long)(nsweep * nbMax) > pr[30]) pr[30] = nsweep * nbMax;
  }
#endif
  if (slot >= 0) {
    T* vo = P.at<T>(P.o_vout) + (size_t)slot * 64;
#pragma unroll
    for (int d = 0; d < EPL; d++)
      {
        const int dof = 8 * (d * (LPS / 8) + (j >> 3)) + (j & 7);
        if (dof < P.nv) vo[dof] = v[d];
      }
    if (j == 0) P.at<int>(P.o_niter)[slot] = it;
  }
}

// big = 0: the main launch over the solver list (one wave per 64 / LPS listed slots); big = 1:
// the slots with capE < nefc <= maxE and those of LDS-arena waves that did not fit, grid-stride
// over a small grid with maxE rows of scalars per slot in LDS. BLDS (main launch only): B in
// the wave's LDS arena; otherwise B is read from global memory (L2 / MALL).
// The slot at position idx (< 0: none) of the main solver list in heaviest-first order: the
// block-count buckets from the top down (o_hist / o_blist). Lanes of one slot pass the same idx;
// the wave's (up to four) positions are resolved together: lane k scans bucket top - k.
__device__ __forceinline__ int sorted_slot(const Pipe& P, int idx, int LPS) {
  const int* hist = P.at<int>(P.o_hist);
  const int* bl = P.at<int>(P.o_blist);
  const int l = lane_id();
  int slot = -1, acc = 0;
  for (int top = P.nbk - 1; top >= 1; top -= 64) {
    const int b = top - l;
    const int h = b >= 1 ? hist[b] : 0;
    int x = h;  // inclusive prefix over the lanes (descending buckets)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (l >= o) x += y;
    }
    for (int q = 0; q < 64; q += LPS) {
      const int iq = __shfl(idx, q);
      const unsigned long long m = __ballot(iq >= 0 && acc + x > iq);
      if (m) {
        const int f = __ffsll((long long)m) - 1;
        const int xf = __shfl(x, f), hf = __shfl(h, f);
        const int rank = iq - (acc + xf - hf);
        const int sq = bl[(size_t)(top - f) * P.S + rank];
        if (l >= q && l < q + LPS && slot < 0) slot = sq;
      }
    }
    acc += __shfl(x, 63);
  }
  return slot;
}

template <typename T, int EPL, int LPS, bool BLDS, bool SQG = false, bool DOFB = false>
__global__ void __launch_bounds__(64) k_pgs_groups(Pipe P, int maxit, T tol, T scale, int spw, int big) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (!big && blockIdx.x == 0 && threadIdx.x == 0) P.ctr()[0] = 0;  // fixup list count, filled by the finisher
  const int cnt = P.ctr()[big ? 2 : 1];
  const int* list = P.at<int>(P.o_k2big);
  const int spn = spw < 0 ? -spw : spw;
  const int s = threadIdx.x / LPS;
  // the wide launch's few long chains (slots over the main launch's rows) run beside the whole
  // main launch and end the step when they trail it: they take their SIMD first
  if (big) __builtin_amdgcn_s_setprio(3);
  const bool dup = big && BLDS;  // the wide LDS-B launch: one slot per wave, every lane group on it
  for (int base = blockIdx.x * spn; base < cnt; base += gridDim.x * spn) {
    const int idx = dup ? base : (s < spn && base + s < cnt) ? base + s : -1;
    const int slot = big ? (idx >= 0 ? list[idx] : -1) : sorted_slot(P, idx, LPS);
    if constexpr (!BLDS && !SQG) {
      if (!big) {
        int nm = slot >= 0 ? P.at<int>(P.o_ne)[slot] : 0;
        nm = max(nm, __shfl_xor(nm, 16));
        nm = max(nm, __shfl_xor(nm, 32));
        nm = __builtin_amdgcn_readfirstlane(nm);
        // the launch's longest chains (heaviest first: the first waves): first pick of their
        // SIMD's issue slots over co-resident waves (another stream's kernels, the next stage of a
        // stream shard), as the wide launch does; no effect on any result
        const bool hi = nm > P.prio_rows;
        if (hi) __builtin_amdgcn_s_setprio(3);
        // a wave holding a slot over the main launch's LDS-scalar rows reads its row scalars from
        // the pipe instead; same arithmetic, so the same results
        if (P.hmain && nm > P.capE) {
          pgs_group<T, EPL, LPS, false, true, DOFB>(P, smem, slot, P.maxE, maxit, tol, scale, spw, -1);
          if (hi) __builtin_amdgcn_s_setprio(0);
          __syncthreads();
          continue;
        }
        pgs_group<T, EPL, LPS, false, false, DOFB>(P, smem, slot, P.capE, maxit, tol, scale, spw, -1);
        if (hi) __builtin_amdgcn_s_setprio(0);
        __syncthreads();
        continue;
      }
    }
    pgs_group<T, EPL, LPS, BLDS && true, SQG, DOFB>(P, smem, slot, big ? P.maxE : P.capE, maxit, tol, scale, spw,
                                                  big ? P.warena : -1);
    __syncthreads();  // the next group reuses the LDS
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
// bank record bi restarts for `episode` from the 36 draws in e.vec1 (LDS)
template <typename T>
__device__ __forceinline__ void bank_init_draws(const DevModel<T>& m, Env<T>& e, const SoccerIds<T>& ids, const Pipe& P,
                                                int bi, int episode, uint64_t seed) {
  int l = lane_id();
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
template <typename T>
__device__ __forceinline__ void bank_init(const DevModel<T>& m, Env<T>& e, const SoccerIds<T>& ids, const Pipe& P, int env,
                                          int b, int episode, uint64_t seed, int env_offset) {
  soccer_philox_draws(seed, (uint32_t)(env_offset + env), (uint32_t)episode, ids.n_noise, e.vec1);
  wsync();
  bank_init_draws(m, e, ids, P, env * P.R + b, episode, seed);
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

// the settled reset of bank record bi becomes env's live state for episode E (soccer_env.py:
// 347-396 outcome: state, obs, prev snapshots, wind, zero stats / step / goal); episode E + 1
template <typename T>
__device__ __forceinline__ void bank_copy_live(const DevModel<T>& m, const Pipe& P, mgx_state s, mgx_soccer_env ev,
                                               float* obs, int env, int bi, int E) {
  int l = lane_id();
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
    if (ev.episode) ev.episode[env] = E + 1;
  }
  wsync();
}

// Install the ready bank of env `env` into its live state and restart the bank for
// episode + R. Returns false if the bank is not ready (caller falls back).
template <typename T>
__device__ __forceinline__ bool bank_install(const DevModel<T>& m, Env<T>& e, const SoccerIds<T>& ids, const Pipe& P,
                                             mgx_state s, mgx_soccer_env ev, float* obs, uint64_t seed, int env_offset,
                                             int env) {
  int E = ev.episode[env];
  int b = E % P.R;
  int bi = env * P.R + b;
  bool ready = P.at<int>(P.o_bk)[bi] == 10 && P.at<int>(P.o_bep)[bi] == E && P.at<uint64_t>(P.o_bseed)[bi] == seed;
  if (!ready) return false;
  bank_copy_live(m, P, s, ev, obs, env, bi, E);
  bank_init(m, e, ids, P, env, b, E + P.R, seed, env_offset);
  return true;
}

// ------------------------------------------------------------------ one-wave settle
// One settle step of bank record bi in one wave, through pipe slot `slot`: the pipeline's own
// stages in sequence — stage_rows, the PGS of the one slot (pgs_group, lane group 0 of the
// wave), the finisher's finish_physics / checkAcc template / bank store. A reset settled here is
// bit-identical to one settled as extra slots of the pipeline launches, so the fallback for a
// bank that is not ready (and reset()) produces exactly what a ready bank would have: the bank
// count is a performance knob only. Returns with the finisher's Env (layout Mf) in `smem`.
template <typename T, int EPL, int LPS>
__device__ __forceinline__ void settle_step(const DevModel<T>& Ms, const DevModel<T>& Mf, const SoccerIds<T>& ids,
                                            const Pipe& P, char* smem, Env<T>& f, int bi, int slot,
                                            int maxit, T tol, T scale, bool last) {
  {
    Env<T> e;
    env_bind(Ms, e, smem);
    bind_carry_tail(Ms, e, P, slot);
    bank_load_state(Ms, e, P, bi);
    int warn = 0;  // mj_checkPos / mj_checkVel
    if (any_bad(e.qpos, Ms.nq)) { reset_env(Ms, e); warn++; }
    if (any_bad(e.qvel, Ms.nv)) { reset_env(Ms, e); warn++; }
    stage_rows(Ms, e, P, slot, warn, false);
  }
  __threadfence();
  __syncthreads();
  pgs_group<T, EPL, LPS, false>(P, smem, threadIdx.x < LPS ? slot : -1, P.maxE, maxit, tol, scale, 64 / LPS);
  __threadfence();
  __syncthreads();
  env_bind(Mf, f, smem);
  int warn = load_carry(Mf, f, P, slot);
  if (!finish_physics(Mf, f, P, slot)) {
    load_template(Mf, f, P);
    warn++;
  }
  bank_store_state(Mf, f, P, bi, warn);
  if (last) bank_finalize(Mf, f, ids, P, bi);
  __threadfence();
  __syncthreads();
}

// Restart record bi for `episode` (draws: host [36] or nullptr for Philox) and settle it
// (soccer_env.py:378-379: 10 mj_steps from the randomised pose); bk = 10 at the end.
template <typename T, int EPL, int LPS>
__device__ __forceinline__ void settle_reset(const DevModel<T>& Ms, const DevModel<T>& Mf, const SoccerIds<T>& ids,
                                             const Pipe& P, char* smem, int env, int bi, int episode,
                                             const T* draws, uint64_t seed, int env_offset, int maxit, T tol, T scale) {
  {
    Env<T> e;
    env_bind(Ms, e, smem);
    bind_carry_tail(Ms, e, P, env);
    if (draws) {
      if (lane_id() < 36) e.vec1[lane_id()] = draws[lane_id()];
    } else {
      soccer_philox_draws(seed, (uint32_t)(env_offset + env), (uint32_t)episode, ids.n_noise, e.vec1);
    }
    wsync();
    bank_init_draws(Ms, e, ids, P, bi, episode, seed);
  }
  __threadfence();
  __syncthreads();
  Env<T> f;
  for (int t = 0; t < 10; t++) settle_step<T, EPL, LPS>(Ms, Mf, ids, P, smem, f, bi, env, maxit, tol, scale, t == 9);
  if (lane_id() == 0) P.at<int>(P.o_bk)[bi] = 10;
  __threadfence();
  __syncthreads();
}

enum { SETTLE_RESET = 0, SETTLE_FIXUP = 1 };
// reset() of a staged batch (SETTLE_RESET: one workgroup per env; with Philox draws and banks it
// also prefills the env's R banks) and the step's fallback for banks that were not ready
// (SETTLE_FIXUP: grid-stride over the finisher's list). Every reset goes through settle_reset,
// the pipeline's arithmetic.
template <typename T, int EPL, int LPS>
__global__ void __launch_bounds__(64) k_soccer_settle(DevModel<T> Ms, DevModel<T> Mf, SoccerIds<T> ids, mgx_state s,
                                                      mgx_soccer_env ev, const T* draws, float* obs, uint64_t seed,
                                                      int env_offset, int n_env, const uint8_t* mask, Pipe P, int mode,
                                                      int maxit, T tol, T scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int cnt = mode == SETTLE_FIXUP ? P.ctr()[0] : n_env;
  for (int i = blockIdx.x; i < cnt; i += gridDim.x) {
    const int env = mode == SETTLE_FIXUP ? P.at<int>(P.o_fix)[i] >> 2 : i;
    if (mode == SETTLE_RESET && mask && !mask[env]) continue;
    const int E = ev.episode ? ev.episode[env] : 0;
    const int bi = P.R > 0 ? env * P.R + E % P.R : env;  // R = 0: one scratch record per env
    const T* d = draws ? draws + (size_t)env * 36 : nullptr;
    settle_reset<T, EPL, LPS>(Ms, Mf, ids, P, smem, env, bi, E, d, seed, env_offset, maxit, tol, scale);
    bank_copy_live(Mf, P, s, ev, obs, env, bi, E);
    if (P.R > 0 && mode == SETTLE_FIXUP) {
      // as bank_install: the consumed bank restarts for episode E + R (the pipeline settles it)
      Env<T> e;
      env_bind(Ms, e, smem);
      bind_carry_tail(Ms, e, P, env);
      bank_init(Ms, e, ids, P, env, E % P.R, E + P.R, seed, env_offset);
    } else if (P.R > 0 && !draws) {
      // reset(): prefill the banks of episodes E + 1 .. E + R, so the first R terminations never wait
      for (int k = 1; k <= P.R; k++)
        settle_reset<T, EPL, LPS>(Ms, Mf, ids, P, smem, env, env * P.R + (E + k) % P.R, E + k, nullptr, seed,
                                  env_offset, maxit, tol, scale);
    } else if (lane_id() == 0) {
      P.at<int>(P.o_bk)[bi] = -1;  // a scratch record (R = 0, or host draws): nothing to settle
    }
    __threadfence();
    __syncthreads();
  }
}

}  // namespace mgx
