// mgx_common.h — device model tables, per-env LDS layout and wavefront helpers.
//
// Execution model: one 64-lane wavefront = one environment. A workgroup is
// exactly one wavefront, so __syncthreads() is a cheap wave barrier (s_waitcnt + s_barrier
// on a single wave) and LDS is private to the env. Lane k owns dof k (nv <= 64), body k,
// joint k, ... in the stages that parallelise over them; per-row solver data is spread
// lane r % 64, register slot r / 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MGX_WAVE 64
#define MGX_MAX_NV 64
#define MGX_MAX_NV_WIDE 128   // wide kernels (mgx_wide.h): two dofs per lane, dof d on lane d % 64
#define MGX_MAX_NBODY 64
#define MGX_MAX_DEPTH 16      // longest dof chain (root..dof), soccer: 13
#define MGX_MAX_CONPAIR 8     // contacts per geom pair (box-box)
// more candidate pairs than this: bounding-box prefilters after the spheres (default; soccer 251,
// martial arts 294, assembly 803, construction 1,202, bipedal 3,185 — not dancing's 106, where the
// filters cost more than the narrowphase they save, nor parkour's 48)
#define MGX_TIGHT_BROADPHASE_PAIRS 200
#define MGX_EFC_SLOTS 6       // staged soccer step: max_nefc <= 64 * MGX_EFC_SLOTS = 384

namespace mgx {

enum { JFREE = 0, JBALL = 1, JSLIDE = 2, JHINGE = 3 };
enum { GPLANE = 0, GHFIELD = 1, GSPHERE = 2, GCAPSULE = 3, GELLIPSOID = 4, GCYLINDER = 5, GBOX = 6 };
enum { C_LIMIT_JOINT = 3, C_CONTACT_FRICTIONLESS = 5, C_CONTACT_PYRAMIDAL = 6 };

// LDS layout, in elements of T (reals) or int32 (ints), offsets computed on the host.
struct Layout {
  int qpos, qvel, ctrl, xfrc, xpos, xquat, xmat, xipos, ximat, subtree_com, cinert, crb, cvel, cfrc;
  int xaxis, xanchor, cdof, cdof_dot, qLD, qMH, vec0, vec1, vec2, vec3, geom_xpos, geom_xmat, act_force, cacc, rowc;
  int con_dist, con_pos, con_frame, con_mu;
  int efc, efc_margin, efc_blk;
  int Bmat, Bstride;
  int reals;  // total reals
  // int region (after reals)
  int con_geom, con_pair, act_list, efc_type, efc_id, con_efcadr;
  int ints;
  int bytes;
  int max_ncon, max_nefc, max_active;
  // staged pipeline: reals [0, carry_reals) and ints [0, carry_ints) are handed from the row
  // builder to the finisher through HBM; B rows are built chunk_rows at a time
  int staged, carry_reals, carry_ints, chunk_rows;
  // RK4 stage storage (X[0] positions, dX velocities; integrator == RK4 only)
  int rk;
  // 1: the monolithic kernel keeps B rows in per-env global scratch (gB_stride reals per env)
  // instead of LDS, for models whose rows do not fit the LDS budget
  int gB, gB_stride;
  // gB only: rows per chunk staged into the (dead) phase-A union region for the row transform
  int tchunk;
  // Newton solver (solver == mjSOL_NEWTON, monolithic kernels only): nv x nv Hessian
  int hess;
  // > 0: the broadphase survivor list lives at this real offset (inside the dead phase-A
  // union) instead of the int region (monolithic rows-in-scratch PGS models; the staged row
  // builder, where efc_id shares it)
  int act_union;
  // staged row builder: carry reals [carry_lds, carry_reals) (xfrc_applied, qMH) live in the
  // slot's pipe carry in global memory instead of LDS (bind_carry_tail); the finisher's layout
  // holds the whole carry in LDS
  int carry_lds;
  // staged row builder: geom poses are computed right before collision (geom_poses), from xquat,
  // over the phase-A arrays dead by then; contacts keep their normal only (3 reals, stride
  // cfs = 3; the frame is rebuilt where it is read) instead of the 9-real frame
  int late_geom, cfs;
  // collision(): the box prefilters after the bounding spheres (mgx_collide.h box_box_separated /
  // sphere_box_separated; conservative, the contact list is unchanged). Set per model: on when it
  // has more than MGX_TIGHT_BROADPHASE_PAIRS candidate pairs (MGX_TIGHT_BROADPHASE=0/1 overrides)
  int tight_bp;
  // staged row builder: LDS copy of xfrc_applied for the velocity stage (its per-dof force sums
  // read it nbody times per lane), in the phase-A region
  int xfrc_lds;
  // staged row builder: the contact points (3 reals per contact, written by collision, read by the
  // row blocks) live in the slot's pipe storage (Pipe.o_cpos, bind_carry_tail), not in LDS
  int gcon;
};
// Derived, not stored (the Layout / DevModel kernel-argument layout stays that of the task
// kernels): wide Newton models (nv > 64, rows in global scratch) keep the per-row constraint data
// efc / efc_margin in the env's global scratch after its rows, at these real offsets, and store
// the Hessian as a packed lower triangle (row i at i (i + 1) / 2); Newton models keep the helper
// wave's command words (mgx_physics.h team_begin) in the four ints after con_efcadr.
__host__ __device__ inline int mgx_align(int x, int a) { return (x + a - 1) / a * a; }
__host__ __device__ inline int gb_efc_off(const Layout& L, int real_bytes) {
  return mgx_align(L.max_nefc * L.Bstride, 16 / real_bytes);
}
__host__ __device__ inline int gb_efm_off(const Layout& L, int real_bytes) {
  return gb_efc_off(L, real_bytes) + mgx_align(8 * L.max_nefc, 16 / real_bytes);
}
__host__ __device__ inline int team_off(const Layout& L) { return L.con_efcadr + 4; }

// Device-resident model: pointers into one device allocation.
template <typename T>
struct DevModel {
  int nq, nv, nu, nbody, njnt, ngeom, npair, nM, nmaskword;
  int solver, integrator, cone, iterations;
  T timestep, tolerance, impratio, meaninertia, gravity[3];
  // bodies
  const int *body_parentid, *body_rootid, *body_jntnum, *body_jntadr, *body_dofnum, *body_dofadr;
  const int *body_subtree_end, *body_chain, *body_depth;  // chain: [nbody][MAX_DEPTH] root..body
  const uint32_t *body_dofmask;                           // [nbody][nmaskword]
  const T *body_pos, *body_quat, *body_ipos, *body_iquat, *body_mass, *body_inertia, *body_invweight0;
  // joints
  const int *jnt_type, *jnt_bodyid, *jnt_qposadr, *jnt_dofadr, *jnt_limited;
  const T *jnt_pos, *jnt_axis, *jnt_range, *jnt_stiffness, *jnt_margin, *jnt_solref, *jnt_solimp;
  // dofs
  const int *dof_bodyid, *dof_jntid, *dof_parentid, *dof_Madr, *dof_chainlen, *dof_anc;  // anc: [nv][MAX_DEPTH]
  const uint64_t *dof_ancmask;  // bit i set if dof i is a strict ancestor of the dof
  const uint64_t *dof_ancmask_hi;  // the same for ancestors i = 64 .. 127 (bit i - 64; wide models)
  const int *dof_ancadr;        // [nv][MAX_DEPTH]: dof_Madr of ancestor t (0 past the chain)
  const T *dof_armature, *dof_damping, *dof_invweight0;
  // geoms
  const int *geom_type, *geom_bodyid;
  const T *geom_size, *geom_pos, *geom_quat, *geom_rbound;
  // pairs
  const int *pair_geom, *pair_condim;
  // broadphase records, one per candidate pair, so a round of 64 pairs is two vector loads with no
  // dependent gathers (prefetched a round ahead): {g1, g2, kind, 0} — kind bit 0: g1 is a plane,
  // bit 1: both geoms have a bounding box (box, capsule, cylinder; geom_obb), bit 2 / 3: g1 / g2 is
  // a sphere and the other has a bounding box — and {reach, margin, the sphere's radius, 0}, reach =
  // rbound[g1] + rbound[g2] + margin (plane: rbound[g2] + margin), the bounding-sphere tests' sums
  const int* pair_bpi;
  const T* pair_bpr;
  const T* geom_obb;  // the geom's bounding box half-sizes in its frame: box (sx, sy, sz), capsule
                      // (r, r, half-length + r), cylinder (r, r, half-height); 0 otherwise
  const T *pair_friction, *pair_margin, *pair_gap, *pair_solref, *pair_solimp;
  // actuators
  const int *actuator_trnid, *actuator_ctrllimited, *actuator_forcelimited;
  const T *actuator_gear, *actuator_ctrlrange, *actuator_forcerange, *actuator_gainprm, *actuator_biasprm;
  const T *qpos0, *qpos_spring;
  Layout L;
};

// ------------------------------------------------------------------ diagnostic stamps
// Built only with -DMGX_PROFILE (libmgx_prof.so, never the shipped library): per-env cycle
// sums per stage, read back by tools/stage_profile.py. Stamps never feed any output.
#ifdef MGX_PROFILE
// one buffer pointer per translation unit (no relocatable device code); each TU exports its
// setter with MGX_PROF_SETTER(name)
static __device__ unsigned long long* g_mgx_prof = nullptr;
#define MGX_PROF_SETTER(name)                                                                     \
  extern "C" int name(void* p) {                                                                 \
    unsigned long long* q = (unsigned long long*)p;                                               \
    return hipMemcpyToSymbol(HIP_SYMBOL(mgx::g_mgx_prof), &q, sizeof(q)) == hipSuccess ? 0 : -3; \
  }
#define MGX_STAMP_DECL unsigned long long _mgx_t0 = __builtin_amdgcn_s_memtime();
#define MGX_STAMP(slot)                                                                 \
  do {                                                                                  \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    unsigned long long _t = __builtin_amdgcn_s_memtime();                               \
    if (g_mgx_prof && threadIdx.x == 0) g_mgx_prof[blockIdx.x * 32 + (slot)] += _t - _mgx_t0; \
    _mgx_t0 = _t;                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                                  \
  } while (0)
#else
#define MGX_PROF_SETTER(name)
#define MGX_STAMP_DECL
#define MGX_STAMP(slot) do {} while (0)
#endif

// ------------------------------------------------------------------ wave helpers
// MGX_TEAM (the translation units whose kernels run a helper wave beside wave 0: assembly and
// construction): lane = thread index mod 64. Every other kernel is one wave per workgroup and keeps
// the plain thread index (its code generation unchanged).
#ifdef MGX_TEAM
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
#else
__device__ __forceinline__ int lane_id() { return threadIdx.x; }
#endif
__device__ __forceinline__ void wsync() { __syncthreads(); }

__device__ __forceinline__ float readlane(float x, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), l));
}
__device__ __forceinline__ double readlane(double x, int l) {
  int2 v = __builtin_bit_cast(int2, x);
  v.x = __builtin_amdgcn_readlane(v.x, l);
  v.y = __builtin_amdgcn_readlane(v.y, l);
  return __builtin_bit_cast(double, v);
}
__device__ __forceinline__ int readlane(int x, int l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ uint64_t readlane_u64(uint64_t x, int l) {
  uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)x, l), hi = __builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// full-wave sum, result in every lane (butterfly over 6 xor steps)
template <typename T>
__device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) x += __shfl_xor(x, o);
  return x;
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float wave_sum_dpp(float x) {
  // rows of 16 with DPP (quad_perm 1,0,3,2 / 2,3,0,1, row_ror 4 / 8), then the four row
  // totals through readlane: fixed order, identical in every lane
  x += dpp_f<0xB1>(x);
  x += dpp_f<0x4E>(x);
  x += dpp_f<0x124>(x);
  x += dpp_f<0x128>(x);
  return (readlane(x, 0) + readlane(x, 16)) + (readlane(x, 32) + readlane(x, 48));
}
__device__ __forceinline__ double wave_sum_dpp(double x) { return wave_sum(x); }

// full-wave sum, 6 DPP steps + one readlane: quad_perm x2, row_half_mirror, row_mirror (row
// totals in every lane), row_bcast:15 / row_bcast:31 (gfx9 DPP) -> total in lane 63
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_upd(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROWS, 0xf, false));
}
__device__ __forceinline__ float wave_sum_fast(float x) {
  x += dpp_f<0xB1>(x);
  x += dpp_f<0x4E>(x);
  x += dpp_f<0x141>(x);
  x += dpp_f<0x140>(x);
  x += dpp_upd<0x142, 0xa>(x);
  x += dpp_upd<0x143, 0xc>(x);
  return readlane(x, 63);
}
// fp64 through the same DPP patterns: both 32-bit halves move with v_mov_b32_dpp (pure data
// movement, exact), so an fp64 reduction costs VALU steps instead of ds_bpermute round trips
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  int2 h = __builtin_bit_cast(int2, v);
  h.x = __builtin_amdgcn_mov_dpp(h.x, CTRL, 0xf, 0xf, false);
  h.y = __builtin_amdgcn_mov_dpp(h.y, CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, h);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_upd_d(double v) {
  int2 h = __builtin_bit_cast(int2, v);
  h.x = __builtin_amdgcn_update_dpp(0, h.x, CTRL, ROWS, 0xf, false);
  h.y = __builtin_amdgcn_update_dpp(0, h.y, CTRL, ROWS, 0xf, false);
  return __builtin_bit_cast(double, h);
}
__device__ __forceinline__ double wave_sum_fast(double x) {
  x += dpp_d<0xB1>(x);
  x += dpp_d<0x4E>(x);
  x += dpp_d<0x141>(x);
  x += dpp_d<0x140>(x);
  x += dpp_upd_d<0x142, 0xa>(x);
  x += dpp_upd_d<0x143, 0xc>(x);
  return readlane(x, 63);
}

// four independent full-wave sums, DPP steps interleaved so the hazard wait states of one
// chain are filled by the others (same per-chain order as wave_sum_fast)
__device__ __forceinline__ void wave_sum4(float& a, float& b, float& c, float& d) {
#define MGX_STEP4(OP) a += OP(a); b += OP(b); c += OP(c); d += OP(d);
  MGX_STEP4(dpp_f<0xB1>)
  MGX_STEP4(dpp_f<0x4E>)
  MGX_STEP4(dpp_f<0x141>)
  MGX_STEP4(dpp_f<0x140>)
#define MGX_B15(x) dpp_upd<0x142, 0xa>(x)
#define MGX_B31(x) dpp_upd<0x143, 0xc>(x)
  MGX_STEP4(MGX_B15)
  MGX_STEP4(MGX_B31)
#undef MGX_B15
#undef MGX_B31
#undef MGX_STEP4
  a = readlane(a, 63); b = readlane(b, 63); c = readlane(c, 63); d = readlane(d, 63);
}
__device__ __forceinline__ void wave_sum4(double& a, double& b, double& c, double& d) {
#define MGX_STEP4(OP) a += OP(a); b += OP(b); c += OP(c); d += OP(d);
  MGX_STEP4(dpp_d<0xB1>)
  MGX_STEP4(dpp_d<0x4E>)
  MGX_STEP4(dpp_d<0x141>)
  MGX_STEP4(dpp_d<0x140>)
#define MGX_B15(x) dpp_upd_d<0x142, 0xa>(x)
#define MGX_B31(x) dpp_upd_d<0x143, 0xc>(x)
  MGX_STEP4(MGX_B15)
  MGX_STEP4(MGX_B31)
#undef MGX_B15
#undef MGX_B31
#undef MGX_STEP4
  a = readlane(a, 63); b = readlane(b, 63); c = readlane(c, 63); d = readlane(d, 63);
}

__device__ __forceinline__ unsigned long long ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int prefix_count(unsigned long long mask) {  // set bits below this lane
  return __builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0));
}
__device__ __forceinline__ int popc64(unsigned long long m) { return __popcll(m); }

// inclusive-exclusive prefix sum of small ints across the wave
__device__ __forceinline__ int wave_excl_scan(int v, int* total) {
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int y = __shfl_up(x, o);
    if (lane_id() >= o) x += y;
  }
  *total = __builtin_amdgcn_readfirstlane(__shfl(x, 63));  // uniform
  return x - v;
}

// ------------------------------------------------------------------ policy actions
// One env's action row: float32, or float64 when the env struct's action_f64 is set. The
// reference's np.clip(action, low, high) keeps a float64 policy's dtype (the bounds are float32
// arrays or Python floats), so ctrl and every action term of the reward follow in float64; a
// float32 action keeps numpy's float32 arithmetic.
struct ActRow {
  const void* p;
  int f64;
  __device__ ActRow(const void* base, int f64_, size_t row, int n)
      : p(f64_ ? (const void*)((const double*)base + row * n) : (const void*)((const float*)base + row * n)),
        f64(f64_) {}
  __device__ const float* f() const { return static_cast<const float*>(p); }
  __device__ const double* d() const { return static_cast<const double*>(p); }
  __device__ double at(int i) const { return f64 ? d()[i] : (double)f()[i]; }
};

// ------------------------------------------------------------------ small math (MuJoCo forms)
template <typename T> __device__ __forceinline__ T clampv(T x, T lo, T hi) { return x < lo ? lo : (x > hi ? hi : x); }
template <typename T> __device__ __forceinline__ T dot3(const T* a, const T* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
template <typename T> __device__ __forceinline__ void cross3(T* r, const T* a, const T* b) {
  T t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
template <typename T> __device__ __forceinline__ T minval() { return (T)1e-15; }
template <> __device__ __forceinline__ float minval<float>() { return 1e-15f; }

template <typename T> __device__ __forceinline__ T normalize3(T* v) {
  T n = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  if (n < minval<T>()) { v[0] = 1; v[1] = 0; v[2] = 0; }
  else { T s = (T)1 / n; v[0] *= s; v[1] *= s; v[2] *= s; }
  return n;
}
template <typename T> __device__ __forceinline__ void normalize4(T* q) {
  T n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < minval<T>()) { q[0] = 1; q[1] = q[2] = q[3] = 0; }
  else if (fabs(n - (T)1) > minval<T>()) { T s = (T)1 / n; q[0] *= s; q[1] *= s; q[2] *= s; q[3] *= s; }
}
template <typename T> __device__ __forceinline__ void mulquat(T* r, const T* a, const T* b) {
  T t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  T t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  T t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  T t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}
template <typename T> __device__ __forceinline__ void quat2mat(T* r, const T* q) {
  if (q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0) {
    r[0] = 1; r[1] = 0; r[2] = 0; r[3] = 0; r[4] = 1; r[5] = 0; r[6] = 0; r[7] = 0; r[8] = 1;
    return;
  }
  T q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  T q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
  T q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
  r[0] = q00 + q11 - q22 - q33; r[4] = q00 - q11 + q22 - q33; r[8] = q00 - q11 - q22 + q33;
  r[1] = 2 * (q12 - q03); r[2] = 2 * (q13 + q02); r[3] = 2 * (q12 + q03);
  r[5] = 2 * (q23 - q01); r[6] = 2 * (q13 - q02); r[7] = 2 * (q23 + q01);
}
template <typename T> __device__ __forceinline__ void rotvecquat(T* r, const T* v, const T* q) {
  if (v[0] == 0 && v[1] == 0 && v[2] == 0) { r[0] = r[1] = r[2] = 0; return; }
  if (q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0) { r[0] = v[0]; r[1] = v[1]; r[2] = v[2]; return; }
  T t0 = q[0] * v[0] + q[2] * v[2] - q[3] * v[1];
  T t1 = q[0] * v[1] + q[3] * v[0] - q[1] * v[2];
  T t2 = q[0] * v[2] + q[1] * v[1] - q[2] * v[0];
  T o0 = v[0] + 2 * (q[2] * t2 - q[3] * t1);
  T o1 = v[1] + 2 * (q[3] * t0 - q[1] * t2);
  T o2 = v[2] + 2 * (q[1] * t1 - q[2] * t0);
  r[0] = o0; r[1] = o1; r[2] = o2;
}
template <typename T> __device__ __forceinline__ void axisangle2quat(T* q, const T* ax, T ang) {
  if (ang == 0) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  T s = sin(ang * (T)0.5);
  q[0] = cos(ang * (T)0.5); q[1] = ax[0] * s; q[2] = ax[1] * s; q[3] = ax[2] * s;
}
template <typename T> __device__ __forceinline__ void mulmatvec3(T* r, const T* M, const T* v) {
  T t0 = M[0] * v[0] + M[1] * v[1] + M[2] * v[2];
  T t1 = M[3] * v[0] + M[4] * v[1] + M[5] * v[2];
  T t2 = M[6] * v[0] + M[7] * v[1] + M[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
template <typename T> __device__ __forceinline__ void mulmatTvec3(T* r, const T* M, const T* v) {
  T t0 = M[0] * v[0] + M[3] * v[1] + M[6] * v[2];
  T t1 = M[1] * v[0] + M[4] * v[1] + M[7] * v[2];
  T t2 = M[2] * v[0] + M[5] * v[1] + M[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
template <typename T> __device__ __forceinline__ bool isbad(T x) { return x != x || x > (T)1e10 || x < (T)-1e10; }

template <typename T> __device__ __forceinline__ T dot6(const T* a, const T* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}
template <typename T> __device__ __forceinline__ void mulinertvec(T* res, const T* i, const T* v) {
  res[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  res[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  res[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  res[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  res[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  res[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}
template <typename T> __device__ __forceinline__ void crossmotion(T* res, const T* v, const T* u) {
  res[0] = -v[2] * u[1] + v[1] * u[2];
  res[1] = v[2] * u[0] - v[0] * u[2];
  res[2] = -v[1] * u[0] + v[0] * u[1];
  res[3] = -v[2] * u[4] + v[1] * u[5];
  res[4] = v[2] * u[3] - v[0] * u[5];
  res[5] = -v[1] * u[3] + v[0] * u[4];
  res[3] += -v[5] * u[1] + v[4] * u[2];
  res[4] += v[5] * u[0] - v[3] * u[2];
  res[5] += -v[4] * u[0] + v[3] * u[1];
}
template <typename T> __device__ __forceinline__ void crossforce(T* res, const T* v, const T* f) {
  res[0] = -v[2] * f[1] + v[1] * f[2];
  res[1] = v[2] * f[0] - v[0] * f[2];
  res[2] = -v[1] * f[0] + v[0] * f[1];
  res[3] = -v[2] * f[4] + v[1] * f[5];
  res[4] = v[2] * f[3] - v[0] * f[5];
  res[5] = -v[1] * f[3] + v[0] * f[4];
  res[0] += -v[5] * f[4] + v[4] * f[5];
  res[1] += v[5] * f[3] - v[3] * f[5];
  res[2] += -v[4] * f[3] + v[3] * f[4];
}

}  // namespace mgx
