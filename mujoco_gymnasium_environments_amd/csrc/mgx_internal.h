// mgx_internal.h — host-side definitions shared by the translation units of libmgx.so
// (mgx_api.hip: model, physics and soccer; mgx_step.hip: generic step; mgx_parkour.hip:
// quadruped_parkour; mgx_bipedal.hip: bipedal_rescue; mgx_dancing.hip: humanoid_dancing).
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/mgx.h"
#include "mgx_bipedal.h"
#include "mgx_construction.h"
#include "mgx_dancing.h"
#include "mgx_martial.h"
#include "mgx_parkour.h"
#include "mgx_staged.h"

namespace mgx {
// A/B and test hooks (MGX_* environment variables). Read once per model, in mgx_model_create, and
// kept with the model, so a launch never depends on the environment at call time. None of them
// changes a result: each selects another schedule of the same arithmetic (tests/test_gpu_capacity.py
// checks the ones that move slots between launches bit for bit). MGX_PGS_LPS (solver lanes per
// slot) is read once per process (pgs_lanes): the solver kernels' LDS limits are set from it.
struct Hooks {
  int pgs_lds_rows = 0;  // MGX_PGS_LDS_ROWS: the soccer main solver launch's LDS rows (0: model default)
  int rk_lds_rows = 0;   // MGX_RK_LDS_ROWS: the RK4 main solver launch's LDS rows (0: 256)
  int pgs_single = 0;    // MGX_PGS_SINGLE: one main launch over every slot, scalars from the pipe
  int pgs_lds_b = 0;     // MGX_PGS_LDS_B: the main launch copies B into an LDS arena
  int pgs_arena = 0;     // MGX_PGS_ARENA: that arena's bytes (0: MGX_PGS_ARENA_F32 / _F64)
  int pgs_lds_pad = 0;   // MGX_PGS_LDS_PAD: pad the main solver launch's LDS (occupancy probe)
  int pgs_wide_lds = 1;  // MGX_PGS_WIDE_LDS: the wide launch copies its slot's B into LDS
  int pgs_spw = 0;       // MGX_PGS_SPW: slots per solver wave (debug)
  int pgs_wpc = 4;       // MGX_PGS_WPC: main solver launch's waves per CU its LDS rows are sized for
  int pgs_prio_rows = 0; // MGX_PGS_PRIO_ROWS: rows above which a main-launch solver wave raises its priority
  int tight_bp = -1;     // MGX_TIGHT_BROADPHASE: box prefilters in the broadphase (-1: by the pair count)
  int side_stream = 1;   // MGX_SIDE_STREAM: the wide solver launch on a side stream
  int gcon = 1;          // MGX_GCON: the row builder's contact points in the pipe (0: in LDS)
  int rows_lds = 0;      // MGX_ROWS_LDS: pad the row builder's LDS (occupancy probe)
};
Hooks read_hooks();
}  // namespace mgx

struct mgx_model {
  mgx::Hooks hooks;
  int precision;
  int device;
  void* dbuf = nullptr;
  size_t dbytes = 0;
  mgx::DevModel<float> mf, mfs, mff;   // monolithic / staged row builder / staged finisher layouts
  mgx::DevModel<double> md, mds, mdf;
  mgx::Layout L, Ls, Lf;
  bool soccer_ok = false;
  mgx::SoccerIds<float> sf;
  mgx::SoccerIds<double> sd;
  bool parkour_ok = false;
  mgx::ParkourIds<float> pkf;
  mgx::ParkourIds<double> pkd;
  bool martial_ok = false;
  mgx::MartialIds ma;
  bool bipedal_ok = false;
  mgx::BipedalIds bp;
  bool dancing_ok = false;
  mgx::DancingIds dn;
  bool assembly_ok = false;
  mgx_assembly_ids as;
  bool construction_ok = false;
  mgx::ConstructionIds cn;
  int npair;
  bool wide = false;       // nv > 64: only the wide kernels (mgx_wide.h) run this model
  bool staged_ok = false;  // the staged soccer pipeline supports this model's capacities
  bool staged_rk_ok = false;  // the staged RK4 pipeline (bipedal) supports this model
};

namespace mgx {
// Debug dump of one forward pass (stage outputs): offsets into one env's record
// (mgx_debug_forward / mgx_debug_layout; the wide kernels write the same layout)
struct DbgOff {
  int xpos, xquat, xipos, subtree_com, cinert, cdof, qM, qLD, geom_xpos, geom_xmat, ncon, con_dist, con_pos,
      con_frame, con_geom, nefc, efc_type, efc_id, efc_pos, efc_margin, efc_R, efc_aref, Bmat, cvel, cdof_dot,
      qfrc_smooth, qacc_smooth, efc_force, qacc, qfrc_constraint, niter, total;
};
inline DbgOff dbg_offsets(int nb, int nv, int nM, int ng, int C, int E) {
  DbgOff o;
  int p = 0;
  auto take = [&](int n) { int r = p; p += n; return r; };
  o.xpos = take(3 * nb); o.xquat = take(4 * nb); o.xipos = take(3 * nb); o.subtree_com = take(3 * nb);
  o.cinert = take(10 * nb); o.cdof = take(6 * nv); o.qM = take(nM); o.qLD = take(nM);
  o.geom_xpos = take(3 * ng); o.geom_xmat = take(9 * ng); o.ncon = take(1); o.con_dist = take(C);
  o.con_pos = take(3 * C); o.con_frame = take(9 * C); o.con_geom = take(2 * C); o.nefc = take(1);
  o.efc_type = take(E); o.efc_id = take(E); o.efc_pos = take(E); o.efc_margin = take(E); o.efc_R = take(E);
  o.efc_aref = take(E); o.Bmat = take(E * nv); o.cvel = take(6 * nb); o.cdof_dot = take(6 * nv);
  o.qfrc_smooth = take(nv); o.qacc_smooth = take(nv); o.efc_force = take(E); o.qacc = take(nv);
  o.qfrc_constraint = take(nv); o.niter = take(1); o.total = p;
  return o;
}
// the wide (nv > 64) physics kernels (mgx_construction.hip)
int wide_step(const mgx_model* m, const mgx_state* s, const mgx_frames& fr, int n_env, int nsub, const uint8_t* mask,
              hipStream_t st);
int wide_debug(const mgx_model* m, const mgx_state* s, int n_env, void* dbg, const DbgOff& o, hipStream_t st);
int wide_kernels_configure(const mgx_model* m);
// records the message returned by mgx_last_error() and returns `code`
int host_fail(int code, const std::string& msg);
int host_check_state(const mgx_state* s);
// dynamic-LDS attributes of the generic step kernels (mgx_step.hip)
int step_kernels_configure(const mgx_model* m);
// the staged solver S2 (mgx_pgs.hip)
template <typename T>
void launch_pgs(const Pipe& P, int slots, int lds, hipStream_t st, int maxit, T tol, T scale, int big, const Hooks& h);
// bytes: the solver kernels' dynamic-LDS limit; wide: the LDS-B instantiations' (the wide launch)
int pgs_configure_lds(int precision, int bytes, int wide);
// S1 / S3 and the one-wave settle (mgx_pgs.hip, the staged TU)
template <typename T>
void launch_soccer_rows(const DevModel<T>& Ms, const SoccerIds<T>& ids, const mgx_state& s, const mgx_soccer_env& ev,
                        const float* action, int n_env, const uint8_t* mask, const Pipe& P, int banks, int slots, int lds,
                        hipStream_t st);
template <typename T>
void launch_soccer_finish(const DevModel<T>& Mf, const SoccerIds<T>& ids, const mgx_state& s, const mgx_soccer_env& ev,
                          const float* action, float* obs, double* reward, uint8_t* terminated, uint8_t* truncated,
                          float* final_obs, int autoreset, uint64_t seed, int env_offset, int n_env, const uint8_t* mask,
                          const Pipe& P, int banks, int lds, hipStream_t st);
template <typename T>
void launch_soccer_settle(const DevModel<T>& Ms, const DevModel<T>& Mf, const SoccerIds<T>& ids, const mgx_state& s,
                          const mgx_soccer_env& ev, const T* draws, float* obs, uint64_t seed, int env_offset, int n_env,
                          const uint8_t* mask, const Pipe& P, int mode, int grid, int lds, hipStream_t st, int maxit, T tol,
                          T scale);
int staged_kernels_configure(int precision, int ls, int lf, int settle);
// staged-step workspace layout (mgx_api.hip) and the LDS of one solver wave holding `rows` rows
// per slot with `lps` lanes per slot and `tw` table words per block
size_t make_staged_pipe(const mgx_model* m, void* ws, int n_env, int banks, Pipe* P, bool rk, int nobs);
// sqg: row scalars in the pipe, only the forces in LDS (the RK4 pipeline; soccer at full capacity)
// twl: block-table words per block in LDS (mgx_twl: 8 for the 8-dof group layout, 4 dof-granular)
int staged_pgs_lds_bytes(const mgx_model* m, int rows, int lps, int sqg, int twl);
// the staged RK4 bipedal step (mgx_rk_staged.hip)
int bipedal_staged_configure(const mgx_model* m);
int bipedal_step_staged(const mgx_model* m, const mgx_state* s, const mgx_bipedal_env* e, const float* action, float* obs,
                        double* reward, uint8_t* terminated, uint8_t* truncated, float* final_obs, int autoreset,
                        uint64_t seed, int env_offset, int n_env, const uint8_t* mask, hipStream_t st);
int bipedal_reset_staged(const mgx_model* m, const mgx_state* s, const mgx_bipedal_env* e, const void* draws,
                         float* obs, uint64_t seed, int env_offset, int n_env, const uint8_t* mask, hipStream_t st);
int64_t bipedal_workspace_bytes(const mgx_model* m, int n_env, int banks);
int bipedal_workspace_init(const mgx_model* m, void* workspace, uint64_t bytes, int n_env, int banks, hipStream_t st);
// the staged quadruped_parkour step (mgx_pk_staged.hip)
bool parkour_staged_ok(const mgx_model* m);
int parkour_staged_configure(const mgx_model* m);
int parkour_step_staged(const mgx_model* m, const mgx_state* s, const mgx_parkour_env* e, const float* action, float* obs,
                        double* reward, uint8_t* terminated, uint8_t* truncated, float* final_obs, int autoreset,
                        uint64_t seed, int env_offset, int n_env, const uint8_t* mask, hipStream_t st);
int parkour_reset_staged(const mgx_model* m, const mgx_state* s, const mgx_parkour_env* e, const void* draws,
                         float* obs, uint64_t seed, int env_offset, int n_env, const uint8_t* mask, hipStream_t st);
int64_t parkour_workspace_bytes(const mgx_model* m, int n_env, int banks);
int parkour_workspace_init(const mgx_model* m, void* workspace, uint64_t bytes, int n_env, int banks, hipStream_t st);
int pgs_lanes();
}  // namespace mgx

#define MGX_WIDE_MSG "nv > 64: this model runs on the wide (two dofs per lane) kernels only"

#define MGX_HIPCHK(x)                                                                                   \
  do {                                                                                                  \
    hipError_t _e = (x);                                                                                \
    if (_e != hipSuccess) return mgx::host_fail(MGX_E_HIP, std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)

template <typename KernelT>
int mgx_set_lds(KernelT k, int bytes) {
  if (bytes > 64 * 1024) MGX_HIPCHK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  return MGX_OK;
}
