// mgx_internal.h — host-side definitions shared by the translation units of libmgx.so
// (mgx_api.hip: model, physics and soccer; mgx_step.hip: generic step; mgx_parkour.hip:
// quadruped_parkour; mgx_bipedal.hip: bipedal_rescue; mgx_dancing.hip: humanoid_dancing).
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/mgx.h"
#include "mgx_bipedal.h"
#include "mgx_dancing.h"
#include "mgx_martial.h"
#include "mgx_parkour.h"
#include "mgx_staged.h"

struct mgx_model {
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
  int npair;
  bool staged_ok = false;  // the staged soccer pipeline supports this model's capacities
};

namespace mgx {
// records the message returned by mgx_last_error() and returns `code`
int host_fail(int code, const std::string& msg);
int host_check_state(const mgx_state* s);
// dynamic-LDS attributes of the generic step kernels (mgx_step.hip)
int step_kernels_configure(const mgx_model* m);
// the staged solver S2 (mgx_pgs.hip)
template <typename T>
void launch_pgs(const Pipe& P, int slots, int lds, hipStream_t st, int maxit, T tol, T scale);
int pgs_configure_lds(int precision, int bytes);
}  // namespace mgx

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
