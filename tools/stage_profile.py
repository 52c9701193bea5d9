"""Per-stage cycle breakdown of the soccer step kernel (diagnostic build, -DMGX_PROFILE).

Builds libmgx_prof.so next to libmgx.so, loads it instead, runs K steps of the soccer
VectorEnv and prints the mean cycles per env step for each stage. Shares only: the
instrumented build's absolute times are not the shipped kernel's (stamps serialise).
"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mujoco_gymnasium_environments_amd import native  # noqa: E402

PROF_LIB = os.path.join(native.PKG, "libmgx_prof.so")
STAGES = ["kinematics", "com_crb", "factorM", "velocity", "qacc_smooth", "collision", "make_constraint",
          "transform_rows", "pgs", "euler"]


def build():
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-DMGX_PROFILE",
           "-o", PROF_LIB, os.path.join(native.CSRC, "mgx_api.hip")]
    subprocess.run(cmd, check=True)


def main():
    if "--build" in sys.argv:
        build()
        return
    import torch
    native.LIB_PATH = PROF_LIB
    L = native.lib()
    L.mgx_prof_set_buffer.argtypes = [C.c_void_p]
    from mujoco_gymnasium_environments_amd.envs.soccer import SoccerVectorEnv
    n = int(os.environ.get("N", "4096"))
    steps = int(os.environ.get("K", "20"))
    env = SoccerVectorEnv(n, seed=3)
    env.reset()
    buf = torch.zeros(n * 32, dtype=torch.int64, device="cuda:0")
    g = torch.Generator(device="cuda:0"); g.manual_seed(0)
    acts = [(torch.rand(n, env.model.nu, device="cuda:0", generator=g) * 300 - 150) for _ in range(4)]
    for k in range(5):
        env.step(acts[k % 4])
    torch.cuda.synchronize()
    assert L.mgx_prof_set_buffer(C.c_void_p(buf.data_ptr())) == 0
    for k in range(steps):
        env.step(acts[k % 4])
    torch.cuda.synchronize()
    v = buf.view(n, 32).double().cpu().numpy() / steps
    tot = v[:, :10].sum(1).mean()
    print(f"envs={n} steps={steps} mean cycles/env-step (s_memtime units) total={tot:.0f}")
    for i, s in enumerate(STAGES):
        print(f"  {s:16s} {v[:, i].mean():12.0f}  {100 * v[:, i].mean() / tot:5.1f}%   p99 {sorted(v[:, i])[int(0.99 * n)]:.0f}")
    print(f"  lds bytes per env {env.native.info.lds_bytes_per_env}")
    raw = buf.view(n, 32).double().cpu().numpy()
    calls = raw[:, 23].sum()
    print(f"  per forward: nefc mean {raw[:, 20].sum() / calls:.1f}  PGS iterations mean {raw[:, 21].sum() / calls:.1f}"
          f"  ncon mean {raw[:, 22].sum() / calls:.1f}  forwards per env-step {calls / (n * steps):.2f}")
    import numpy as np
    nefc_env = raw[:, 20] / np.maximum(raw[:, 23], 1)
    print(f"  per-env mean nefc p50 {np.percentile(nefc_env, 50):.0f} p90 {np.percentile(nefc_env, 90):.0f} max {nefc_env.max():.0f}")


if __name__ == "__main__":
    main()
