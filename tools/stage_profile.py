"""Per-stage cycle breakdown of the step kernels (diagnostic build, -DMGX_PROFILE).

    python tools/stage_profile.py --build            # CPU: all translation units -> libmgx_prof.so
    TASK=soccer|assembly|bipedal|martial|construction N=... K=... python tools/stage_profile.py   # GPU

Loads libmgx_prof.so instead of libmgx.so, runs K steps of the task's VectorEnv and prints the
mean cycles per env step for each stage of the forward pass (each translation unit has its own
stamp buffer, set through its MGX_PROF_SETTER export). Shares only: the instrumented build's
absolute times are not the shipped kernel's (stamps serialise).
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
# staged row builder (k_soccer_rows): blocks 0..N-1 live envs, N.. bank slots
STAGES_ROWS = ["kinematics", "com_crb", "factorM", "velocity", "qacc_smooth", "collision", "rows_plan",
               "rows (all blocks)", "  block: J + metadata + dots", "  block: transform", "  block: B.B, A_ij sums",
               "  block: scalars + stores"]
SUBSTAGES = 4  # the block sub-stamps are inside 'rows (all blocks)'; excluded from the total


def build():
    """Every translation unit of libmgx.so with -DMGX_PROFILE, objects in _build_prof/."""
    bdir = os.path.join(native.PKG, "_build_prof")
    os.makedirs(bdir, exist_ok=True)
    base = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-DMGX_PROFILE"]
    procs, objs = [], []
    for src in native.SOURCES:
        obj = os.path.join(bdir, src.replace(".hip", ".o"))
        objs.append(obj)
        procs.append(subprocess.Popen(base + native.SOURCE_FLAGS.get(src, []) + ["-c", "-o", obj,
                                                                                 os.path.join(native.CSRC, src)]))
    for p in procs:
        if p.wait() != 0:
            raise SystemExit("profile build failed")
    subprocess.run(base + ["-shared", "-o", PROF_LIB] + objs, check=True)


TASK_TU = {"assembly": "mgx_prof_set_buffer_assembly", "bipedal": "mgx_prof_set_buffer_bipedal",
           "bipedal_staged": "mgx_prof_set_buffer_rk_staged",
           "martial": "mgx_prof_set_buffer_martial", "construction": "mgx_prof_set_buffer_construction"}


def make_task(task, n):
    import torch
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0)
    if task == "assembly":
        from mujoco_gymnasium_environments_amd.envs.assembly import AssemblyVectorEnv
        env = AssemblyVectorEnv(n)
        lo = torch.tensor([-2.0] * 7 + [0, 0], device="cuda:0")
        span = torch.tensor([4.0] * 7 + [100, 50], device="cuda:0")
        acts = [torch.rand(n, 9, device="cuda:0", generator=g) * span + lo for _ in range(4)]
    elif task == "construction":
        from mujoco_gymnasium_environments_amd.envs.construction import ConstructionVectorEnv
        env = ConstructionVectorEnv(n, seed=3, precision=os.environ.get("PREC", "f64"))
        acts = [(torch.rand(n, 33, device="cuda:0", generator=g) * 2 - 1) * 200 for _ in range(4)]
    elif task.startswith("bipedal"):
        from mujoco_gymnasium_environments_amd.envs.bipedal import BipedalVectorEnv
        env = BipedalVectorEnv(n, seed=3, staged=task == "bipedal_staged")
        acts = [(torch.rand(n, 26, device="cuda:0", generator=g) * 2 - 1) * 100 for _ in range(4)]
    else:
        from mujoco_gymnasium_environments_amd.envs.martial import MartialArtsVectorEnv
        env = MartialArtsVectorEnv(n, seed=3)
        acts = [torch.rand(n, 28, device="cuda:0", generator=g) * 2 - 1 for _ in range(4)]
    return env, acts


def main_task(task):
    import numpy as np
    import torch
    native.LIB_PATH = PROF_LIB
    L = native.lib()
    setter = getattr(L, TASK_TU[task])
    setter.argtypes = [C.c_void_p]
    n = int(os.environ.get("N", "1024"))
    steps = int(os.environ.get("K", "5"))
    env, acts = make_task(task, n)
    env.reset()
    for k in range(2):
        env.step(acts[k % 4])
    torch.cuda.synchronize()
    # staged RK4 (bipedal_staged): the row builder's blocks are the slots (live + reset banks) and
    # the solver's blocks its waves, so the stamp buffer holds a row per slot, 4 x the envs at most
    staged = task == "bipedal_staged"
    nslot = 4 * n if staged else n
    buf = torch.zeros(nslot * 32, dtype=torch.int64, device="cuda:0")
    assert setter(C.c_void_p(buf.data_ptr())) == 0
    for k in range(steps):
        env.step(acts[k % 4])
    torch.cuda.synchronize()
    raw = buf.view(nslot, 32).double().cpu().numpy()
    if staged:
        return report_rows(raw, n, steps, env, "staged RK4 row builder (per RK4 stage)")
    v = raw / steps
    tot = v[:, :len(STAGES)].sum(1).mean()
    calls = raw[:, 23].sum()
    print(f"{task}: envs={n} steps={steps} mean cycles per env-step (s_memtime units), total {tot:.0f}; "
          f"forwards per env-step {calls / (n * steps):.2f}")
    for i, st in enumerate(STAGES):
        print(f"  {st:16s} {v[:, i].mean():14.0f}  {100 * v[:, i].mean() / tot:5.1f}%   p99 {np.percentile(v[:, i], 99):.0f}")
    print(f"  per forward: nefc mean {raw[:, 20].sum() / calls:.1f}  solver iterations mean {raw[:, 21].sum() / calls:.2f}"
          f"  ncon mean {raw[:, 22].sum() / calls:.1f}")
    sub = ["setup", "Hessian", "Cholesky", "triangular solves", "J p", "line search", "update+gradient+stop"]
    if v[:, 10:17].sum() > 0:
        print("  Newton sub-stages (inside the solver slot):")
        for i, st in enumerate(sub):
            print(f"    {st:22s} {v[:, 10 + i].mean():14.0f}")
    print(f"  lds bytes per env {env.native.info.lds_bytes_per_env}, scratch bytes per env "
          f"{env.native.info.scratch_bytes_per_env}")


def report_rows(raw, n, steps, env, title):
    """The staged row builders' stamps (stage_rows: one row per slot, live envs first, then the
    reset banks) and the solver's sweep counters (slots 26..30 of its wave rows)."""
    import numpy as np
    calls = np.maximum(raw[:, 23], 1)
    act = raw[:, 23] > 0
    v = raw[act] / calls[act, None]
    names = STAGES_ROWS
    print(f"{title}: envs={n} steps={steps} slots with work {act.sum()} (live {act[:n].sum()}, bank "
          f"{act[n:].sum()}); mean cycles per slot-stage (s_memtime units)")
    tot = v[:, :len(names) - SUBSTAGES].sum(1).mean()
    print(f"  total {tot:.0f}")
    for i, s in enumerate(names):
        print(f"  {s:40s} {v[:, i].mean():12.0f}  {100 * v[:, i].mean() / tot:5.1f}%   p99 {np.percentile(v[:, i], 99):.0f}")
    k2 = raw[:, 28] > 0
    if k2.any():
        cyc, blks = raw[k2, 26].sum(), raw[k2, 27].sum()
        rt = raw[k2, 29].sum()
        print(f"  solver waves: {int(raw[k2, 28].sum())} wave-launches; sweep cycles per block "
              f"{cyc / max(blks, 1):.0f}; blocks swept by the heaviest wave {raw[k2, 30].max():.0f} "
              f"(mean {blks / raw[k2, 28].sum():.0f}); shader clock {cyc / max(rt, 1) * 0.1:.2f} GHz")
    print(f"  per slot-stage: nefc mean {(raw[:, 20].sum() / max(raw[:, 23].sum(), 1)):.1f}  ncon mean "
          f"{(raw[:, 22].sum() / max(raw[:, 23].sum(), 1)):.1f}")


def main():
    import numpy as np
    if "--build" in sys.argv:
        build()
        return
    task = os.environ.get("TASK", "soccer")
    if task != "soccer":
        return main_task(task)
    import torch
    native.LIB_PATH = PROF_LIB
    L = native.lib()
    L.mgx_prof_set_buffer.argtypes = [C.c_void_p]
    from mujoco_gymnasium_environments_amd.envs.soccer import SoccerVectorEnv
    n = int(os.environ.get("N", "4096"))
    steps = int(os.environ.get("K", "20"))
    staged = os.environ.get("MODE", "staged") == "staged"
    env = SoccerVectorEnv(n, seed=3, staged=staged, precision=os.environ.get("PREC", "f64"))
    env.reset()
    nslot = n * 5 if staged else n
    buf = torch.zeros(nslot * 32, dtype=torch.int64, device="cuda:0")
    g = torch.Generator(device="cuda:0"); g.manual_seed(0)
    acts = [(torch.rand(n, env.model.nu, device="cuda:0", generator=g) * 300 - 150) for _ in range(4)]
    for k in range(5):
        env.step(acts[k % 4])
    torch.cuda.synchronize()
    assert L.mgx_prof_set_buffer(C.c_void_p(buf.data_ptr())) == 0
    if staged:  # the staged kernels live in their own translation unit (mgx_pgs.hip)
        L.mgx_prof_set_buffer_pgs.argtypes = [C.c_void_p]
        assert L.mgx_prof_set_buffer_pgs(C.c_void_p(buf.data_ptr())) == 0
    for k in range(steps):
        env.step(acts[k % 4])
    torch.cuda.synchronize()
    raw = buf.view(nslot, 32).double().cpu().numpy()
    if staged:
        calls = np.maximum(raw[:, 23], 1)
        act = raw[:, 23] > 0
        v = raw[act] / calls[act, None]
        names = STAGES_ROWS
        print(f"staged row builder: envs={n} steps={steps} slots with work {act.sum()} "
              f"(live {act[:n].sum()}, bank {act[n:].sum()}); mean cycles per slot-step (s_memtime units)")
    else:
        v = raw / steps
        names = STAGES
        print(f"monolithic: envs={n} steps={steps} mean cycles/env-step (s_memtime units)")
    tot = v[:, :len(names) - (SUBSTAGES if staged else 0)].sum(1).mean()
    print(f"  total {tot:.0f}")
    for i, s in enumerate(names):
        print(f"  {s:40s} {v[:, i].mean():12.0f}  {100 * v[:, i].mean() / tot:5.1f}%   p99 {np.percentile(v[:, i], 99):.0f}")
    print(f"  lds bytes per env: monolithic {env.native.info.lds_bytes_per_env} rows {env.native.info.lds_bytes_rows} "
          f"finish {env.native.info.lds_bytes_finish}")
    if staged:
        k2 = raw[:, 28] > 0
        if k2.any():
            cyc, blks = raw[k2, 26].sum(), raw[k2, 27].sum()
            print(f"  solver waves (block index = wave): {int(raw[k2, 28].sum())} wave-launches; sweep cycles per "
                  f"block {cyc / max(blks, 1):.0f}; mean sweep cycles per wave-launch {cyc / raw[k2, 28].sum():.0f}")
            rt = raw[k2, 29].sum()
            print(f"  s_memtime ticks per s_memrealtime tick (100 MHz): {cyc / max(rt, 1):.2f} -> shader clock "
                  f"{cyc / max(rt, 1) * 0.1:.2f} GHz; solver sweep time per wave-launch {rt / raw[k2, 28].sum() / 100:.1f} us "
                  f"mean, blocks swept by the heaviest wave {raw[k2, 30].max():.0f} (mean {blks / raw[k2, 28].sum():.0f})")
        print(f"  per slot-step: nefc mean {(raw[:, 20].sum() / raw[:, 23].sum()):.1f}  ncon mean "
              f"{(raw[:, 22].sum() / raw[:, 23].sum()):.1f}  nefc max {raw[:, 24].max():.0f}  "
              f"slot-steps with capacity overflow {raw[:, 25].sum():.0f} of {raw[:, 23].sum():.0f}")
        return
    calls = raw[:, 23].sum()
    print(f"  per forward: nefc mean {raw[:, 20].sum() / calls:.1f}  PGS iterations mean {raw[:, 21].sum() / calls:.1f}"
          f"  ncon mean {raw[:, 22].sum() / calls:.1f}  forwards per env-step {calls / (n * steps):.2f}")
    nefc_env = raw[:, 20] / np.maximum(raw[:, 23], 1)
    print(f"  per-env mean nefc p50 {np.percentile(nefc_env, 50):.0f} p90 {np.percentile(nefc_env, 90):.0f} max {nefc_env.max():.0f}")


if __name__ == "__main__":
    main()
