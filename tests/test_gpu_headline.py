"""GPU: properties of the headline workload at its full size (BASELINE configs[2]: humanoid_soccer,
4096 envs, fp64, staged step, U(-150, 150) actions — exactly what bench.py times).

At this size the oracle cannot follow every env, so the test asserts what holds at
any size: every state finite, no row beyond the capacity (MuJoCo's arena keeps every row: the
overflow counter stays 0), slots with more rows than the round-1 capacity of 192 kept and solved
(the main solver launch's heavy-slot path, Pipe.hmain, takes those over its LDS rows), and the
reset-bank count invisible — 3 banks (the bench default) and 1 bank give bit-identical
observations, rewards, flags and episode counts, whichever resets came from a bank and which
from the fallback settle.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _slot_rows(env):
    """Per-slot row counts of the last step (the workspace's o_ne array) and the main launch's LDS
    rows (mgx_soccer_workspace_layout)."""
    import ctypes as C

    from mujoco_gymnasium_environments_amd.native import check, lib
    out = (C.c_int64 * 11)()
    banks = env._env.banks
    check(lib().mgx_soccer_workspace_layout(env.native.handle, env.num_envs, banks, out, 11), "layout")
    o_ne, cap_e, slots = int(out[1]), int(out[7]), int(out[8])
    ne = env.workspace[o_ne:o_ne + 4 * slots].view(torch.int32)
    return ne, cap_e


def test_headline_size_properties():
    from mujoco_gymnasium_environments_amd.envs.soccer import SoccerVectorEnv
    n, steps = 4096, 60
    a = SoccerVectorEnv(n, precision="f64", seed=1234, banks=3)
    b = SoccerVectorEnv(n, precision="f64", seed=1234, banks=1)
    a.reset()
    b.reset()
    g = torch.Generator(device="cuda:0")
    g.manual_seed(1000)
    over192 = over_cap = 0
    max_rows = 0
    for t in range(steps):
        act = (torch.rand(n, a.model.nu, device="cuda:0", generator=g) * 300.0 - 150.0).contiguous()
        ra = a.step(act)
        rb = b.step(act)
        ne, cap_e = _slot_rows(a)
        ne = ne[:n]  # live slots (bank slots follow)
        over192 += int((ne > 192).sum())
        over_cap += int((ne > cap_e).sum())
        max_rows = max(max_rows, int(ne.max()))
        for x, y, name in zip(ra[:4], rb[:4], ("obs", "reward", "terminated", "truncated")):
            assert torch.equal(x, y), (t, name)
    torch.cuda.synchronize()
    for e in (a, b):
        assert torch.isfinite(e.batch.qpos).all() and torch.isfinite(e.batch.qvel).all()
        assert torch.isfinite(e.obs).all()
        assert int(e.batch.overflow.sum()) == 0
    assert torch.equal(a.episode, b.episode) and torch.equal(a.batch.qpos, b.batch.qpos)
    eps = int(a.episode.sum()) - n
    print(f"\nheadline 4096 x {steps}: episodes ended {eps}, live slots over 192 rows {over192}, over the main "
          f"launch's {cap_e} LDS rows {over_cap}, max rows {max_rows}, bad-state resets "
          f"{int(a.batch.warning.sum())}")
    assert eps > 0
    assert over192 >= 1, "no slot above the round-1 capacity: the full-capacity path was not exercised"
