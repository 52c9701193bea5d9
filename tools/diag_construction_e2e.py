"""Diagnostic (GPU box): device vs oracle per (env, step) state error on the construction end to
end trajectory of tests/test_gpu_construction.py, beside the oracle's local one-step sensitivity
(a copy of the oracle state with qpos perturbed by 1e-13, stepped once)."""
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from mujoco_gymnasium_environments_amd import cabi  # noqa: E402
from mujoco_gymnasium_environments_amd.envs.construction import (ConstructionTables, ConstructionVectorEnv,  # noqa: E402
                                                                  construction_model)
from mujoco_gymnasium_environments_amd.seeding import np_random  # noqa: E402
from oracle.construction_logic import ConstructionLogic  # noqa: E402
from oracle.mjref import RefSim  # noqa: E402
from tests.helpers import STATE_FIELDS, oracle_at  # noqa: E402

m = construction_model()
pk = cabi.pack_model(m)
n = 6
env = ConstructionVectorEnv(n, precision="f64", autoreset=False)
tb = ConstructionTables(m)
L = ConstructionLogic(tb.humanoid, m.nu)
draws = np.stack([tb.reset_draws(np_random(70 + i)[0]) for i in range(n)])
env.reset(draws=draws)
sims = []
for i in range(n):
    L.reset(np_random(70 + i)[0])
    s = RefSim(pk)
    s.reset()
    sims.append(s)
rng = np.random.default_rng(9)
for t in range(30):
    act = rng.uniform(-200, 200, (n, m.nu)).astype(np.float32)
    env.step(torch.from_numpy(act).cuda())
    torch.cuda.synchronize()
    qg, vg = env.batch.qpos.cpu().numpy(), env.batch.qvel.cpu().numpy()
    row = []
    for i in range(n):
        a = L.pre(act[i])
        sims[i].ctrl[:] = a
        st = {f: sims[i].field(f).copy() for f in STATE_FIELDS}
        sims[i].step()
        tw = oracle_at(pk, {**st, "qpos": st["qpos"] + np.random.default_rng(t).normal(size=st["qpos"].shape) * 1e-13})
        tw.step()
        e = max(np.max(np.abs(qg[i] - sims[i].qpos) / np.maximum(1, np.abs(sims[i].qpos))),
                np.max(np.abs(vg[i] - sims[i].qvel) / np.maximum(1, np.abs(sims[i].qvel))))
        sp = np.max(np.abs(tw.qvel - sims[i].qvel) / np.maximum(1, np.abs(sims[i].qvel)))
        row.append(f"{e:.0e}/{sp:.0e}")
    print("step", t, " ".join(row), flush=True)
