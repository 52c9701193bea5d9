"""Diagnostic: staged vs monolithic bipedal fp64 RK4 step from identical states (the monolithic
batch re-synced to the staged one every step), plus the monolithic step's own sensitivity: a third
(monolithic) batch with qpos perturbed by 1e-14. A stage-3 difference as large as the monolithic
step's own response to a 1e-14 perturbation is the solver's conditioning, not an error."""
import numpy as np
import torch

from mujoco_gymnasium_environments_amd.envs.bipedal import BipedalVectorEnv
from mujoco_gymnasium_environments_amd.seeding import np_random

n = 6
a = BipedalVectorEnv(n, precision="f64", autoreset=False, staged=True)
b = BipedalVectorEnv(n, precision="f64", autoreset=False, staged=False)
c = BipedalVectorEnv(n, precision="f64", autoreset=False, staged=False)
draws = np.stack([a.tables.reset_draws(np_random(200 + i)[0]) for i in range(n)])
for e in (a, b, c):
    e.reset(draws=draws)
torch.cuda.synchronize()
rng = np.random.default_rng(11)
g = torch.Generator(device="cuda:0")
g.manual_seed(0)


def d(x, y):
    return (x - y).abs().reshape(x.shape[0], -1).max(1).values.cpu().numpy()


for k in range(8):
    act = torch.from_numpy((rng.uniform(-1, 1, (n, 26)) * 10.0).astype(np.float32)).cuda()
    for e in (b, c):
        for kk in ("qpos", "qvel", "qacc_warmstart", "ctrl", "qfrc_applied", "xfrc_applied", "time"):
            getattr(e.batch, kk).copy_(getattr(a.batch, kk))
    c.batch.qpos.add_((torch.rand(c.batch.qpos.shape, device="cuda:0", generator=g, dtype=torch.float64) - 0.5) * 2e-14)
    for e in (a, b, c):
        e.step(act)
    torch.cuda.synchronize()
    np.set_printoptions(precision=2)
    print(f"step {k}: staged-mono qvel {d(a.batch.qvel, b.batch.qvel)} ws {d(a.batch.qacc_warmstart, b.batch.qacc_warmstart)}")
    print(f"        mono(1e-14)-mono qvel {d(c.batch.qvel, b.batch.qvel)} ws {d(c.batch.qacc_warmstart, b.batch.qacc_warmstart)}")
