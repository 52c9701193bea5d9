import numpy as np, torch, sys
sys.path.insert(0, '.')
from mujoco_gymnasium_environments_amd.envs.soccer import SoccerVectorEnv
nu = 33
def run(n, off, steps=3, seed=11, prec="f32"):
    e = SoccerVectorEnv(n, seed=seed, env_offset=off, precision=prec)
    e.reset()
    rng = np.random.default_rng(0)
    outs = []
    for t in range(steps):
        a = torch.from_numpy(rng.uniform(-150, 150, (4, nu)).astype(np.float32)).cuda()
        o, r, te, tr, _ = e.step(a[off:off + n].contiguous())
        torch.cuda.synchronize()
        outs.append((o.clone(), e.batch.qpos.clone(), e.batch.qvel.clone()))
    return e, outs
e1, A = run(4, 0)
e2, B = run(4, 0)
e3, C = run(2, 2)
for t in range(3):
    print(t, "4vs4 obs eq", torch.equal(A[t][0], B[t][0]), "qpos", torch.equal(A[t][1], B[t][1]),
          "| 4vs2 obs eq", torch.equal(A[t][0][2:], C[t][0]), "maxdiff", (A[t][1][2:] - C[t][1]).abs().max().item(),
          (A[t][2][2:] - C[t][2]).abs().max().item())
