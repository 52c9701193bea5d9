"""Episode-length / termination-reason histogram of the bench workload (diagnostic)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mujoco_gymnasium_environments_amd.envs.soccer import SoccerVectorEnv  # noqa: E402


def main():
    n = int(os.environ.get("N", "4096"))
    steps = int(os.environ.get("K", "300"))
    env = SoccerVectorEnv(n, seed=1234)
    env.reset()
    g = torch.Generator(device="cuda:0"); g.manual_seed(1000)
    pool = [(torch.rand(n, env.model.nu, device="cuda:0", generator=g) * 300 - 150) for _ in range(16)]
    length = torch.zeros(n, dtype=torch.int64, device="cuda:0")
    lens = []
    for k in range(steps):
        obs, rew, term, trunc, info = env.step(pool[k % 16])
        length += 1
        done = (term | trunc).bool()
        if k > 20:
            lens.append(length[done].cpu().numpy())
        length[done] = 0
    lens = np.concatenate(lens) if lens else np.zeros(0)
    h = np.bincount(lens, minlength=40)
    print(f"episodes {len(lens)} mean len {lens.mean():.2f} p5 {np.percentile(lens, 5)} p50 {np.percentile(lens, 50)}")
    print("len<=10:", (lens <= 10).mean(), "len<=11:", (lens <= 11).mean(), "len<=15:", (lens <= 15).mean())
    print("hist[0:40]", h[:40].tolist())


if __name__ == "__main__":
    main()
