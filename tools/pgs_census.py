"""Census of the staged soccer solver's input at bench conditions (GPU).

After each step of a 4096-env SoccerVectorEnv (U(-150, 150) actions, same-step autoreset,
4 reset banks) read the workspace (mgx_soccer_workspace_layout): the compacted solver list,
each listed slot's row count and the length of its group-compressed B (from its block table:
the end of its last A / dof-group record). Prints quantiles of rows / blocks / B bytes per slot
and of the per-wave sums (MGX_PGS_SPW consecutive list entries) — the numbers that size an
LDS-resident B in k_pgs_groups.

    python tools/pgs_census.py [--precision f64] [--steps 20] [--envs 4096]
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from mujoco_gymnasium_environments_amd.envs.soccer import SoccerVectorEnv
from mujoco_gymnasium_environments_amd.native import lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="f64")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--spw", type=int, default=1)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    env = SoccerVectorEnv(a.envs, device=str(dev), precision=a.precision, seed=1234)
    env.reset(seed=1234)
    lay = (C.c_int64 * 10)()
    assert lib().mgx_soccer_workspace_layout(env.native.handle, a.envs, int(env._env.banks), lay, 10) == 0
    o_ctr, o_ne, o_list, o_blk, o_B, bcap, maxE, capE, S, rb = list(lay)
    g = torch.Generator(device=dev)
    g.manual_seed(1000)
    nu = env.model.nu
    rows, blocks, bbytes, wave_b, wave_rows, wave_nbmax, cnts, wave_need, spilled = [], [], [], [], [], [], [], {}, []
    for _ in range(a.steps):
        act = ((torch.rand(a.envs, nu, device=dev, generator=g) * 2 - 1) * 150.0).contiguous()
        env.step(act)
        torch.cuda.synchronize()
        ws = env.workspace
        # ctr[3] / ctr[4]: the last step's main solver list / global-B list sizes (the finisher
        # keeps them when it clears the lists)
        cnt, gb = (int(x) for x in ws[o_ctr + 12:o_ctr + 20].view(torch.int32).cpu())
        spilled.append(gb)
        lst = ws[o_list:o_list + 4 * cnt].view(torch.int32).cpu().numpy()
        ne = ws[o_ne:o_ne + 4 * S].view(torch.int32).cpu().numpy()
        # block table (mgx_staged.h MGX_TW): [B offset, dof support lo, hi, 0] per 4-row block
        blk = ws[o_blk:o_blk + 4 * S * maxE].view(torch.int32).cpu().numpy().view(np.uint32).reshape(S, maxE)
        cnts.append(cnt)
        per = []
        for s in lst:
            nb = ne[s] // 4
            t = blk[s, :4 * nb].reshape(nb, 4).astype(np.int64)
            ndof = [bin(int(a) | (int(b) << 32)).count("1") for a, b in zip(t[:, 1], t[:, 2])]
            end = int((t[:, 0] + 8 + 4 * np.array(ndof)).max()) if nb else 32
            per.append((ne[s], nb, end * rb))
        per = np.array(per)
        rows += list(per[:, 0]); blocks += list(per[:, 1]); bbytes += list(per[:, 2])
        for w in range(0, len(per), a.spw):
            p = per[w:w + a.spw]
            wave_b.append(p[:, 2].sum()); wave_rows.append(p[:, 0].sum()); wave_nbmax.append(p[:, 1].max())
            # the main launch's arena need (mgx_staged.h pgs_group<BLDS>): per slot the row
            # scalars + table for the wave's block count (ring 2) and the slot's B
            nbA = (p[:, 1].max() + 1) // 2 * 2 + 1
            need = len(p) * nbA * (20 * rb + 16) + int(((p[:, 2] // rb + 3) // 4 * 4).sum()) * rb
            wave_need.setdefault("all", []).append(need)
    q = lambda x: {k: float(np.percentile(x, k)) for k in (10, 50, 90, 99, 100)} | {"mean": float(np.mean(x))}
    print(json.dumps({"precision": a.precision, "envs": a.envs, "steps": a.steps, "slots_listed_mean": float(np.mean(cnts)),
                      "global_B_slots_mean": float(np.mean(spilled)),
                      "rows": q(rows), "blocks": q(blocks), "B_bytes": q(bbytes), "wave_B_bytes": q(wave_b),
                      "wave_rows": q(wave_rows), "wave_max_blocks": q(wave_nbmax), "bcap_bytes": bcap * rb,
                      "capE": capE, "wave_arena_need": q(wave_need["all"]),
                      "waves_fitting": {str(kb): float(np.mean(np.array(wave_need["all"]) <= kb * 1024))
                                        for kb in (16, 20, 24, 32, 40, 48, 64, 80)}}, indent=1))


if __name__ == "__main__":
    main()
