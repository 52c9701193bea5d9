"""Diagnostic (GPU box): device vs oracle contact lists on the parity-test states, per pair."""
import sys

import numpy as np

sys.path.insert(0, '.')
from tests.helpers import load_states, oracle_at, oracle_states  # noqa: E402
from mujoco_gymnasium_environments_amd import cabi  # noqa: E402
from mujoco_gymnasium_environments_amd.batch import PhysicsBatch  # noqa: E402


def run(name, m, states):
    pk = cabi.pack_model(m)
    b = PhysicsBatch(m, len(states), precision="f64")
    load_states(b, states)
    dbg = b.debug_forward()
    gt = m.arrays["geom_type"]
    for i, st in enumerate(states):
        o = oracle_at(pk, st)
        o.forward()
        nc_o = int(o.ncon[0])
        nc_d = int(dbg["ncon"][i][0])
        cg_o = o.con_geom[:2 * nc_o].reshape(-1, 2)
        cg_d = dbg["con_geom"][i][:2 * nc_d].astype(int).reshape(-1, 2)
        pairs = sorted(set(map(tuple, cg_o)) | set(map(tuple, cg_d)))
        for pr in pairs:
            io = [k for k in range(nc_o) if tuple(cg_o[k]) == pr]
            idd = [k for k in range(nc_d) if tuple(cg_d[k]) == pr]
            po = o.con_pos[:3 * nc_o].reshape(-1, 3)[io]
            pd = dbg["con_pos"][i][:3 * nc_d].reshape(-1, 3)[idd]
            no = o.con_frame[:9 * nc_o].reshape(-1, 9)[io, :3]
            nd = dbg["con_frame"][i][:9 * nc_d].reshape(-1, 9)[idd, :3]
            do = o.con_dist[:nc_o][io]
            dd = dbg["con_dist"][i][:nc_d][idd]
            bad = len(io) != len(idd) or (len(io) and (np.abs(po - pd).max() > 1e-8 or np.abs(no - nd).max() > 1e-8))
            if bad:
                print(f"{name} env {i} pair {pr} types {gt[pr[0]]},{gt[pr[1]]}: oracle {len(io)} device {len(idd)}")
                print("   oracle dist", do, "pos", po.tolist(), "n", no.tolist())
                print("   device dist", dd, "pos", pd.tolist(), "n", nd.tolist())
                print("   sizes", m.arrays["geom_size"][pr[0]], m.arrays["geom_size"][pr[1]])
                print("   geom1 xpos", dbg["geom_xpos"][i][3 * pr[0]:3 * pr[0] + 3].tolist(), "xmat",
                      dbg["geom_xmat"][i][9 * pr[0]:9 * pr[0] + 9].tolist())
                print("   geom2 xpos", dbg["geom_xpos"][i][3 * pr[1]:3 * pr[1] + 3].tolist(), "xmat",
                      dbg["geom_xmat"][i][9 * pr[1]:9 * pr[1] + 9].tolist())


from mujoco_gymnasium_environments_amd.envs.bipedal import bipedal_model  # noqa: E402
from mujoco_gymnasium_environments_amd.envs.dancing import dancing_model  # noqa: E402
from mujoco_gymnasium_environments_amd.envs.construction import construction_model  # noqa: E402
for name, m, kw in [("bipedal", bipedal_model(), dict(seed=7, max_steps=40, action_scale=30.0)),
                    ("dancing", dancing_model(), dict(seed=7, max_steps=40, action_scale=50.0)),
                    ("construction", construction_model(), dict(seed=4, max_steps=40, action_scale=100.0))]:
    run(name, m, oracle_states(cabi.pack_model(m), 8, **kw))
print("done")
