"""Diagnostic (GPU box): fp32 vs oracle contact lists on the dancing parity states."""
import sys

import numpy as np

sys.path.insert(0, '.')
from tests.helpers import load_states, oracle_at, oracle_states  # noqa: E402
from mujoco_gymnasium_environments_amd import cabi  # noqa: E402
from mujoco_gymnasium_environments_amd.batch import PhysicsBatch  # noqa: E402
from mujoco_gymnasium_environments_amd.envs.dancing import dancing_model  # noqa: E402

m = dancing_model()
pk = cabi.pack_model(m)
states = oracle_states(pk, 8, seed=7, max_steps=40, action_scale=50.0)
for prec in ("f32", "f64"):
    b = PhysicsBatch(m, len(states), precision=prec)
    load_states(b, states)
    dbg = b.debug_forward()
    for i, st in enumerate(states):
        o = oracle_at(pk, st)
        o.forward()
        nc, gnc = int(o.ncon[0]), int(dbg["ncon"][i][0])
        if nc == gnc:
            continue
        print(prec, "env", i, "ncon", gnc, nc, "margin geoms", )
        print("  dev", [(tuple(dbg["con_geom"][i][2 * k:2 * k + 2].astype(int)), float(dbg["con_dist"][i][k]),
                         tuple(np.round(dbg["con_pos"][i][3 * k:3 * k + 3], 4))) for k in range(gnc)])
        print("  orc", [(tuple(o.con_geom[2 * k:2 * k + 2]), float(o.con_dist[k]),
                         tuple(np.round(o.con_pos[3 * k:3 * k + 3], 4))) for k in range(nc)])
        print("  geom types", {int(g): int(m.geom_type[g]) for g in set(o.con_geom[:2 * nc].tolist())},
              "margins", {int(g): float(m.geom_margin[g]) for g in set(o.con_geom[:2 * nc].tolist())})
