"""Diagnostic (GPU box): device Newton vs oracle newton_solve, max relative force / qacc error and
iteration counts, on soccer-as-Newton and martial oracle states at tolerance 1e-10 and 1e-8."""
import copy
import sys

import numpy as np

sys.path.insert(0, '.')
from tests.helpers import load_states, oracle_at, oracle_states  # noqa: E402
from mujoco_gymnasium_environments_amd import cabi  # noqa: E402
from mujoco_gymnasium_environments_amd.batch import PhysicsBatch  # noqa: E402
from mujoco_gymnasium_environments_amd.envs.martial import martial_model  # noqa: E402
from mujoco_gymnasium_environments_amd.envs.soccer import soccer_model  # noqa: E402

rel = lambda a, b: float(np.max(np.abs(a - b)) / max(1.0, np.max(np.abs(b))))  # noqa: E731
for name, base in (("soccer", soccer_model()), ("martial", martial_model())):
    for tol in (1e-10, 1e-8):
        m = copy.deepcopy(base)
        m.solver = 2
        m.tolerance = tol
        pk = cabi.pack_model(m)
        states = oracle_states(pk, 16, seed=11, action_scale=150.0 if name == "soccer" else 1.0)
        b = PhysicsBatch(m, len(states), precision="f64")
        load_states(b, states)
        dbg = b.debug_forward()
        ef, eq, its = [], [], []
        for i, st in enumerate(states):
            o = oracle_at(pk, st)
            o.forward()
            ne = int(o.nefc[0])
            ef.append(rel(dbg["efc_force"][i][:ne], o.efc_force[:ne]) if ne else 0.0)
            eq.append(rel(dbg["qacc"][i], o.qacc))
            its.append((int(dbg["niter"][i][0]), int(o.solver_niter[0])))
        print(name, tol, "force max", f"{max(ef):.1e}", "qacc max", f"{max(eq):.1e}", "iters", its, flush=True)
