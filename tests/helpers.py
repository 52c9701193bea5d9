"""Shared test helpers: oracle trajectories used as GPU parity inputs."""
import numpy as np

STATE_FIELDS = ("qpos", "qvel", "qacc_warmstart", "ctrl", "qfrc_applied", "xfrc_applied")


def oracle_states(packed, n, seed=0, max_steps=60, action_scale=150.0, init=None):
    """n oracle states reached from qpos0 (with qpos overrides ``init`` {index: value}) under
    random actions (snapshot before a step)."""
    from oracle.mjref import RefSim
    rng = np.random.default_rng(seed)
    m = packed.model
    out = []
    for i in range(n):
        s = RefSim(packed)
        for a, v in (init or {}).items():
            s.qpos[a] = v
        k = int(rng.integers(0, max_steps))
        for _ in range(k):
            s.ctrl[:] = rng.uniform(-action_scale, action_scale, m.nu)
            s.step()
        s.ctrl[:] = rng.uniform(-action_scale, action_scale, m.nu)
        s.qfrc_applied[0] = rng.uniform(-50, 50)
        s.xfrc_applied[6 * 4:6 * 4 + 2] = rng.normal(size=2)
        out.append({f: s.field(f).copy() for f in STATE_FIELDS})
    return out


def load_states(batch, states):
    import torch
    for f in STATE_FIELDS:
        t = getattr(batch, f)
        arr = np.stack([s[f] for s in states]).reshape(t.shape)
        t.copy_(torch.from_numpy(arr).to(t.dtype))


def oracle_at(packed, state):
    from oracle.mjref import RefSim
    s = RefSim(packed)
    for f in STATE_FIELDS:
        s.field(f)[:] = state[f]
    return s
