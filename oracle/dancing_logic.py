"""numpy restatement of the humanoid_dancing env logic (TEST INFRASTRUCTURE ONLY).

Follows humanoid_dancing_env/dancing_env.py line by line: step :833-894 (clip :837, ctrl
:840, _update_rhythm :924-937 and _update_visual_effects :939-955 BEFORE mj_step, counter
:849), observation :1028-1120 (joint i's range normalises qpos[7 + i] -- the model has no root
joint, so indices are shifted; slots past nq / nv are 0), reward :1122-1207 (np.float64 once the
smoothness term is added; the energy term is float32), termination :1209-1235 (the
fall_start_step attribute is created lazily, deleted when upright and survives reset),
_update_episode_stats :1004-1026, _update_crowd_excitement :975-1002,
_check_move_transition :957-973, reset :763-831 with _generate_dance_sequence :896-905
(Generator.choice over 10 names == integers(0, 10)) and _set_initial_pose :907-922 (writes
qpos[0:7] of the first seven hinges, quirk). The spotlight position and disco rotation are
never reset.
Pinned against golden vectors produced by the reference's own step() and reset()
(tests/golden/dancing_*.npz, tests/test_oracle_dancing.py).
"""
from __future__ import annotations

import numpy as np

MOVES = ['basic_step', 'spin', 'jump', 'moonwalk', 'robot_wave', 'freeze', 'hip_hop_bounce', 'breakdance_toprock',
         'salsa_basic', 'ballet_pirouette']
DIFFICULTY = [1, 2, 2, 3, 2, 1, 2, 3, 2, 4]     # dancing_env.py:57-68
DT = 0.01667
BEAT = 60.0 / 120
MAX_EPISODE_STEPS = 3600
OBS_DIM = 94
SEQ_LEN = 20


def _policy(action):
    """The action as the reference's np.clip against float32 bounds types it: float32 stays float32,
    float64 (and anything numpy promotes with float32 to float64) stays float64."""
    a = np.asarray(action)
    return a.astype(np.result_type(a.dtype, np.float32), copy=False)


class DancingTables:
    def __init__(self, m):
        self.model = m
        self.torso = m.name2id("body", "torso")
        self.right_foot = m.name2id("geom", "right_foot")
        self.left_foot = m.name2id("geom", "left_foot")
        self.floor = m.name2id("geom", "dance_floor")
        self.stage = m.name2id("geom", "stage")
        self.nu = m.nu

    @staticmethod
    def reset_draws(rng: np.random.Generator) -> np.ndarray:
        """The 40 draws of one reset in reference order: (move index, duration) x 20."""
        d = []
        for _ in range(SEQ_LEN):
            d += [float(rng.integers(0, 10)), rng.uniform(1.0, 3.0)]
        return np.array(d)


class DancingLogic:
    """State dict keys: the reference attributes (see tests/golden/make_fixtures.py
    _dance_state; hist = the last <= 3 entries of move_history as move indices) plus qpos qvel ctrl xpos xquat subtree_com con_geom (ncon x 2) moves
    durations."""

    def __init__(self, tables: DancingTables, max_episode_steps: int = MAX_EPISODE_STEPS):
        self.t = tables
        self.max_episode_steps = max_episode_steps

    # ---------------------------------------------------------------- reset
    def apply_reset(self, s, draws):
        m = self.t.model
        s["qpos"][:] = m.qpos0
        s["qvel"][:] = 0
        s["ctrl"][:] = 0
        s.update(current_step=0, beat_count=0, measure=0, t_beat=0.0, score=0.0, combo=1.0, crowd=0.5,
                 applause=0.0, move_idx=0, move_start=0.0, stats=np.zeros(5), hist=[], hist_len=0)
        s["moves"] = np.array(draws[0::2], dtype=np.int64)
        s["durations"] = np.array(draws[1::2])
        q = s["qpos"]
        q[0], q[1], q[2] = 0.0, 0.0, 1.8
        q[3:7] = [1.0, 0.0, 0.0, 0.0]
        for i in range(m.njnt):
            if 7 + i < m.nq and i < m.njnt:
                q[7 + i] = 0.0

    def after_reset(self, s):
        s["prev_jvel"] = s["qvel"][6:].copy()

    # ---------------------------------------------------------------- pre-physics
    def pre(self, s, action):
        a = np.clip(_policy(action), np.float32(-200.0), np.float32(200.0))  # float32 bounds: dtype kept
        s["ctrl"][:] = a
        s["t_beat"] += DT
        if s["t_beat"] >= BEAT:
            s["t_beat"] -= BEAT
            s["beat_count"] += 1
            if s["beat_count"] % 4 == 0:
                s["measure"] += 1
        s["disco"] = s.get("disco", 0.0) + 0.5 * DT
        if s["disco"] > 2 * np.pi:
            s["disco"] -= 2 * np.pi
        r = s["xpos"][self.t.torso]
        target = np.array([r[0], r[1], 5.0])
        s["spotlight"] = s["spotlight"] + 0.1 * (target - s["spotlight"])
        return a

    # ---------------------------------------------------------------- helpers
    def upright(self, s):
        w, x, y, z = np.asarray(s["xquat"][self.t.torso], dtype=np.float64)
        n = max(1e-15, float(np.linalg.norm([w, x, y, z])))
        w, x, y, z = w / n, x / n, y / n, z / n
        return w * w - x * x - y * y + z * z > 0.7

    def foot_contacts(self, s):
        t = self.t
        c = np.zeros(2)
        ground = (t.floor, t.stage)
        for g1, g2 in s["con_geom"]:
            if (g1 == t.right_foot and g2 in ground) or (g2 == t.right_foot and g1 in ground):
                c[0] = 1.0
            if (g1 == t.left_foot and g2 in ground) or (g2 == t.left_foot and g1 in ground):
                c[1] = 1.0
        return c

    def obs(self, s):
        m = self.t.model
        q, v = s["qpos"], s["qvel"]
        o = []
        for i in range(m.nu):
            if i < m.njnt and 7 + i < m.nq:
                lo, hi = m.jnt_range[i]
                o.append(np.clip(2 * (q[7 + i] - lo) / (hi - lo) - 1, -1.0, 1.0) if lo < hi else 0.0)
            else:
                o.append(0.0)
        for i in range(m.nu):
            o.append(np.clip(v[6 + i] / 10.0, -1.0, 1.0) if i < m.nv - 6 else 0.0)
        o += list(s["xquat"][self.t.torso])
        o += list(np.clip(v[:3] / 5.0, -1.0, 1.0))
        o += list(np.clip(v[3:6] / 10.0, -1.0, 1.0))
        o += list(np.clip(s["subtree_com"][self.t.torso] / 10.0, -1.0, 1.0))
        o += list(self.foot_contacts(s))
        o += [0.0, 0.0, 0.0]
        o.append(s["t_beat"] / BEAT)
        o.append((BEAT - s["t_beat"]) / BEAT)
        enc = np.zeros(10)
        if s["move_idx"] < SEQ_LEN:
            enc[s["moves"][s["move_idx"]]] = 1.0
        o += list(enc)
        o.append(np.clip(s["combo"] / 10.0, 0.0, 1.0))
        o.append(s["crowd"])
        o += list(np.clip((s["spotlight"] - s["xpos"][self.t.torso]) / 10.0, -1.0, 1.0))
        o.append(1.0 - min(s["stats"][0] / 1000.0, 1.0))
        return np.array(o, dtype=np.float32)

    def reward(self, s, action):
        m = self.t.model
        v = s["qvel"]
        r = 0.0
        bp = s["t_beat"] / BEAT
        if bp < 0.1 or bp > 0.9:
            if np.linalg.norm(v[6:]) > 1.0:
                r += 100.0
                s["combo"] = min(s["combo"] + 0.1, 10.0)
            else:
                s["combo"] = max(s["combo"] - 0.05, 1.0)
        up = self.upright(s)
        if up:
            r += 30.0
            if np.linalg.norm(v[6:] - s["prev_jvel"]) > 0.5:
                r += 30.0 * 0.5
        jerk = np.linalg.norm(v[6:] - s["prev_jvel"])
        r += 20.0 * np.exp(-0.1 * jerk)
        if s["hist_len"] > 2 and len(set(int(x) for x in s["hist"][-3:])) == 3:
            r += 50.0
        elapsed = s["current_step"] * DT - s["move_start"]
        if s["move_idx"] < SEQ_LEN:
            if elapsed > s["durations"][s["move_idx"]] * 0.8:
                r += 200.0 * DIFFICULTY[s["moves"][s["move_idx"]]]
        used = 0
        for i in range(m.njnt):
            if 7 + i < m.nq:
                lo, hi = m.jnt_range[i]
                if lo < hi:
                    used += abs(s["qpos"][7 + i] - (lo + hi) / 2) / (hi - lo)
        if used > 5.0:
            r += 100.0 * 0.1
        r += -0.05 * np.sum(np.square(action))  # the clipped action's dtype (:1186-1187)
        if not up:
            r += -500.0
            s["combo"] = 1.0
        if 0.2 < bp < 0.8:
            if np.linalg.norm(v[6:]) > 3.0:
                r += -50.0 * 0.1
        if r > 0:
            r *= s["combo"]
        s["score"] += r
        return r

    def terminated(self, s):
        if not self.upright(s):
            if not s["fall_present"]:
                s["fall_present"], s["fall_start"] = True, s["current_step"]
            elif s["current_step"] - s["fall_start"] > 120:
                return True
        elif s["fall_present"]:
            s["fall_present"], s["fall_start"] = False, 0   # delattr

        r = s["xpos"][self.t.torso]
        if np.linalg.norm(r[:2]) > 15.0:
            return True
        return bool(r[2] < 0.0 or r[2] > 5.0)

    def post(self, s, action):
        """After the physics step (dancing_env.py:849-894)."""
        s["current_step"] += 1
        o = self.obs(s)
        r = self.reward(s, action)
        term = self.terminated(s)
        trunc = s["current_step"] >= self.max_episode_steps
        st = s["stats"]
        st[0] += np.sum(np.abs(s["ctrl"])) * DT
        bp = s["t_beat"] / BEAT
        if bp < 0.1 or bp > 0.9:
            st[1] += DT
        st[2] = max(st[2], int(s["combo"]))
        st[3] = s["crowd"]
        st[4] = s["score"]
        on = 0.1 if (s["t_beat"] < 0.1 or s["t_beat"] > BEAT - 0.1) else 0.0
        cf = min(s["combo"] / 10.0, 1.0) * 0.2
        df = DIFFICULTY[s["moves"][s["move_idx"]]] / 4.0 * 0.1 if s["move_idx"] < SEQ_LEN else 0.0
        s["crowd"] = np.clip(s["crowd"] + (on + cf + df) * 0.01, 0.0, 1.0)
        s["crowd"] *= 0.999
        s["applause"] = s["crowd"] * 100.0
        now = s["current_step"] * DT
        if s["move_idx"] < SEQ_LEN and now - s["move_start"] >= s["durations"][s["move_idx"]]:
            s["move_idx"] += 1
            s["move_start"] = now
            if s["move_idx"] < SEQ_LEN:
                s["hist"] = (list(s["hist"]) + [int(s["moves"][s["move_idx"]])])[-3:]
                s["hist_len"] += 1
        s["prev_jvel"] = s["qvel"][6:].copy()
        return o, r, term, trunc
