"""numpy restatement of the quadruped_parkour env logic (TEST INFRASTRUCTURE ONLY).

Follows quadruped_parkour_env/parkour_env.py line by line: step :356-394 (clip :360, ctrl
:363-364, 10 mj_step's :367-368, dynamic obstacles :371 / :776-795, truncation before the
counter increments :381,384), observation :396-468 (foot contacts :470-485 compare geom ids
with BODY ids, quirk P2; foot positions :487-502; constant lidar :504-530; obstacle table
:532-557; terrain :619-634 -- the distance-to-finish slot is never reached, P4), reward
:646-725 (float32 from the energy term on, see `reward`), termination :727-755, reset
:314-354 with the obstacle randomisation :757-774 (joint ids used as qpos indices, P1).
Pinned against the golden vectors produced by the reference's own step()
(tests/golden/parkour_envlogic.npz, tests/test_oracle_parkour.py). Used with oracle/mjref.c
physics as the end-to-end CPU oracle.
"""
from __future__ import annotations

import numpy as np

START_POS = np.array([2.0, 0.0, 0.6])     # parkour_env.py:45
FINISH_X = 98.0                            # parkour_env.py:46
COURSE_HALF_WIDTH = 10.0                   # course_width / 2, parkour_env.py:44
MAX_EPISODE_STEPS = 6000                   # parkour_env.py:41
DT = 0.01                                  # parkour_env.py:38
FRAME_SKIP = 10                            # parkour_env.py:39
CHECKPOINTS = [15, 30, 45, 60, 75, 90]     # parkour_env.py:69
# (x, type code, height, difficulty) -- parkour_env.py:282-297, :559-617
OBSTACLES = [
    (8.0, 1.0, 0.225, 0.3), (16.0, 2.0, 0.2, 0.6), (24.0, 3.0, 0.5, 0.8), (30.0, 4.0, 0.6, 0.4),
    (36.0, 5.0, 0.6, 0.7), (44.0, 6.0, 0.3, 0.9), (50.0, 7.0, 0.08, 0.5), (58.0, 8.0, 0.4, 0.6),
    (72.0, 9.0, 0.25, 0.4), (78.0, 10.0, 0.3, 0.8), (88.0, 11.0, 0.0, 1.0), (92.0, 12.0, 0.2, 1.0)]
ACTION_LIMITS = np.array([80.0, 80.0, 60.0, 40.0] * 4, dtype=np.float32)  # parkour_env.py:236-249
OBS_DIM = 95


def _policy(action):
    """The action as the reference's np.clip against float32 bounds types it: float32 stays float32,
    float64 (and anything numpy promotes with float32 to float64) stays float64."""
    a = np.asarray(action)
    return a.astype(np.result_type(a.dtype, np.float32), copy=False)


class ParkourTables:
    """Index tables looked up exactly as parkour_env.py:180-222 / :757-795 do."""

    def __init__(self, m):
        self.model = m
        self.torso = m.name2id("body", "torso")
        self.feet = [m.name2id("body", f"{k}_foot") for k in ("fl", "fr", "bl", "br")]
        # joint ids, used directly as qpos indices by _randomize_obstacles (quirk P1)
        self.platform_qpos = m.name2id("joint", "platform_slide")
        self.pendulum_qpos = m.name2id("joint", "pendulum_swing")
        self.platform_act = m.name2id("actuator", "platform_motor")
        self.pendulum_act = m.name2id("actuator", "pendulum_motor")
        self.n_leg = 16

    def reset_draws(self, rng: np.random.Generator) -> np.ndarray:
        """The 2 uniform draws of one reset, in reference order (parkour_env.py:764,772)."""
        return np.array([rng.uniform(-1.5, 1.5), rng.uniform(-1.0, 1.0)])


class ParkourLogic:
    def __init__(self, tables: ParkourTables, max_episode_steps: int = MAX_EPISODE_STEPS):
        self.t = tables
        self.max_episode_steps = max_episode_steps

    # ----- reset (parkour_env.py:314-354) on an MjData-like dict; physics settles afterwards
    def apply_reset(self, s, draws):
        s["qpos"][:] = self.t.model.qpos0
        s["qvel"][:] = 0
        s["qpos"][0:3] = START_POS
        s["qpos"][3:7] = [1, 0, 0, 0]
        s["qpos"][self.t.platform_qpos] = draws[0]
        s["qpos"][self.t.pendulum_qpos] = draws[1]
        s.update(step_count=0, episode_reward=0.0, er_kind=0, last_position=START_POS.copy(), max_progress=0.0,
                 reached=0, fall_count=0, stuck=0)

    # ----- pre-physics (parkour_env.py:359-364)
    def pre(self, s, action):
        action = np.clip(_policy(action), -ACTION_LIMITS, ACTION_LIMITS)  # float32 bounds: dtype kept
        s["ctrl"][:self.t.n_leg] = action
        return action

    def after_physics(self, s):
        """_update_dynamic_obstacles (parkour_env.py:776-795): t = step_count * dt, pre-increment."""
        t = s["step_count"] * DT
        s["ctrl"][self.t.platform_act] = 50.0 * np.sin(0.5 * t)
        s["ctrl"][self.t.pendulum_act] = 100.0 * np.sin(0.3 * t)

    def foot_contacts(self, s):
        c = np.zeros(4, dtype=np.float32)
        for i, f in enumerate(self.t.feet):
            for g1, g2 in s["con_geom"]:
                if g1 == f or g2 == f:
                    c[i] = 1.0
                    break
        return c

    def obs(self, s):
        o = np.zeros(OBS_DIM, dtype=np.float32)
        q, v, xpos = s["qpos"], s["qvel"], s["xpos"]
        o[0:16] = q[7:23]
        o[16:32] = v[6:22]
        o[32:36] = q[3:7]
        o[36:39] = v[0:3]
        o[39:42] = v[3:6]
        o[42:45] = q[0:3]
        o[45:49] = self.foot_contacts(s)
        torso = xpos[self.t.torso]
        fp = np.zeros((4, 3), dtype=np.float32)
        for i, f in enumerate(self.t.feet):
            fp[i] = xpos[f] - torso
        o[49:61] = fp.reshape(-1)
        o[61:85] = 10.0
        x = torso[0]
        k = 0
        for pos, code, h, diff in OBSTACLES:
            if pos > x and k < 2:
                o[85 + 4 * k:89 + 4 * k] = [pos - x, code, h, diff]
                k += 1
        o[93] = 0.0
        o[94] = 0.8
        return o

    def reward(self, s, action):
        """Mirrors the reference's dtype flow (numpy >= 2 promotion): the reward is a Python
        float, or np.float64 once the forward-progress term (progress is np.float64) is added.
        The energy term subtracts a numpy float32 (np.sum of |float32 action|): a Python float
        then becomes float32 for every later update, an np.float64 stays float64.
        Returns (reward, is_float32)."""
        pos = s["xpos"][self.t.torso]
        x = pos[0]
        r = 0.0
        r -= 20.0
        progress = x - s["last_position"][0]
        if progress > 0:
            r += progress * 500.0
            s["max_progress"] = max(s["max_progress"], x)
        elif progress < -0.1:
            r -= 100.0
        for b, cx in enumerate(CHECKPOINTS):
            if not (s["reached"] >> b) & 1 and x >= cx:
                s["reached"] |= 1 << b
                r += 1000.0
        for b, (ox, _, _, diff) in enumerate(OBSTACLES):
            if not (s["reached"] >> (6 + b)) & 1 and x > ox + 2.0:
                s["reached"] |= 1 << (6 + b)
                r += 1000.0 + diff * 1000.0
        if x >= FINISH_X:
            r += 5000.0
        if abs(s["qpos"][3]) > 0.7:
            r += 100.0
        n = np.sum(self.foot_contacts(s))
        if 1 <= n <= 3:
            r += 200.0
        effort = np.sum(np.abs(action))  # the clipped action's dtype (parkour_env.py:702-703)
        if effort.dtype == np.float64:  # a float64 action: the reward is np.float64 from here on
            f32 = False
            r = r - effort * 0.1
        else:
            f32 = not progress > 0
            r = np.float32(r) - effort * np.float32(0.1) if f32 else r - float(effort * np.float32(0.1))
        c = np.float32 if f32 else float
        if pos[2] < 0.2:
            r -= c(2000.0)
            s["fall_count"] += 1
        if s["ncon"] > 8:
            r -= c(500.0)
        if abs(progress) < 0.01:
            s["stuck"] += 1
            if s["stuck"] > 100:
                r -= c(100.0)
        else:
            s["stuck"] = 0
        s["last_position"] = pos.copy()
        return float(r), f32

    def terminated(self, s):
        pos = s["xpos"][self.t.torso]
        return bool(pos[0] >= FINISH_X or pos[2] < 0.15 or abs(pos[1]) > COURSE_HALF_WIDTH or
                    s["stuck"] > 1000 or s["fall_count"] > 3)

    def post(self, s, action):
        """After the 10 physics substeps: obstacles, obs, reward, termination, truncation, counters."""
        self.after_physics(s)
        o = self.obs(s)
        r, f32 = self.reward(s, action)
        term = self.terminated(s)
        trunc = s["step_count"] >= self.max_episode_steps
        s["step_count"] += 1
        self.accumulate(s, r, f32)
        return o, r, term, trunc

    @staticmethod
    def accumulate(s, r, f32):
        """episode_reward += reward with numpy >= 2 promotion. The accumulator's kind
        (s["er_kind"]): 0 Python float (after reset), 1 np.float64, 2 np.float32.
        Python float + float32 -> float32; float32 + float32 -> float32; anything with an
        np.float64 -> np.float64."""
        k = s.get("er_kind", 0)
        if f32 and k in (0, 2):
            s["episode_reward"] = float(np.float32(s["episode_reward"]) + np.float32(r))
            s["er_kind"] = 2
        else:
            s["episode_reward"] = s["episode_reward"] + r
            s["er_kind"] = 1 if (not f32 or k == 1 or k == 2) else 0

    @staticmethod
    def course_completion(s, torso_x):
        return min(1.0, max(0.0, (torso_x - START_POS[0]) / (FINISH_X - START_POS[0])))
