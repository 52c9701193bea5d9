"""numpy restatement of the bipedal_rescue env logic (TEST INFRASTRUCTURE ONLY).

Follows bipedal_rescue_env/rescue_env.py line by line: step :416-471 (clip :420, ctrl
:423-424, energy :427-429 -- float32 because np.sum of a float32 action is float32, one RK4
mj_step :432, counter :435), victim pickup / rescue :510-543 (the capacity test runs once
before the loop, so a step can exceed it; gripper check :757-763), observation :545-600
(102 floats; foot "forces" :741-751 sum |dist| of the first 10 contacts into slot 0),
reward :602-668 (persisting _prev_* attributes created lazily, quirk B3; the approach term
is +inf on the first step after a reset when a victim is within 10 m, because
closest_victim_distance restarts at inf), termination :670-697 (the _fall_timer also
persists), stats :699-706, reset :347-396 with _randomize_initial_state :473-508.
Pinned against golden vectors produced by the reference's own step() and reset()
(tests/golden/bipedal_*.npz, tests/test_oracle_bipedal.py). Prints (B4) are not restated.
"""
from __future__ import annotations

import numpy as np

JOINT_NAMES = [
    'neck_pitch', 'neck_yaw',
    'right_shoulder_pitch', 'right_shoulder_roll', 'right_elbow', 'right_wrist',
    'right_finger1_joint', 'right_finger2_joint',
    'left_shoulder_pitch', 'left_shoulder_roll', 'left_elbow', 'left_wrist',
    'left_finger1_joint', 'left_finger2_joint',
    'right_hip_roll', 'right_hip_pitch', 'right_hip_yaw', 'right_knee_joint',
    'right_ankle_pitch', 'right_ankle_roll',
    'left_hip_roll', 'left_hip_pitch', 'left_hip_yaw', 'left_knee_joint',
    'left_ankle_pitch', 'left_ankle_roll']       # rescue_env.py:298-308
SAFE_ZONE = np.array([20.0, 0.0, 0.0])          # rescue_env.py:47
SAFE_RADIUS = 3.0
FIRES = [(np.array([-5.0, -3.0, 0.0]), 1.5), (np.array([8.0, 6.0, 0.0]), 1.2)]  # :75-78
MAX_EPISODE_STEPS = 10000
DT = 0.02
ENERGY_LIMIT = 1000.0
OBS_DIM = 102


class BipedalTables:
    def __init__(self, m):
        self.model = m
        self.torso = m.name2id("body", "torso")
        self.victims = [m.name2id("body", f"victim{i}") for i in range(1, 6)]
        self.joints = [m.name2id("joint", n) for n in JOINT_NAMES]
        self.root_x = int(m.jnt_qposadr[m.name2id("joint", "root_x")])
        self.root_y = int(m.jnt_qposadr[m.name2id("joint", "root_y")])
        self.root_z = int(m.jnt_qposadr[m.name2id("joint", "root_z")])
        self.root_dof = int(m.jnt_dofadr[m.name2id("joint", "root_x")])
        self.victim_x = [int(m.jnt_qposadr[m.name2id("joint", f"victim{i}_x")]) for i in range(1, 6)]
        self.victim_y = [int(m.jnt_qposadr[m.name2id("joint", f"victim{i}_y")]) for i in range(1, 6)]

    @staticmethod
    def reset_draws(rng: np.random.Generator) -> np.ndarray:
        """The 12 uniform draws of one reset, in reference order (rescue_env.py:476-508)."""
        d = [rng.uniform(-5.0, 5.0), rng.uniform(-5.0, 5.0)]
        for _ in range(5):
            d += [rng.uniform(-1.0, 1.0), rng.uniform(-1.0, 1.0)]
        return np.array(d)


def _policy(action):
    """The action as the reference's np.clip against float32 bounds types it: float32 stays float32,
    float64 (and anything numpy promotes with float32 to float64) stays float64."""
    a = np.asarray(action)
    return a.astype(np.result_type(a.dtype, np.float32), copy=False)


def quat2mat(q):
    w, x, y, z = np.asarray(q, dtype=np.float64)
    return np.array([[w*w + x*x - y*y - z*z, 2*(x*y - w*z), 2*(x*z + w*y)],
                     [2*(x*y + w*z), w*w - x*x + y*y - z*z, 2*(y*z - w*x)],
                     [2*(x*z - w*y), 2*(y*z + w*x), w*w - x*x - y*y + z*z]])


class BipedalLogic:
    """State dict keys: qpos qvel ctrl xpos xquat con_dist (first ncon contact dists) step energy
    energy_used rescued carried carrying closest prev_rescued prev_carried prev_sz fall_timer
    (-1 / NaN = attribute absent) stats{victims_rescued, distance, ttfr(None), falls, collisions}
    prev_robot_pos."""

    def __init__(self, tables: BipedalTables, max_episode_steps: int = MAX_EPISODE_STEPS):
        self.t = tables
        self.max_episode_steps = max_episode_steps

    def apply_reset(self, s, draws):
        """rescue_env.py:353-371 + _randomize_initial_state; the _prev_* / _fall_timer attributes
        are NOT touched (quirk B3)."""
        t = self.t
        s["qpos"][:] = t.model.qpos0
        s["qvel"][:] = 0
        s["ctrl"][:] = 0
        s.update(step=0, energy=ENERGY_LIMIT, rescued=[], carried=[], carrying=False, closest=float("inf"),
                 stats=dict(victims_rescued=0, distance=0.0, energy_used=0.0, ttfr=None, falls=0, collisions=0))
        s["qpos"][t.root_x] = draws[0]
        s["qpos"][t.root_y] = draws[1]
        s["qpos"][t.root_z] = 1.2
        for i in range(5):
            s["qpos"][t.victim_x[i]] = s["qpos"][t.victim_x[i]] + draws[2 + 2 * i]
            s["qpos"][t.victim_y[i]] = s["qpos"][t.victim_y[i]] + draws[3 + 2 * i]

    def after_reset(self, s):
        s["prev_robot_pos"] = s["xpos"][self.t.torso].copy()

    def pre(self, s, action):
        # the float32 action_space bounds keep the action's dtype (rescue_env.py:420); the cost, and
        # current_energy / energy_used with it, follow numpy's promotion: a Python float (after reset)
        # or np.float32 minus a float32 cost is float32, anything with a float64 operand float64
        a = np.clip(_policy(action), np.float32(-100.0), np.float32(100.0))
        s["ctrl"][:len(a)] = a
        cost = np.sum(np.abs(a)) * 0.001
        s["energy"] = s["energy"] - cost
        s["stats"]["energy_used"] = s["stats"]["energy_used"] + cost
        return a

    def _robot(self, s):
        return s["xpos"][self.t.torso]

    def _victim(self, s, i):
        return s["xpos"][self.t.victims[i]]

    def interactions(self, s):
        robot = self._robot(s)
        if len(s["carried"]) < 2:
            for i in range(5):
                if i not in s["rescued"] and i not in s["carried"]:
                    d = np.linalg.norm(robot[:2] - self._victim(s, i)[:2])
                    if d < 1.0 and d < 0.8:
                        s["carried"].append(i)
                        s["carrying"] = True
        if s["carrying"]:
            if np.linalg.norm(robot[:2] - SAFE_ZONE[:2]) < SAFE_RADIUS:
                for v in s["carried"]:
                    s["rescued"].append(v)
                    s["stats"]["victims_rescued"] += 1
                    if s["stats"]["ttfr"] is None:
                        s["stats"]["ttfr"] = s["step"] * DT
                s["carried"] = []
                s["carrying"] = False

    def upright(self, s):
        return quat2mat(s["xquat"][self.t.torso])[2, 2] > 0.7

    def obs(self, s):
        m, t = self.t.model, self.t
        o = []
        for j in t.joints:
            o += [s["qpos"][m.jnt_qposadr[j]], s["qvel"][m.jnt_dofadr[j]]]
        robot = self._robot(s)
        o += list(robot) + list(s["xquat"][t.torso])
        o += list(s["qvel"][t.root_dof:t.root_dof + 6])
        f = 0.0
        for dd in s["con_dist"][:10]:
            f += abs(dd)
        o += [f, 0.0, 0.0, 0.0]
        for i in range(5):
            v = self._victim(s, i)
            o += [v[0], v[1], 1.0 if i in s["rescued"] else 0.0, 1.0 if i in s["carried"] else 0.0]
        o += list(SAFE_ZONE - robot)
        o.append(s["energy"] / ENERGY_LIMIT)  # in current_energy's numpy type (:586)
        o.append(1.0 - (s["step"] / self.max_episode_steps))
        o += [len(s["carried"]), len(s["rescued"])]
        for fp, _ in FIRES:
            o += list(fp - robot)
        return np.array(o, dtype=np.float32)

    def reward(self, s, action):
        r = 0.0
        if s["prev_rescued"] >= 0:
            new = len(s["rescued"]) - s["prev_rescued"]
            if new > 0:
                r += 5000.0 * new
        s["prev_rescued"] = len(s["rescued"])
        if s["prev_carried"] >= 0:
            new = len(s["carried"]) - s["prev_carried"]
            if new > 0:
                r += 1000.0 * new
        s["prev_carried"] = len(s["carried"])
        robot = self._robot(s)
        mind = float("inf")
        for i in range(5):
            if i not in s["rescued"] and i not in s["carried"]:
                mind = min(mind, np.linalg.norm(robot[:2] - self._victim(s, i)[:2]))
        if mind < s["closest"] and mind < 10.0:
            r += 100.0 * (s["closest"] - mind)
        s["closest"] = mind
        if s["carrying"]:
            sz = np.linalg.norm(robot[:2] - SAFE_ZONE[:2])
            if not np.isnan(s["prev_sz"]):
                if sz < s["prev_sz"]:
                    r += 200.0 * (s["prev_sz"] - sz)
            s["prev_sz"] = sz
        if self.upright(s):
            r += 50.0
        else:
            r += -500.0
            s["stats"]["falls"] += 1
        usage = np.sum(np.abs(action)) * 0.001  # the clipped action's dtype (:650)
        if usage < 0.5:
            r += 10.0
        for fp, rad in FIRES:
            if np.linalg.norm(robot[:2] - fp[:2]) < rad:
                r += -200.0
        for dd in s["con_dist"][:20]:
            if abs(dd) > 0.1:
                r += -100.0
                s["stats"]["collisions"] += 1
                break
        r += -1.0
        return r

    def terminated(self, s):
        if len(s["rescued"]) == 5:
            return True
        if not self.upright(s):
            if s["fall_timer"] < 0:
                s["fall_timer"] = 0
            s["fall_timer"] += 1
            if s["fall_timer"] > 100:
                return True
        else:
            s["fall_timer"] = 0
        if s["energy"] <= 0:
            return True
        robot = self._robot(s)
        return bool(abs(robot[0]) > 25 or abs(robot[1]) > 25)

    def post(self, s, action):
        """After the physics step: counter, interactions, obs, reward, termination, stats."""
        s["step"] += 1
        self.interactions(s)
        o = self.obs(s)
        r = self.reward(s, action)
        term = self.terminated(s)
        trunc = s["step"] >= self.max_episode_steps
        robot = self._robot(s)
        s["stats"]["distance"] += np.linalg.norm(robot[:2] - s["prev_robot_pos"][:2])
        s["prev_robot_pos"] = robot.copy()
        return o, r, term, trunc
