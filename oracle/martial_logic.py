"""numpy restatement of the humanoid_martial_arts env logic (TEST INFRASTRUCTURE ONLY).

Follows humanoid_martial_arts_env/martial_arts_env.py line by line: step :489-523 (clip :492,
ctrl = action * ctrlrange[:, 1] :495), observation :525-560, reward :562-606, termination
:608-621, statistics :632-640, reset :442-487. Pinned against the golden vectors produced by the
reference's own methods (tests/golden/martial_envlogic.npz, martial_reset.npz;
tests/test_oracle_martial.py). Used with oracle/mjref.c physics (Newton, Euler) as the
end-to-end CPU oracle.

Quirks reproduced, not fixed:
  M1  reset writes the "torso" pose into qpos[0:7], which is dummy1's free joint (the first
      body in the scene), so the humanoid starts at its qpos0 pose and dummy1 is moved.
  M2  the observation is 113 floats (qpos[7:], qvel[6:] cover dummy2 / board / humanoid) while
      observation_space declares 29 + 2 nu = 85 (:408-420); cvel[:3], observed as the "linear"
      velocity, is the angular part of MuJoCo's com-based cvel.
  M3  prev_torso_pos is an attribute created at the first step with current_step > 1 and it
      survives reset(); total_distance_moved uses it from then on.
"""
from __future__ import annotations

import numpy as np

DT = 0.01667                 # martial_arts_env.py:45
ROBOT_HEIGHT = 1.75          # :55
BALANCE_REWARD = 100.0       # :78
STANCE_REWARD = 200          # :64 (int)
PUNCH_REWARD = 500           # :60
KICK_REWARD = 800            # :61
THIRD_DUMMY = (0.0, -2.0, 1.0)   # :550
MAX_EPISODE_STEPS = 6000     # :46
STAT_KEYS = ('techniques_performed', 'successful_combos', 'balance_maintained', 'max_power_generated',
             'total_distance_moved', 'falls')


class MartialTables:
    """Index tables of _get_model_indices (martial_arts_env.py:383-395)."""

    def __init__(self, m):
        self.model = m
        self.torso = m.name2id("body", "torso")
        self.head = m.name2id("body", "head")
        self.right_hand = m.name2id("body", "right_hand")
        self.left_hand = m.name2id("body", "left_hand")
        self.right_foot = m.name2id("body", "right_ankle")
        self.left_foot = m.name2id("body", "left_ankle")
        self.dummy1 = m.name2id("body", "dummy1")
        self.dummy2 = m.name2id("body", "dummy2")
        self.ctrl_scale = np.asarray(m.actuator_ctrlrange)[:, 1].copy()
        self.nu = m.nu

    @staticmethod
    def reset_draws(rng: np.random.Generator) -> np.ndarray:
        """The 2 uniform draws of one reset, in reference order (:460-463)."""
        return np.array([rng.uniform(-0.5, 0.5), rng.uniform(-0.5, 0.5)])


class MartialLogic:
    def __init__(self, tables: MartialTables, max_episode_steps: int = MAX_EPISODE_STEPS):
        self.t = tables
        self.max_episode_steps = max_episode_steps

    @staticmethod
    def new_state():
        """Per-env Python-side state of the reference env (constructor + attributes)."""
        return dict(current_step=0, stance=0.0, stats={k: 0 for k in STAT_KEYS}, prev_torso=None)

    def apply_reset(self, s, qpos0, draws):
        """reset() (:442-487) on a freshly mj_resetData'd state: returns the new qpos."""
        q = np.array(qpos0, dtype=np.float64)
        q[0:3] = [0, 0, 1.4]
        q[3:7] = [1, 0, 0, 0]
        q[0] += draws[0]
        q[1] += draws[1]
        s["current_step"] = 0
        s["stance"] = 0.0
        for k in s["stats"]:
            s["stats"][k] = 0
        return q

    def pre(self, action):
        """clip (float32 stays float32) and ctrl = action * ctrlrange[:, 1] (:492-495)."""
        a = np.clip(np.asarray(action), -1.0, 1.0)
        return a, a * self.t.ctrl_scale

    def obs(self, s):
        t = self.t
        o = []
        o.extend(s["xpos"][t.torso])
        o.extend(s["xquat"][t.torso])
        o.extend(s["cvel"][t.torso][:3])
        o.extend(s["cvel"][t.torso][3:])
        o.extend(s["qpos"][7:])
        o.extend(s["qvel"][6:])
        o.extend(s["xpos"][t.dummy1])
        o.extend(s["xpos"][t.dummy2])
        o.extend(THIRD_DUMMY)
        o.extend([0.0, 0.0, 0.0, 0.0])
        o.append(0.0)                 # technique_accuracy
        o.append(0)                   # len(combo_chain)
        o.append(s["stance"])
        return np.array(o, dtype=np.float32)

    def reward(self, s, action):
        """_calculate_reward (:562-606) with the reference's numpy types: min(1.0, np.float64) keeps
        whichever argument wins, the velocity and distance terms are np.float64, the energy term
        np.float32 (float32 pairwise sum x 0.01), so a still-Python-float reward turns float32
        there (NEP 50) and the approach term promotes it back to float64."""
        t = self.t
        reward = 0.0
        torso_height = s["xpos"][t.torso][2]
        reward += BALANCE_REWARD * min(1.0, torso_height / ROBOT_HEIGHT)
        rh = np.linalg.norm(s["cvel"][t.right_hand][:3])
        lh = np.linalg.norm(s["cvel"][t.left_hand][:3])
        if rh > 2.0 or lh > 2.0:
            reward += PUNCH_REWARD
            s["stats"]['techniques_performed'] += 1
        rf = np.linalg.norm(s["cvel"][t.right_foot][:3])
        lf = np.linalg.norm(s["cvel"][t.left_foot][:3])
        if rf > 3.0 or lf > 3.0:
            reward += KICK_REWARD
            s["stats"]['techniques_performed'] += 1
        ang = np.linalg.norm(s["cvel"][t.torso][3:])
        if ang < 0.5:
            s["stance"] += DT
            reward += STANCE_REWARD * DT
        reward -= np.sum(np.abs(action)) * 0.01
        dist = np.linalg.norm(s["xpos"][t.dummy1][:2] - s["xpos"][t.torso][:2])
        if dist < 2.0:
            reward += 50 * (2.0 - dist)
        return reward

    def terminated(self, s):
        z = s["xpos"][self.t.torso][2]
        if z < 0.5:
            s["stats"]['falls'] += 1
            return True
        p = s["xpos"][self.t.torso]
        return bool(abs(p[0]) > 5.5 or abs(p[1]) > 5.5)

    def statistics(self, s):
        """_update_statistics (:632-640): prev_torso_pos is created lazily and survives reset."""
        if s["current_step"] > 1:
            tp = s["xpos"][self.t.torso]
            if s["prev_torso"] is not None:
                s["stats"]['total_distance_moved'] += np.linalg.norm(tp[:2] - s["prev_torso"][:2])
            s["prev_torso"] = tp.copy()

    def post(self, s, action):
        """After mj_step: counter, obs, reward, termination, truncation, stats (:500-517).
        Returns (obs, reward (the reference's numpy scalar), terminated, truncated)."""
        s["current_step"] += 1
        o = self.obs(s)
        r = self.reward(s, action)
        term = self.terminated(s)
        trunc = s["current_step"] >= self.max_episode_steps
        self.statistics(s)
        return o, r, term, trunc
