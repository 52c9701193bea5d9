"""numpy restatement of the humanoid_soccer env logic (TEST INFRASTRUCTURE ONLY).

Follows humanoid_soccer_env/soccer_env.py line by line: goalkeeper :506-524, wind :526-537,
observation :539-631, reward :633-690 (ball contact :787-803, upright :818-833), termination
:692-716, truncation :427, stats :718-730. Pinned against the golden vectors produced by
the reference's own methods (tests/golden/soccer_envlogic.npz, tests/test_oracle_soccer.py).
Used with oracle/mjref.c physics as the end-to-end CPU oracle and CPU baseline.
"""
from __future__ import annotations

import numpy as np

GOAL_OBS = np.array([24.5, 0.0, 1.22])
GOAL = np.array([24.5, 0.0, 0.0])


def quat2mat(q):
    w, x, y, z = np.asarray(q, dtype=np.float64)
    return np.array([[w*w + x*x - y*y - z*z, 2*(x*y - w*z), 2*(x*z + w*y)],
                     [2*(x*y + w*z), w*w - x*x + y*y - z*z, 2*(y*z - w*x)],
                     [2*(x*z - w*y), 2*(y*z + w*x), w*w - x*x - y*y + z*z]])


class SoccerLogic:
    def __init__(self, tables, max_episode_steps=5000):
        self.t = tables
        m = tables.model
        self.m = m
        self.robot_geoms = {g for g, n in enumerate(m.geom_names) if n and any(p in n for p in
                            ['foot', 'shin', 'thigh', 'torso', 'head', 'hand', 'arm'])}
        self.max_episode_steps = max_episode_steps

    # ----- pre-physics (state = dict of numpy arrays; mutated in place)
    @staticmethod
    def action_array(action):
        """The action as the reference holds it after np.clip against the float32 action_space
        bounds: float64 stays float64, anything else becomes float32 (soccer_env.py:401-405)."""
        a = np.asarray(action)
        return a if a.dtype == np.float64 else a.astype(np.float32)

    def pre(self, s, action):
        action = np.clip(self.action_array(action), -150.0, 150.0)
        s["ctrl"][:] = action
        ball = s["xpos"][self.t.ball]
        if ball[0] < -10.0:
            target = np.clip(ball[1], -3.0, 3.0)
            err = target - s["qpos"][self.t.gk_qposadr]
            s["qfrc_applied"][self.t.gk_qfrc_index] = np.clip(50.0 * err, -100.0, 100.0)
        if ball[2] > 0.5:
            s["xfrc_applied"][self.t.ball, :2] += s["wind_strength"] * s["wind_direction"] * 0.1
        return action

    def contact_forces(self, s):
        f = np.zeros(4)
        for (g1, g2), dist, mu in zip(s["con_geom"], s["con_dist"], s["con_mu"]):
            if (g1 == self.t.right_foot and g2 == 0) or (g2 == self.t.right_foot and g1 == 0):
                f[0], f[1] = dist, mu
            if (g1 == self.t.left_foot and g2 == 0) or (g2 == self.t.left_foot and g1 == 0):
                f[2], f[3] = dist, mu
        return f

    def ball_contact(self, s):
        for g1, g2 in s["con_geom"]:
            if g1 == self.t.ball_geom or g2 == self.t.ball_geom:
                other = g2 if g1 == self.t.ball_geom else g1
                if other in self.robot_geoms:
                    return True
        return False

    def upright(self, s):
        return quat2mat(s["xquat"][self.t.torso])[2, 2] > 0.7

    def obs(self, s, step):
        m, t = self.m, self.t
        o = []
        for j in t.obs_joints:
            lo, hi = m.jnt_range[j]
            q = s["qpos"][m.jnt_qposadr[j]]
            o.append(np.clip(2 * (q - lo) / (hi - lo) - 1, -1, 1) if lo < hi else 0.0)
        for j in t.obs_joints:
            o.append(np.clip(s["qvel"][m.jnt_dofadr[j]] / 10.0, -1, 1))
        robot, ball = s["xpos"][t.torso], s["xpos"][t.ball]
        o.extend(s["xquat"][t.torso])
        o.extend(np.clip(s["qvel"][:3] / 5.0, -1, 1))
        o.extend(np.clip(s["qvel"][3:6] / 10.0, -1, 1))
        rel = ball - robot
        o.extend(np.clip(rel / 30.0, -1, 1))
        o.extend(np.clip(s["qvel"][t.ball_dofadr:t.ball_dofadr + 3] / 20.0, -1, 1))
        o.extend(np.clip((GOAL_OBS - robot) / 30.0, -1, 1))
        o.extend(np.clip(self.contact_forces(s) / 1000.0, -1, 1))
        o.extend(np.clip(s["subtree_com"][t.torso] / 30.0, -1, 1))
        o.append(1.0 - step / self.max_episode_steps)
        o.append(np.clip(np.linalg.norm(rel) / 50.0, 0, 1))
        o.extend(np.clip(s["xpos"][t.goalkeeper][:2] / 15.0, -1, 1))
        return np.array(o, dtype=np.float32)

    def reward(self, s, action, ball_contact, upright):
        """_calculate_reward (soccer_env.py:633-690) with the reference's own numpy arithmetic:
        the reward starts as a Python float; the approach / progress terms are np.float64
        (np.linalg.norm); the energy term is np.float32 (-0.1 * float32 pairwise sum), so a reward
        that is still a Python float becomes float32 there (NEP 50), and a later np.float64 term
        promotes it back. Updates goal_scored and the goals / contacts / time_upright stats."""
        t = self.t
        robot, ball = s["xpos"][t.torso], s["xpos"][t.ball]
        r = 0.0
        if ball[0] > 24.0 and abs(ball[1]) < 3.66 and ball[2] < 2.44:
            r += 10000.0
            s["goal_scored"] = True
            s["stats"][0] += 1
        if ball_contact:
            r += 1000.0
            s["stats"][1] += 1
        cur = np.linalg.norm(ball - robot)
        prev = np.linalg.norm(s["prev_ball_pos"] - s["prev_robot_pos"])
        if cur < prev and cur > 2.0:
            r += 500.0 * (prev - cur)
        if upright:
            r += 200.0
            s["stats"][3] += 0.02
        pg, cg = np.linalg.norm(s["prev_robot_pos"] - GOAL), np.linalg.norm(robot - GOAL)
        if cg < pg:
            r += 100.0 * (pg - cg)
        r += -0.1 * np.sum(np.square(self.action_array(action)))
        if not upright:
            r += -1000.0
        pb, cb = np.linalg.norm(s["prev_ball_pos"] - GOAL), np.linalg.norm(ball - GOAL)
        if cb < pb:
            r += 300.0 * (pb - cb)
        return float(r)

    def post(self, s, action, step):
        """Returns obs, reward, terminated, truncated; updates s['goal_scored'], prev_*, stats
        (soccer_env.py:420-446 order: obs, reward, termination, truncation, stats, prev_*)."""
        t = self.t
        obs = self.obs(s, step)
        robot, ball = s["xpos"][t.torso], s["xpos"][t.ball]
        bc = self.ball_contact(s)
        up = self.upright(s)
        r = self.reward(s, action, bc, up)
        term = bool(s["goal_scored"] or (not up and step > 100) or
                    abs(ball[0]) > 30.0 or abs(ball[1]) > 20.0 or ball[2] < -1.0 or ball[2] > 10.0 or
                    abs(robot[0]) > 30.0 or abs(robot[1]) > 20.0 or robot[2] < 0.0 or robot[2] > 5.0)
        trunc = step >= self.max_episode_steps
        # _update_episode_stats :718-730
        s["stats"][2] += np.linalg.norm(robot - s["prev_robot_pos"])
        s["stats"][4] = max(s["stats"][4], np.linalg.norm(s["qvel"][t.ball_dofadr:t.ball_dofadr + 3]))
        s["prev_ball_pos"] = ball.copy()
        s["prev_robot_pos"] = robot.copy()
        return obs, r, term, trunc, bc, up
