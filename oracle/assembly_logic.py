"""numpy restatement of the robotic_arm_assembly env logic (TEST INFRASTRUCTURE ONLY).

Follows robotic_arm_assembly_env/assembly_env.py line by line: step :220-250 (clip + ctrl
:252-265, 10 mj_steps :228-229), task state :267-297, gripper contacts :299-322, reward
:331-387, max contact "force" :389-397, termination :399-417, observation :419-472, info
:474-484, reset :162-218 (deterministic: home pose, components in their bins, 10 settle
steps). Pinned against the golden vectors produced by the reference's own methods
(tests/golden/assembly_envlogic.npz, assembly_reset.npz; tests/test_oracle_assembly.py). Used with
oracle/mjref.c physics (Newton, Euler) as the end-to-end CPU oracle.

Quirks reproduced, not fixed:
  A1  the observation loop writes 9 components x 7 from obs[23], so 'cover' lands on
      obs[79:86]; the status loop then overwrites obs[79:88] with the 9 assembly flags, and
      obs[87] is overwritten again by the held flag. obs[89:114] = 0.5 on a 110-vector fills
      obs[89:110], then obs[104:110] = 0, obs[108] = progress %, obs[109] = phase.
  A2  components are matched to contact geoms by substring in assembly_sequence order, so a
      pad touching a bin ('pcb_bin_base', 'cpu_bin_base', 'cover_bin_base', 'cable_bin_base')
      or a fixture part ('cpu_socket', 'battery_connector', 'cable_connector') "holds" that
      component.
  A3  with two or more distinct components in contact, list(set(names))[0] depends on Python's
      per-process string hashing; we take the first in assembly_sequence order (the case
      with one component, the only deterministic one, matches exactly).
  A4  a 'dropped' component costs -2000 on every later step until it is picked up again;
      once assembled, the progress flag never clears (re-picking only changes the status).
"""
from __future__ import annotations

import numpy as np

SEQUENCE = ('pcb', 'screw1', 'screw2', 'screw3', 'screw4', 'cpu', 'battery', 'cable', 'cover')
TARGETS = {                                       # assembly_env.py:77-87
    'pcb': (0, 0, 0.74), 'cpu': (0, 0, 0.76),
    'screw1': (-0.08, -0.06, 0.735), 'screw2': (0.08, -0.06, 0.735),
    'screw3': (-0.08, 0.06, 0.735), 'screw4': (0.08, 0.06, 0.735),
    'battery': (0.05, 0, 0.77), 'cable': (-0.05, 0, 0.77), 'cover': (0, 0, 0.79)}
BINS = {                                          # assembly_env.py:197-207
    'pcb': [-0.6, 0.3, 0.76], 'cpu': [-0.6, 0, 0.76],
    'screw1': [-0.6, -0.3, 0.76], 'screw2': [-0.58, -0.3, 0.76],
    'screw3': [-0.62, -0.3, 0.76], 'screw4': [-0.6, -0.28, 0.76],
    'battery': [0.6, 0.3, 0.76], 'cable': [0.6, -0.3, 0.76], 'cover': [0.6, 0, 0.76]}
HOME = (0, -0.5, 0.5, 0, 0.5, 0, 0)               # :171
PLACE_REWARD = {'pcb': 2000, 'screw1': 500, 'screw2': 500, 'screw3': 500, 'screw4': 500, 'cpu': 2000,
                'battery': 1000, 'cable': 1000, 'cover': 1000}   # :340-353
JOINT_LOW = (-3.14, -2.36, -2.97, -3.14, -2.09, -3.14, -3.14)    # :411
JOINT_HIGH = (3.14, 0.78, 2.97, 3.14, 2.09, 3.14, 3.14)          # :412
ACTION_LOW = (-2, -2, -2, -2, -2, -2, -2, 0, 0)                   # :150
ACTION_HIGH = (2, 2, 2, 2, 2, 2, 2, 100, 50)                      # :151
ASSEMBLY_TOLERANCE = 0.002     # :42
FORCE_THRESHOLD = 50.0         # :43
GENTLE_FORCE_THRESHOLD = 10.0  # :44
MAX_EPISODE_STEPS = 150000     # :36
SKIP_FRAMES = 10               # :37-39
OBS_DIM = 110
PHASES = ('idle', 'pickup', 'transport', 'align', 'insert')      # :469
STATUS = ('in_bin', 'held', 'assembled', 'dropped', 'damaged')


class AssemblyTables:
    """Name lookups of the reference done once: per-geom component / pad tags (:299-322),
    component body ids (:324-329), the ee_site frame (:437-439), the reset qpos (:162-218)."""

    def __init__(self, m):
        self.model = m
        self.comp_body = np.array([m.name2id("body", c) for c in SEQUENCE], np.int32)
        names = [m.id2name("geom", g) for g in range(m.ngeom)]
        self.geom_named = np.array([bool(n) for n in names])
        self.geom_pad = np.array([bool(n) and 'gripper' in n and 'pad' in n for n in names])
        comp = []
        for n in names:
            k = -1
            if n:
                for i, c in enumerate(SEQUENCE):
                    if c in n:
                        k = i
                        break
            comp.append(k)
        self.geom_comp = np.array(comp, np.int32)
        s = m.name2id("site", "ee_site")
        self.ee_body = int(m.site_bodyid[s])
        self.ee_pos = np.asarray(m.site_pos[s], np.float64).copy()
        self.targets = np.array([TARGETS[c] for c in SEQUENCE], np.float64)
        self.place_reward = np.array([PLACE_REWARD[c] for c in SEQUENCE], np.float64)
        self.joint_low = np.array(JOINT_LOW) * 0.95     # float64 products, as :414 forms them
        self.joint_high = np.array(JOINT_HIGH) * 0.95
        self.action_low = np.array(ACTION_LOW, np.float32)
        self.action_high = np.array(ACTION_HIGH, np.float32)
        q = np.asarray(m.qpos0, np.float64).copy()
        q[0:7] = HOME
        for c in SEQUENCE:
            b = m.name2id("body", c)
            a = m.jnt_qposadr[m.body_jntadr[b]]
            q[a:a + 3] = BINS[c]
            q[a + 3:a + 7] = [1, 0, 0, 0]
        self.reset_qpos = q


def site_xpos(xpos, xmat, body, pos):
    """mj_kinematics' site position: xpos[body] + xmat[body] @ site_pos."""
    R = np.asarray(xmat[body], np.float64).reshape(3, 3)
    return np.asarray(xpos[body], np.float64) + R @ pos


class AssemblyLogic:
    def __init__(self, tables: AssemblyTables, max_episode_steps: int = MAX_EPISODE_STEPS):
        self.t = tables
        self.max_episode_steps = max_episode_steps

    @staticmethod
    def new_state():
        """Tracking state after reset() (:177-183)."""
        return dict(step=0, held=-1, phase=0, progress=[False] * 9, status=[0] * 9, cumulative=0)

    def pre(self, action):
        """np.clip to the float32 action bounds; ctrl[0:7] = a[0:7], ctrl[7] = ctrl[8] = a[7] / 1000
        (float32 stays float32: NEP 50) (:252-265)."""
        a = np.clip(np.asarray(action), self.t.action_low, self.t.action_high)
        ctrl = np.zeros(9)
        ctrl[0:7] = a[0:7]
        g = a[7] / 1000.0
        ctrl[7] = g
        ctrl[8] = g
        return a, ctrl

    def contact_components(self, con_geom):
        """Components touched by a gripper pad (:299-322) as a set of sequence indices."""
        t = self.t
        out = set()
        for g1, g2 in con_geom:
            if not (t.geom_named[g1] and t.geom_named[g2]):
                continue
            if t.geom_pad[g1]:
                if t.geom_comp[g2] >= 0:
                    out.add(int(t.geom_comp[g2]))
            elif t.geom_pad[g2]:
                if t.geom_comp[g1] >= 0:
                    out.add(int(t.geom_comp[g1]))
        return out

    @staticmethod
    def max_force(con_dist):
        """:389-397: max |dist| * 1000 over the contacts (the int 0 with none)."""
        mf = 0
        for d in con_dist:
            mf = max(mf, abs(float(d)) * 1000)
        return mf

    def update_task_state(self, s, comps, xpos):
        """:267-297 (quirk A3: the first touched component in sequence order)."""
        if comps:
            if s["held"] < 0:
                s["held"] = min(comps)
                s["phase"] = 1
                s["status"][s["held"]] = 1
            else:
                s["phase"] = 2
        elif s["held"] >= 0:
            h = s["held"]
            d = np.linalg.norm(np.asarray(xpos[self.t.comp_body[h]]) - self.t.targets[h])
            if d < ASSEMBLY_TOLERANCE:
                s["progress"][h] = True
                s["status"][h] = 2
                s["phase"] = 4
            else:
                s["status"][h] = 3
                s["phase"] = 0
            s["held"] = -1
        else:
            s["phase"] = 0

    def reward(self, s, xpos, qvel, con_dist):
        """_calculate_reward (:331-387), float64 in the reference's order."""
        t = self.t
        r = -10
        if s["phase"] == 1 and s["held"] >= 0:
            r += 1000
        for i in range(9):
            if s["progress"][i] and s["status"][i] == 2:
                r += int(t.place_reward[i])
        if s["held"] >= 0:
            h = s["held"]
            dist = np.linalg.norm(np.asarray(xpos[t.comp_body[h]]) - t.targets[h])
            if dist < 0.05:
                r += 300 * (1 - dist / 0.05)
        mf = self.max_force(con_dist)
        if mf > FORCE_THRESHOLD:
            r -= 5000
        elif mf < GENTLE_FORCE_THRESHOLD:
            r += 200
        r += -np.sum(np.abs(np.asarray(qvel[0:7]))) * 10
        for i in range(9):
            if s["status"][i] == 3:
                r -= 2000
            elif s["status"][i] == 4:
                r -= 5000
        if all(s["progress"]):
            r += 10000
        return r

    def terminated(self, s, qpos):
        if all(s["progress"]):
            return True
        if any(st == 4 for st in s["status"]):
            return True
        q = np.asarray(qpos[0:7])
        return bool(np.any(q < self.t.joint_low) or np.any(q > self.t.joint_high))

    def obs(self, s, qpos, qvel, xpos, xmat, con_dist):
        t = self.t
        o = np.zeros(OBS_DIM, dtype=np.float32)
        o[0:7] = qpos[0:7]
        o[7:14] = qvel[0:7]
        o[14] = (qpos[7] + qpos[8]) / 2.0 * 1000
        o[15] = self.max_force(con_dist)
        o[16:19] = site_xpos(xpos, xmat, t.ee_body, t.ee_pos)
        o[19:23] = [1, 0, 0, 0]
        idx = 23
        for i in range(9):
            o[idx:idx + 3] = xpos[t.comp_body[i]]
            o[idx + 3:idx + 7] = [1, 0, 0, 0]
            idx += 7
        for i in range(9):
            o[79 + i] = float(s["progress"][i])
        o[87] = float(s["held"] >= 0)
        o[88] = s["held"] if s["held"] >= 0 else -1
        o[89:114] = 0.5
        o[104:110] = 0
        o[108] = sum(s["progress"]) / len(s["progress"]) * 100
        o[109] = s["phase"]
        return o

    def post(self, s, qpos, qvel, xpos, xmat, con_geom, con_dist):
        """After the 10 mj_steps (:232-244). Returns (obs, reward, terminated, truncated)."""
        s["step"] += 1
        self.update_task_state(s, self.contact_components(con_geom), xpos)
        r = self.reward(s, xpos, qvel, con_dist)
        s["cumulative"] += r
        term = self.terminated(s, qpos)
        trunc = s["step"] >= self.max_episode_steps
        return self.obs(s, qpos, qvel, xpos, xmat, con_dist), r, term, trunc
