"""Generate the committed golden fixtures from the reference's own Python code.

Run in the build container only (needs /root/reference):  python tests/golden/make_fixtures.py

The reference's env modules import `mujoco` and `gymnasium`, neither of which is installed
(SURVEY.md §8c). We import them with tiny stub modules and call the reference's own methods:

1. composed MJCF strings: HumanoidSoccerEnv._load_xml_models (soccer_env.py:120-220),
   QuadrupedParkourEnv._combine_models (parkour_env.py:105-179),
   BipedalRescueEnv._load_xml_models (rescue_env.py:121-277),
   HumanoidDancingEnv._load_xml_models (dancing_env.py:156-678); the construction,
   martial-arts and assembly XML are the reference's on-disk assets (byte-identical to
   their generators per SURVEY.md §8c).
2. soccer reset randomisation (soccer_env.py:454-504) for a list of seeds.
3. soccer env-logic vectors: _update_goalkeeper, _apply_environmental_effects,
   _get_observation, _calculate_reward, _check_termination (soccer_env.py:506-716) on
   synthetic MjData-like state with contact lists.

Only data (inputs -> outputs) is written; nothing from the reference is copied into the repo.
The fake MjModel/MjData fields come from our own MJCF compiler (name tables, jnt_* arrays).
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)

from mujoco_gymnasium_environments_amd import mjcf  # noqa: E402


# ------------------------------------------------------------------------------- stubs
class _Box:
    def __init__(self, low, high, shape=None, dtype=np.float32):
        dtype = np.dtype(dtype)
        if shape is not None:
            self.low = np.full(shape, low, dtype=dtype)
            self.high = np.full(shape, high, dtype=dtype)
        else:
            self.low = np.asarray(low, dtype=dtype)
            self.high = np.asarray(high, dtype=dtype)
        self.shape = self.low.shape
        self.dtype = dtype


# dtype of the synthetic policy actions fed to the reference step() (main_f64: float64)
ACTION_DTYPE = np.float32

def _np_random(seed=None):
    ss = np.random.SeedSequence(seed)
    return np.random.Generator(np.random.PCG64(ss)), ss.entropy


class _ObjT:
    mjOBJ_BODY, mjOBJ_JOINT, mjOBJ_GEOM, mjOBJ_SITE, mjOBJ_ACTUATOR, mjOBJ_SENSOR = range(6)


_KIND = {0: "body", 1: "joint", 2: "geom", 3: "site", 4: "actuator"}
CURRENT_MODEL: dict = {}


def _quat2mat(res, quat):
    w, x, y, z = quat
    R = mjcf.quat2mat(np.array([w, x, y, z], dtype=np.float64) /
                      max(1e-15, float(np.linalg.norm(quat))))
    res[:] = R.reshape(-1)


def install_stubs():
    mj = types.ModuleType("mujoco")
    mj.mjtObj = _ObjT
    mj.mj_name2id = lambda m, t, n: m._c.name2id(_KIND[t], n) if t in _KIND else -1
    mj.mj_id2name = lambda m, t, i: m._c.id2name(_KIND[t], i)
    mj.mju_quat2Mat = _quat2mat
    mj.mj_step = lambda m, d: setattr(d, "nstep", getattr(d, "nstep", 0) + 1)
    mj.mj_resetData = lambda m, d: d.reset()
    mj.mj_forward = lambda m, d: None

    class MjModel:
        @staticmethod
        def from_xml_string(xml):
            return FakeModel(mjcf.compile_xml(xml))
    mj.MjModel = MjModel
    mj.MjData = lambda m: FakeData(m)
    viewer = types.ModuleType("mujoco.viewer")
    mj.viewer = viewer
    sys.modules["mujoco"] = mj
    sys.modules["mujoco.viewer"] = viewer

    gym = types.ModuleType("gymnasium")

    class Env:
        """gymnasium.Env.reset's seeding (gymnasium/core.py): a given seed reseeds _np_random."""
        def reset(self, seed=None, options=None):
            if seed is not None:
                self._np_random, self._np_random_seed = _np_random(seed)
    gym.Env = Env
    spaces = types.ModuleType("gymnasium.spaces")
    spaces.Box = _Box
    spaces.Dict = dict
    spaces.Discrete = lambda n: n
    gym.spaces = spaces
    utils = types.ModuleType("gymnasium.utils")
    seeding = types.ModuleType("gymnasium.utils.seeding")
    seeding.np_random = _np_random
    utils.seeding = seeding
    gym.utils = utils
    gym.register = lambda *a, **k: None
    err = types.ModuleType("gymnasium.error")
    err.Error = Exception
    gym.error = err
    envs = types.ModuleType("gymnasium.envs")
    reg = types.ModuleType("gymnasium.envs.registration")
    reg.register = lambda *a, **k: None
    envs.registration = reg
    gym.envs = envs
    for k, v in {"gymnasium": gym, "gymnasium.spaces": spaces, "gymnasium.utils": utils,
                 "gymnasium.utils.seeding": seeding, "gymnasium.error": err,
                 "gymnasium.envs": envs, "gymnasium.envs.registration": reg}.items():
        sys.modules[k] = v


class FakeModel:
    def __init__(self, c: mjcf.Model):
        self._c = c
        self.nu, self.nq, self.nv, self.nbody, self.ngeom = c.nu, c.nq, c.nv, c.nbody, c.ngeom
        self.njnt = c.njnt
        self.jnt_qposadr = c.jnt_qposadr.copy()
        self.body_jntadr = c.body_jntadr.copy()
        self.jnt_dofadr = c.jnt_dofadr.copy()
        self.jnt_range = c.jnt_range.copy()
        self.qpos0 = c.qpos0.copy()
        self.actuator_ctrlrange = c.actuator_ctrlrange.copy()

    def body(self, name):
        """mjModel.body(name) accessor (martial_arts_env.py:386-395)."""
        return types.SimpleNamespace(id=self._c.name2id("body", name))


class FakeContact:
    def __init__(self, g1, g2, dist, friction):
        self.geom1, self.geom2, self.dist = int(g1), int(g2), float(dist)
        self.friction = np.asarray(friction, dtype=np.float64)


class FakeData:
    def __init__(self, m: FakeModel):
        self.m = m
        self.reset()

    def reset(self):
        c = self.m._c
        self.qpos = c.qpos0.copy()
        self.qvel = np.zeros(c.nv)
        self.ctrl = np.zeros(c.nu)
        self.qfrc_applied = np.zeros(c.nv)
        self.xfrc_applied = np.zeros((c.nbody, 6))
        self.xpos = np.zeros((c.nbody, 3))
        self.xquat = np.tile([1.0, 0, 0, 0], (c.nbody, 1))
        self.xmat = np.tile(np.eye(3).reshape(-1), (c.nbody, 1))
        self.subtree_com = np.zeros((c.nbody, 3))
        self.cvel = np.zeros((c.nbody, 6))
        self.site_xpos = np.zeros((len(c.site_names), 3))
        self.contact = []
        self.ncon = 0
        self.time = 0.0


def load_module(path, name):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


# ------------------------------------------------------------------------------- XML
def dump_xml():
    out = {}
    soccer = load_module(f"{REF}/humanoid_soccer_env/soccer_env.py", "ref_soccer_env")
    o = object.__new__(soccer.HumanoidSoccerEnv)
    o.dt = 0.02
    soccer.HumanoidSoccerEnv._load_xml_models(o)
    out["humanoid_soccer"] = o.xml_string

    parkour = load_module(f"{REF}/quadruped_parkour_env/parkour_env.py", "ref_parkour_env")
    o = object.__new__(parkour.QuadrupedParkourEnv)
    a = f"{REF}/quadruped_parkour_env/assets"
    out["quadruped_parkour"] = parkour.QuadrupedParkourEnv._combine_models(
        o, f"{a}/quadruped.xml", f"{a}/parkour_course.xml", f"{a}/terrain_variations.xml")

    bip = load_module(f"{REF}/bipedal_rescue_env/rescue_env.py", "ref_rescue_env")
    o = object.__new__(bip.BipedalRescueEnv)
    o.dt = 0.02
    bip.BipedalRescueEnv._load_xml_models(o)
    out["bipedal_rescue"] = o.xml_string
    # the dancing composition reads constructor attributes (floor_radius, ...): run the
    # reference constructor itself (stub mujoco) and keep the string it compiled
    import contextlib
    import io
    dan = load_module(f"{REF}/humanoid_dancing_env/dancing_env.py", "ref_dancing_env")
    with contextlib.redirect_stdout(io.StringIO()):
        out["humanoid_dancing"] = dan.HumanoidDancingEnv(render_mode=None).xml_string
    # construction / martial arts / assembly load their on-disk assets unchanged; those files
    # are read from /root/reference by the tests that need them, never copied into the repo.
    os.makedirs(f"{HERE}/xml", exist_ok=True)
    for k, v in out.items():
        with open(f"{HERE}/xml/{k}.xml", "w") as f:
            f.write(v)
    # the package ships the composed soccer / parkour models it simulates
    pkg_assets = f"{REPO}/mujoco_gymnasium_environments_amd/assets"
    os.makedirs(pkg_assets, exist_ok=True)
    for k in ("humanoid_soccer", "quadruped_parkour", "bipedal_rescue", "humanoid_dancing"):
        with open(f"{pkg_assets}/{k}.xml", "w") as f:
            f.write(out[k])
    return out


# ------------------------------------------------------------------------------- soccer
def soccer_env():
    install_stubs()
    soccer = load_module(f"{REF}/humanoid_soccer_env/soccer_env.py", "ref_soccer_env2")
    env = soccer.HumanoidSoccerEnv(render_mode=None)
    return env


def soccer_reset_vectors(env, seeds):
    rows = []
    for s in seeds:
        env.seed(int(s))
        env.data.reset()
        env._randomize_initial_state()
        env._update_environmental_factors()
        rows.append(dict(qpos=env.data.qpos.copy(), wind_strength=env.wind_strength,
                         wind_direction=env.wind_direction.copy(),
                         friction_var=env.field_friction_variation))
    return dict(seeds=np.asarray(seeds, np.int64),
                qpos=np.stack([r["qpos"] for r in rows]),
                wind_strength=np.array([r["wind_strength"] for r in rows]),
                wind_direction=np.stack([r["wind_direction"] for r in rows]),
                friction_var=np.array([r["friction_var"] for r in rows]))


def soccer_envlogic_vectors(env, n, seed=1234, max_contacts=12):
    """Random synthetic states -> reference env-logic outputs."""
    c = env.model._c
    rng = np.random.default_rng(seed)
    torso, ball, gk = env.torso_id, env.ball_id, env.goalkeeper_id
    cand = c.pair_geom
    nb, nq, nv = c.nbody, c.nq, c.nv
    keys = ["qpos", "qvel", "xpos", "xquat", "subtree_com", "ncon", "con_geom", "con_dist",
            "con_friction", "prev_ball_pos", "prev_robot_pos", "current_step", "goal_scored_in",
            "wind_strength", "wind_direction", "qfrc_applied_in", "xfrc_applied_in", "action",
            # outputs
            "qfrc_applied_out", "xfrc_applied_out", "obs", "reward", "terminated", "truncated",
            "goal_scored_out", "ball_contact", "upright", "stats_in", "stats_out"]
    out = {k: [] for k in keys}
    # episode stats come from their own stream so the other vectors do not depend on them
    srng = np.random.default_rng(seed + 1)
    for i in range(n):
        d = env.data
        d.reset()
        lo, hi = c.jnt_range[:, 0], c.jnt_range[:, 1]
        qpos = c.qpos0.copy()
        for j in range(c.njnt):
            a = c.jnt_qposadr[j]
            if c.jnt_type[j] == mjcf.JNT_FREE:
                qpos[a:a + 3] = rng.uniform(-20, 20, 3)
                q = rng.normal(size=4)
                qpos[a + 3:a + 7] = q / np.linalg.norm(q)
            else:
                span = hi[j] - lo[j]
                qpos[a] = rng.uniform(lo[j] - 0.2 * span, hi[j] + 0.2 * span)
        d.qpos[:] = qpos
        d.qvel[:] = rng.normal(scale=rng.choice([0.5, 5.0, 30.0]), size=nv)
        xpos = rng.uniform(-5, 5, (nb, 3))
        scen = i % 8
        xpos[torso] = [rng.uniform(-32, 32), rng.uniform(-22, 22), rng.uniform(-0.5, 5.5)]
        xpos[ball] = [rng.uniform(-32, 32), rng.uniform(-22, 22), rng.uniform(-1.5, 11)]
        if scen == 0:   # goal zone
            xpos[ball] = [rng.uniform(24.0, 26), rng.uniform(-3.6, 3.6), rng.uniform(0, 2.4)]
        elif scen == 1:  # ball deep in own half -> goalkeeper reacts
            xpos[ball] = [rng.uniform(-25, -10.01), rng.uniform(-6, 6), rng.uniform(0.1, 1.5)]
        elif scen == 2:  # in bounds, calm
            xpos[torso] = [rng.uniform(-20, 20), rng.uniform(-10, 10), rng.uniform(0.5, 2)]
            xpos[ball] = [rng.uniform(-20, 20), rng.uniform(-10, 10), rng.uniform(0.1, 3)]
        xpos[gk] = [-23.0, rng.uniform(-3.7, 3.7), 0.9]
        d.xpos[:] = xpos
        q = rng.normal(size=(nb, 4))
        if scen in (2, 3):
            q[torso] = [1, rng.normal(scale=0.2), rng.normal(scale=0.2), rng.normal()]
        d.xquat[:] = q / np.linalg.norm(q, axis=1, keepdims=True)
        d.subtree_com[:] = rng.uniform(-40, 40, (nb, 3))
        ncon = int(rng.integers(0, max_contacts + 1))
        picks = rng.integers(0, len(cand), ncon)
        geoms = cand[picks].copy()
        # force foot-ground and ball-limb contacts into some cases
        if scen in (4, 5) and ncon >= 2:
            geoms[0] = [0, env.right_foot_id]
            geoms[-1] = [env.left_foot_id, 0] if scen == 4 else [0, env.left_foot_id]
        if scen in (5, 6) and ncon >= 3:
            geoms[1] = [env.ball_geom_id, int(rng.integers(31, 45))]
        dist = rng.uniform(-0.05, 0.01, ncon)
        fric = np.tile([1.0, 1.0, 0.5, 0.5, 0.5], (ncon, 1)) * rng.uniform(0.5, 1.5, (ncon, 1))
        d.contact = [soccer_contact(g[0], g[1], dd, ff) for g, dd, ff in zip(geoms, dist, fric)]
        d.ncon = ncon
        env.prev_ball_pos = xpos[ball] + rng.normal(scale=0.3, size=3)
        env.prev_robot_pos = xpos[torso] + rng.normal(scale=0.3, size=3)
        env.current_step = int(rng.choice([0, 50, 100, 101, 2000, 4999, 5000, int(rng.integers(0, 6000))]))
        env.goal_scored = bool(rng.random() < 0.15)
        goal_in = env.goal_scored
        env.wind_strength = float(rng.uniform(0, 2))
        ang = float(rng.uniform(0, 2 * np.pi))
        env.wind_direction = np.array([np.cos(ang), np.sin(ang)])
        d.qfrc_applied[:] = 0
        d.qfrc_applied[0] = rng.uniform(-100, 100)
        d.xfrc_applied[:] = 0
        d.xfrc_applied[ball, :2] = rng.normal(size=2)
        qfrc_in = d.qfrc_applied[0]
        xfrc_in = d.xfrc_applied[ball, :2].copy()
        action = rng.uniform(-200, 200, c.nu).astype(ACTION_DTYPE)
        action = np.clip(action, env.action_space.low, env.action_space.high)
        # the episode stats entering this step; _calculate_reward advances goals / contacts /
        # time_upright on them (soccer_env.py:640-662)
        sin = np.array([srng.integers(0, 3), srng.integers(0, 50), srng.uniform(0, 40), srng.uniform(0, 30),
                        srng.choice([0.0, srng.uniform(0, 20)])])
        env.episode_stats = {'goals_scored': int(sin[0]), 'ball_contacts': int(sin[1]),
                             'distance_traveled': float(sin[2]), 'time_upright': float(sin[3]),
                             'max_ball_speed': float(sin[4])}
        # pre-physics env logic (soccer_env.py:408-411)
        env._update_goalkeeper()
        env._apply_environmental_effects()
        # post-physics (soccer_env.py:420-427); physics is not run: state is synthetic
        obs = env._get_observation()
        reward = env._calculate_reward(action)
        term = env._check_termination()
        trunc = env.current_step >= env.max_episode_steps
        # _update_episode_stats (soccer_env.py:718-730): after the flags, before prev_* move
        env._update_episode_stats()
        es = env.episode_stats
        sout = np.array([es['goals_scored'], es['ball_contacts'], es['distance_traveled'], es['time_upright'],
                         es['max_ball_speed']], dtype=np.float64)
        vals = dict(qpos=qpos, qvel=d.qvel.copy(), xpos=xpos, xquat=d.xquat.copy(),
                    subtree_com=d.subtree_com.copy(), ncon=ncon,
                    con_geom=_pad(geoms, max_contacts, 2, -1), con_dist=_pad(dist, max_contacts),
                    con_friction=_pad(fric, max_contacts, 5), prev_ball_pos=env.prev_ball_pos,
                    prev_robot_pos=env.prev_robot_pos, current_step=env.current_step,
                    goal_scored_in=goal_in, wind_strength=env.wind_strength,
                    wind_direction=env.wind_direction, qfrc_applied_in=qfrc_in,
                    xfrc_applied_in=xfrc_in, action=action,
                    qfrc_applied_out=d.qfrc_applied[0], xfrc_applied_out=d.xfrc_applied[ball, :2].copy(),
                    obs=obs, reward=float(reward), terminated=bool(term), truncated=bool(trunc),
                    goal_scored_out=bool(env.goal_scored), ball_contact=bool(env._check_ball_contact()),
                    upright=bool(env._is_robot_upright()), stats_in=sin.astype(np.float64), stats_out=sout)
        for k in keys:
            out[k].append(vals[k])
    return {k: np.asarray(v) for k, v in out.items()}


def soccer_contact(g1, g2, dist, fr):
    return FakeContact(g1, g2, dist, fr)


def _pad(a, n, w=None, fill=0.0):
    a = np.asarray(a, dtype=np.float64)
    shape = (n,) if w is None else (n, w)
    out = np.full(shape, fill, dtype=np.float64)
    if len(a):
        out[:len(a)] = a
    return out


# ------------------------------------------------------------------------------- parkour
PARKOUR_OBSTACLES = [8.0, 16.0, 24.0, 30.0, 36.0, 44.0, 50.0, 58.0, 72.0, 78.0, 88.0, 92.0]
PARKOUR_CHECKPOINTS = [15, 30, 45, 60, 75, 90]


def parkour_env():
    install_stubs()
    mod = load_module(f"{REF}/quadruped_parkour_env/parkour_env.py", "ref_parkour_env2")
    return mod.QuadrupedParkourEnv(render_mode=None)


def _parkour_keys(env):
    """bit k of the reached-mask <-> key k of checkpoints_reached: 6 checkpoints, 12 obstacles"""
    return list(PARKOUR_CHECKPOINTS) + [f"{x}_{t}" for x, t in env.obstacle_positions]


def parkour_reset_vectors(env, seeds):
    """reset(seed) (parkour_env.py:314-354): the randomised qpos before the settle steps (the
    stub mj_step does not move the state)."""
    rows = []
    for s in seeds:
        env.reset(seed=int(s))
        rows.append(env.data.qpos.copy())
    return dict(seeds=np.asarray(seeds, np.int64), qpos=np.stack(rows))


def parkour_envlogic_vectors(env, n, seed=4321, max_contacts=14):
    """Random synthetic MjData-like states -> the reference's own step() (parkour_env.py:356-394)
    with physics stubbed out: clip + ctrl write, dynamic obstacles, obs, reward, termination,
    truncation, counters and info."""
    c = env.model._c
    rng = np.random.default_rng(seed)
    keys = _parkour_keys(env)
    torso = env.torso_id
    feet = list(env.foot_ids.values())
    nb = c.nbody
    cols = {k: [] for k in ["qpos", "qvel", "xpos", "ncon", "con_geom", "action", "ctrl_in", "last_position_in",
                            "max_progress_in", "reached_in", "fall_count_in", "stuck_in", "step_count_in",
                            "episode_reward_in",
                            "obs", "reward", "terminated", "truncated", "ctrl_out", "last_position_out",
                            "max_progress_out", "reached_out", "fall_count_out", "stuck_out", "step_count_out",
                            "episode_reward_out", "course_completion"]}
    for i in range(n):
        d = env.data
        d.reset()
        scen = i % 10
        qpos = c.qpos0.copy()
        qpos[:] = rng.normal(scale=0.8, size=c.nq)
        q = rng.normal(size=4)
        if scen in (1, 2):
            q = np.array([rng.uniform(0.6, 1.0), *rng.normal(scale=0.3, size=3)])
        qpos[3:7] = q / np.linalg.norm(q) if scen != 3 else q  # scen 3: unnormalised
        d.qpos[:] = qpos
        d.qvel[:] = rng.normal(scale=rng.choice([0.5, 5.0, 30.0]), size=c.nv)
        xpos = rng.uniform(-1, 1, (nb, 3))
        x = float(rng.choice([rng.uniform(-5, 105), rng.choice([15, 30, 45, 60, 75, 90, 98]) + rng.uniform(-0.02, 0.02),
                              rng.choice(PARKOUR_OBSTACLES) + 2 + rng.uniform(-0.02, 0.02)]))
        xpos[torso] = [x, rng.choice([rng.uniform(-11, 11), rng.uniform(-1, 1)]),
                       rng.choice([rng.uniform(0.1, 0.25), rng.uniform(0.1, 0.8)])]
        for f in feet:
            xpos[f] = xpos[torso] + rng.normal(scale=0.3, size=3)
        d.xpos[:] = xpos
        ncon = int(rng.integers(0, max_contacts + 1))
        geoms = rng.integers(0, c.ngeom, (ncon, 2))
        if scen in (4, 5, 6) and ncon:  # geom ids that equal the feet's BODY ids (quirk P2)
            for k in range(min(ncon, int(rng.integers(1, 5)))):
                geoms[k, int(rng.integers(0, 2))] = feet[int(rng.integers(0, 4))]
        d.contact = [FakeContact(g[0], g[1], 0.0, np.zeros(5)) for g in geoms]
        d.ncon = ncon
        d.ctrl[:] = rng.normal(size=c.nu)
        ctrl_in = d.ctrl.copy()
        prog = float(rng.choice([rng.uniform(-0.3, 0.3), rng.uniform(-0.012, 0.012), rng.uniform(-0.12, -0.08)]))
        env.last_position = np.array([x - prog, rng.normal(), rng.normal()])
        env.max_forward_progress = float(rng.uniform(0, 100))
        mask = int(rng.integers(0, 1 << 18)) if scen in (7, 8) else 0
        env.checkpoints_reached = {k for b, k in enumerate(keys) if (mask >> b) & 1}
        env.fall_count = int(rng.integers(0, 5))
        env.stuck_counter = int(rng.choice([0, 99, 100, 101, 999, 1000, 1001, int(rng.integers(0, 1200))]))
        env.step_count = int(rng.choice([0, 1, 5999, 6000, 6001, int(rng.integers(0, 7000))]))
        env.episode_reward = float(rng.normal(scale=1e4))
        inp = dict(qpos=qpos, qvel=d.qvel.copy(), xpos=xpos, ncon=ncon, con_geom=_pad(geoms, max_contacts, 2, -1),
                   ctrl_in=ctrl_in, last_position_in=env.last_position.copy(), max_progress_in=env.max_forward_progress,
                   reached_in=mask, fall_count_in=env.fall_count, stuck_in=env.stuck_counter,
                   step_count_in=env.step_count, episode_reward_in=env.episode_reward)
        lim = env.action_space.high
        action = (rng.uniform(-1.3, 1.3, len(lim)) * lim).astype(ACTION_DTYPE)
        obs, reward, term, trunc, info = env.step(action)
        reached = sum(1 << b for b, k in enumerate(keys) if k in env.checkpoints_reached)
        out = dict(action=action, obs=obs, reward=float(reward), terminated=bool(term), truncated=bool(trunc),
                   ctrl_out=d.ctrl.copy(), last_position_out=np.asarray(env.last_position, np.float64),
                   max_progress_out=env.max_forward_progress, reached_out=reached, fall_count_out=env.fall_count,
                   stuck_out=env.stuck_counter, step_count_out=env.step_count,
                   episode_reward_out=float(env.episode_reward), course_completion=info["course_completion"])
        assert info["checkpoints_reached"] == len(env.checkpoints_reached)
        for k, v in {**inp, **out}.items():
            cols[k].append(v)
    return {k: np.asarray(v) for k, v in cols.items()}


# ------------------------------------------------------------------------------- bipedal
def bipedal_env():
    install_stubs()
    mod = load_module(f"{REF}/bipedal_rescue_env/rescue_env.py", "ref_rescue_env2")
    return mod.BipedalRescueEnv(render_mode=None)


def bipedal_reset_vectors(env, seeds):
    """reset(seed) (rescue_env.py:347-396): qpos after _randomize_initial_state (the stub
    mj_step does not move the state)."""
    import contextlib
    import io
    rows = []
    for s in seeds:
        with contextlib.redirect_stdout(io.StringIO()):
            env.reset(seed=int(s))
        rows.append(env.data.qpos.copy())
    return dict(seeds=np.asarray(seeds, np.int64), qpos=np.stack(rows))


def bipedal_envlogic_vectors(env, n, seed=777, max_contacts=24):
    """Random synthetic MjData-like states -> the reference's own step() (rescue_env.py:416-471)
    with physics stubbed out: clip + ctrl, energy, victim pickup / rescue, obs, reward,
    termination, truncation, stats, and the attributes that persist across resets (B3)."""
    import contextlib
    import io
    c = env.model._c
    rng = np.random.default_rng(seed)
    torso, victims = env.torso_id, env.victim_ids
    nb = c.nbody
    cols = {}

    def put(k, v):
        cols.setdefault(k, []).append(v)
    for i in range(n):
        d = env.data
        d.reset()
        scen = i % 12
        d.qpos[:] = rng.normal(scale=0.7, size=c.nq)
        d.qvel[:] = rng.normal(scale=rng.choice([0.5, 5.0]), size=c.nv)
        xpos = rng.uniform(-3, 3, (nb, 3))
        rx, ry = rng.choice([rng.uniform(-27, 27), rng.uniform(-6, 6), rng.uniform(17, 23)]), rng.uniform(-27, 27) \
            if scen in (0, 1) else rng.uniform(-4, 4)
        xpos[torso] = [rx, ry, rng.uniform(0.3, 2.5)]
        for k, v in enumerate(victims):
            if scen in (2, 3, 4) and k < 3:  # victims near the robot: pickups
                xpos[v] = xpos[torso] + [rng.uniform(-1.0, 1.0), rng.uniform(-1.0, 1.0), rng.uniform(-1, 0)]
            else:
                xpos[v] = [rng.uniform(-12, 12), rng.uniform(-12, 12), rng.uniform(0, 1)]
        if scen in (5, 6):  # in the safe zone (20, 0), radius 3
            xpos[torso][:2] = [20 + rng.uniform(-3.2, 3.2), rng.uniform(-3.2, 3.2)]
        if scen == 7:  # in a fire zone
            xpos[torso][:2] = [-5 + rng.uniform(-1.6, 1.6), -3 + rng.uniform(-1.6, 1.6)]
        d.xpos[:] = xpos
        q = rng.normal(size=4)
        if scen % 3:
            q = np.array([1.0, *rng.normal(scale=0.3, size=3)])
        d.xquat[:] = np.tile(q / np.linalg.norm(q), (nb, 1))
        ncon = int(rng.integers(0, max_contacts + 1))
        dists = rng.choice([rng.uniform(-0.05, 0.01), rng.uniform(-0.3, 0.01)], size=ncon)
        d.contact = [FakeContact(0, 1, dd, np.zeros(5)) for dd in dists]
        d.ncon = ncon
        perm = list(rng.permutation(5))
        nres = int(rng.integers(0, 6)) if scen != 8 else 4
        rescued = [int(x) for x in perm[:nres]]
        rest = perm[nres:]
        ncar = int(rng.integers(0, min(3, len(rest)) + 1))
        carried = [int(x) for x in rest[:ncar]]
        env.victims_rescued = list(rescued)
        env.victims_carried = list(carried)
        env.carrying_victims = bool(carried) if scen != 9 else bool(rng.random() < 0.5)
        env.current_step = int(rng.choice([0, 1, 9998, 9999, 10000, int(rng.integers(0, 10000))]))
        env.current_energy = np.float32(rng.choice([1000.0, rng.uniform(0.0, 3.0), rng.uniform(0, 1000)])) \
            if scen != 10 else 1000.0
        env.closest_victim_distance = float(rng.choice([np.inf, rng.uniform(0, 15)]))
        persist = {}
        for k, gen in (("_prev_rescued_count", lambda: int(rng.integers(0, 6))),
                       ("_prev_carried_count", lambda: int(rng.integers(0, 3))),
                       ("_prev_safe_zone_distance", lambda: float(rng.uniform(0, 30))),
                       ("_fall_timer", lambda: int(rng.choice([0, 99, 100, 101, int(rng.integers(0, 200))])))):
            if rng.random() < 0.75:
                setattr(env, k, gen())
                persist[k] = getattr(env, k)
            elif hasattr(env, k):
                delattr(env, k)
        es = env.episode_stats
        es.update(victims_rescued=len(rescued), distance_traveled=float(rng.uniform(0, 50)),
                  energy_used=np.float32(rng.uniform(0, 100)), falls=int(rng.integers(0, 10)),
                  collisions=int(rng.integers(0, 10)),
                  time_to_first_rescue=None if rng.random() < 0.5 else float(rng.uniform(0, 100)))
        env.prev_robot_pos = xpos[torso] + rng.normal(scale=0.2, size=3)
        inp = dict(qpos=d.qpos.copy(), qvel=d.qvel.copy(), xpos=xpos, xquat=d.xquat.copy(), ncon=ncon,
                   con_dist=_pad(dists, max_contacts), rescued_mask_in=sum(1 << v for v in rescued),
                   carried_in=_pad(np.array(carried, dtype=np.float64), 5, None, -1.0),
                   rescued_in=_pad(np.array(rescued, dtype=np.float64), 5, None, -1.0),
                   carrying_in=env.carrying_victims, current_step_in=env.current_step,
                   energy_in=float(env.current_energy), closest_in=env.closest_victim_distance,
                   prev_rescued_in=persist.get("_prev_rescued_count", -1),
                   prev_carried_in=persist.get("_prev_carried_count", -1),
                   prev_sz_in=persist.get("_prev_safe_zone_distance", np.nan),
                   fall_timer_in=persist.get("_fall_timer", -1),
                   stats_in=np.array([es["victims_rescued"], es["distance_traveled"], es["energy_used"],
                                      np.nan if es["time_to_first_rescue"] is None else es["time_to_first_rescue"],
                                      es["falls"], es["collisions"]], dtype=np.float64),
                   prev_robot_pos_in=env.prev_robot_pos.copy())
        lim = env.action_space.high
        action = (rng.uniform(-1.3, 1.3, len(lim)) * lim * rng.choice([1.0, 0.01])).astype(ACTION_DTYPE)
        with contextlib.redirect_stdout(io.StringIO()):
            obs, reward, term, trunc, info = env.step(action)
        es = env.episode_stats
        out = dict(action=action, obs=obs, reward=float(reward), terminated=bool(term), truncated=bool(trunc),
                   ctrl_out=d.ctrl.copy(), rescued_out=_pad(np.array(env.victims_rescued, dtype=np.float64), 5, None, -1),
                   carried_out=_pad(np.array(env.victims_carried, dtype=np.float64), 5, None, -1),
                   carrying_out=env.carrying_victims, current_step_out=env.current_step,
                   energy_out=float(env.current_energy), energy_is_f32=isinstance(env.current_energy, np.float32),
                   closest_out=float(env.closest_victim_distance),
                   prev_rescued_out=getattr(env, "_prev_rescued_count", -1),
                   prev_carried_out=getattr(env, "_prev_carried_count", -1),
                   prev_sz_out=getattr(env, "_prev_safe_zone_distance", np.nan),
                   fall_timer_out=getattr(env, "_fall_timer", -1),
                   stats_out=np.array([es["victims_rescued"], es["distance_traveled"], es["energy_used"],
                                       np.nan if es["time_to_first_rescue"] is None else es["time_to_first_rescue"],
                                       es["falls"], es["collisions"]], dtype=np.float64),
                   prev_robot_pos_out=env.prev_robot_pos.copy(), upright=bool(info["robot_upright"]))
        for k, v in {**inp, **out}.items():
            put(k, v)
    return {k: np.asarray(v) for k, v in cols.items()}


# ------------------------------------------------------------------------------- dancing
MOVES = ['basic_step', 'spin', 'jump', 'moonwalk', 'robot_wave', 'freeze', 'hip_hop_bounce', 'breakdance_toprock',
         'salsa_basic', 'ballet_pirouette']   # dancing_env.py:57-68 key order


def dancing_env():
    import contextlib
    import io
    install_stubs()
    mod = load_module(f"{REF}/humanoid_dancing_env/dancing_env.py", "ref_dancing_env2")
    with contextlib.redirect_stdout(io.StringIO()):
        return mod.HumanoidDancingEnv(render_mode=None)


def _dance_state(env):
    es = env.episode_stats
    return dict(current_step=env.current_step, t_beat=float(env.time_since_last_beat), beat_count=env.beat_count,
                measure=env.current_measure, disco=float(env.disco_ball_rotation),
                spotlight=np.asarray(env.spotlight_position, dtype=np.float64).copy(),
                combo=float(env.combo_multiplier), score=float(env.performance_score),
                move_idx=env.current_move_idx, move_start=float(env.move_start_time),
                hist=_pad(np.array([MOVES.index(x) for x in env.move_history[-3:]], dtype=np.float64), 3, None, -1.0),
                hist_len=len(env.move_history), crowd=float(env.crowd_excitement), applause=float(env.applause_level),
                stats=np.array([es['energy_used'], es['time_on_beat'], es['longest_combo'], es['crowd_rating'],
                                es['total_score']], dtype=np.float64),
                fall_start=getattr(env, 'fall_start_step', 0), fall_present=hasattr(env, 'fall_start_step'),
                prev_jvel=np.asarray(env.prev_joint_vel, dtype=np.float64).copy())


def dancing_reset_vectors(env, seeds):
    """reset(seed) (dancing_env.py:763-831): the 20-move sequence draws and the initial pose
    (the stub mj_step does not move the state)."""
    rows = []
    for s in seeds:
        env.reset(seed=int(s))
        rows.append(dict(qpos=env.data.qpos.copy(),
                         moves=np.array([MOVES.index(d['move']) for d in env.dance_sequence], dtype=np.int64),
                         durations=np.array([d['duration'] for d in env.dance_sequence])))
    return dict(seeds=np.asarray(seeds, np.int64), qpos=np.stack([r["qpos"] for r in rows]),
                moves=np.stack([r["moves"] for r in rows]), durations=np.stack([r["durations"] for r in rows]))


def dancing_envlogic_vectors(env, n, seed=999, max_contacts=16):
    """Random synthetic MjData-like states -> the reference's own step() (dancing_env.py:833-894)
    with physics stubbed out: clip + ctrl, rhythm, spotlight, obs, reward, termination, stats,
    crowd, move transitions and the fall_start_step attribute that survives reset."""
    c = env.model._c
    rng = np.random.default_rng(seed)
    torso = env.torso_id
    nb = c.nbody
    cand = c.pair_geom
    cols = {}

    def put(k, v):
        cols.setdefault(k, []).append(v)
    env.reset(seed=0)
    for i in range(n):
        d = env.data
        scen = i % 10
        d.qpos[:] = rng.normal(scale=rng.choice([0.3, 1.5]), size=c.nq)
        d.qvel[:] = rng.normal(scale=rng.choice([0.05, 0.3, 3.0]), size=c.nv)
        d.xpos[:] = rng.uniform(-3, 3, (nb, 3))
        d.xpos[torso] = [rng.normal(scale=0.2), rng.normal(scale=0.2), 1.8] if scen != 9 else \
            [rng.uniform(-20, 20), rng.uniform(-20, 20), rng.uniform(-1, 6)]
        q = rng.normal(size=4)
        if scen % 3:
            q = np.array([1.0, *rng.normal(scale=0.3, size=3)])
        d.xquat[:] = np.tile(q / np.linalg.norm(q), (nb, 1))
        d.subtree_com[:] = rng.uniform(-12, 12, (nb, 3))
        ncon = int(rng.integers(0, max_contacts + 1))
        pairs = []
        for _ in range(ncon):
            if rng.random() < 0.4:
                pairs.append((int(rng.choice([0, 1])), int(rng.choice([env.right_foot_id, env.left_foot_id]))))
            else:
                g1, g2 = cand[int(rng.integers(0, len(cand)))]
                pairs.append((int(g1), int(g2)))
        d.contact = [FakeContact(g1, g2, rng.uniform(-0.05, 0.01), np.zeros(5)) for g1, g2 in pairs]
        d.ncon = ncon
        env.current_step = int(rng.choice([0, 1, 3599, int(rng.integers(0, 3600))]))
        env.time_since_last_beat = float(rng.choice([rng.uniform(0, 0.5), rng.uniform(0.47, 0.5), rng.uniform(0, 0.06),
                                                     rng.uniform(0.08, 0.12), rng.uniform(0.38, 0.42)]))
        env.beat_count = int(rng.integers(0, 500))
        env.current_measure = env.beat_count // 4
        env.disco_ball_rotation = float(rng.uniform(0, 6.3))
        env.spotlight_position = np.array([rng.normal(), rng.normal(), rng.uniform(4, 6)])
        env.combo_multiplier = float(rng.choice([1.0, 10.0, rng.uniform(1, 10), 1.02]))
        env.performance_score = float(rng.normal(scale=1000))
        env.dance_sequence = [{'move': MOVES[int(rng.integers(0, 10))], 'duration': float(rng.uniform(1, 3))}
                              for _ in range(20)]
        env.current_move_idx = int(rng.choice([0, 19, 20, int(rng.integers(0, 21))]))
        now = env.current_step * env.dt
        env.move_start_time = float(now - rng.choice([rng.uniform(0, 3.5), rng.uniform(0, 0.2)]))
        hl = int(rng.integers(0, 6))
        env.move_history = [MOVES[int(rng.integers(0, 10))] if rng.random() < 0.7 else MOVES[k % 10] for k in range(hl)]
        env.crowd_excitement = float(rng.choice([0.5, rng.uniform(0, 1), 0.9999, 0.0]))
        env.applause_level = env.crowd_excitement * 100.0
        es = env.episode_stats
        es.update(energy_used=float(rng.choice([0.0, rng.uniform(0, 1500)])), time_on_beat=float(rng.uniform(0, 10)),
                  longest_combo=int(rng.integers(0, 11)), crowd_rating=float(rng.uniform(0, 1)),
                  total_score=float(rng.normal(scale=100)))
        if rng.random() < 0.5:
            env.fall_start_step = int(env.current_step - rng.choice([0, 119, 120, 121, int(rng.integers(0, 300))]))
        elif hasattr(env, 'fall_start_step'):
            delattr(env, 'fall_start_step')
        env.prev_joint_vel = d.qvel[6:] + rng.normal(scale=rng.choice([0.01, 0.3, 3.0]), size=c.nv - 6)
        inp = {k + "_in": v for k, v in _dance_state(env).items()}
        inp.update(qpos=d.qpos.copy(), qvel=d.qvel.copy(), xpos=d.xpos.copy(), xquat=d.xquat.copy(),
                   subtree_com=d.subtree_com.copy(), ncon=ncon,
                   con_geom=_pad(np.array(pairs, dtype=np.float64).reshape(-1, 2), max_contacts, 2, -1.0),
                   moves=np.array([MOVES.index(x['move']) for x in env.dance_sequence], dtype=np.int64),
                   durations=np.array([x['duration'] for x in env.dance_sequence]))
        lim = env.action_space.high
        action = (rng.uniform(-1.3, 1.3, len(lim)) * lim * rng.choice([1.0, 0.01, 0.1])).astype(ACTION_DTYPE)
        obs, reward, term, trunc, info = env.step(action)
        out = {k + "_out": v for k, v in _dance_state(env).items()}
        out.update(action=action, obs=obs, reward=float(reward), reward_is_f64=isinstance(reward, np.float64),
                   terminated=bool(term), truncated=bool(trunc), ctrl_out=d.ctrl.copy())
        for k, v in {**inp, **out}.items():
            put(k, v)
    return {k: np.asarray(v) for k, v in cols.items()}


# ------------------------------------------------------------------------------- martial arts
def martial_xml():
    """The composed scene from the reference's own generator (martial_arts_env.py:150-381),
    written to a scratch directory (the reference tree is read-only)."""
    import tempfile
    mod = load_module(f"{REF}/humanoid_martial_arts_env/martial_arts_env.py", "ref_martial_env")
    o = object.__new__(mod.HumanoidMartialArtsEnv)
    d = tempfile.mkdtemp()
    mod.HumanoidMartialArtsEnv._generate_xml_files(o, d)
    with open(os.path.join(d, "martial_arts_scene.xml")) as f:
        return mod, f.read()


def martial_env():
    install_stubs()
    mod, xml = martial_xml()
    cls = mod.HumanoidMartialArtsEnv
    # the constructor reads the scene from its own assets directory; hand it the generated string
    orig = cls._load_xml_models
    cls._load_xml_models = lambda self: setattr(self, "xml_string", xml)
    try:
        env = cls(render_mode=None)
    finally:
        cls._load_xml_models = orig
    return env, xml


def martial_reset_vectors(env, seeds):
    """reset(seed) (martial_arts_env.py:442-487): two uniform draws move qpos[0:2] (dummy1's free
    joint, quirk M1), then mj_forward. A seeded reset followed by an unseeded one continues the
    same stream."""
    rows = []
    for s in seeds:
        env.reset(seed=int(s))
        q1 = env.data.qpos.copy()
        env.reset()
        q2 = env.data.qpos.copy()
        rows.append((q1, q2))
    return dict(seeds=np.asarray(seeds, np.int64), qpos_first=np.stack([r[0] for r in rows]),
                qpos_second=np.stack([r[1] for r in rows]))


def martial_envlogic_vectors(env, n, seed=2468):
    """Random synthetic states -> the reference's step() with mj_step stubbed out: clip, ctrl,
    observation, reward (numpy promotion), termination, truncation, stats, the stance timer and
    the prev_torso_pos attribute that survives reset (quirk M3)."""
    c = env.model._c
    rng = np.random.default_rng(seed)
    nb, nq, nv, nu = c.nbody, c.nq, c.nv, c.nu
    torso = env.torso_idx
    out = {k: [] for k in ("qpos", "qvel", "xpos", "xquat", "cvel", "action", "current_step", "stance_in",
                           "stats_in", "has_prev", "prev_torso_in", "ctrl", "obs", "reward", "reward_kind",
                           "terminated", "truncated", "stance_out", "stats_out", "has_prev_out", "prev_torso_out")}
    keys = ['techniques_performed', 'successful_combos', 'balance_maintained', 'max_power_generated',
            'total_distance_moved', 'falls']
    for i in range(n):
        d = env.data
        d.reset()
        d.qpos[:] = c.qpos0 + rng.normal(scale=0.5, size=nq)
        d.qvel[:] = rng.normal(scale=rng.choice([0.3, 2.0, 8.0]), size=nv)
        xpos = rng.uniform(-3, 3, (nb, 3))
        scen = i % 6
        xpos[torso] = [rng.uniform(-6, 6), rng.uniform(-6, 6), rng.uniform(0.2, 2.2)]
        if scen == 0:  # near dummy 1
            xpos[torso, :2] = xpos[env.dummy1_idx, :2] + rng.uniform(-1.5, 1.5, 2)
        elif scen == 1:  # standing tall
            xpos[torso, 2] = rng.uniform(1.6, 2.0)
        d.xpos[:] = xpos
        q = rng.normal(size=(nb, 4))
        d.xquat[:] = q / np.linalg.norm(q, axis=1, keepdims=True)
        d.cvel[:] = rng.normal(scale=rng.choice([0.2, 1.5, 4.0]), size=(nb, 6))
        if scen == 2:  # calm torso rotation -> stance bonus
            d.cvel[torso, 3:] = rng.normal(scale=0.1, size=3)
        env.current_step = int(rng.choice([0, 1, 2, 100, 5998, 5999, int(rng.integers(0, 7000))]))
        env.stance_stability_time = float(rng.choice([0.0, rng.uniform(0, 20)]))
        st = [int(rng.integers(0, 50)), 0, 0, 0, float(rng.uniform(0, 30)), int(rng.integers(0, 3))]
        env.episode_stats = dict(zip(keys, st))
        has_prev = bool(rng.random() < 0.7)
        prev = xpos[torso] + rng.normal(scale=0.2, size=3)
        if has_prev:
            env.prev_torso_pos = prev.copy()
        elif hasattr(env, "prev_torso_pos"):
            del env.prev_torso_pos
        action = rng.uniform(-1.5, 1.5, nu).astype(ACTION_DTYPE)
        stance_in, stats_in, step_in = env.stance_stability_time, [env.episode_stats[k] for k in keys], env.current_step
        obs, reward, term, trunc, info = env.step(action)
        vals = dict(qpos=d.qpos.copy(), qvel=d.qvel.copy(), xpos=xpos, xquat=d.xquat.copy(), cvel=d.cvel.copy(),
                    action=action, current_step=step_in, stance_in=stance_in,
                    stats_in=np.array(stats_in, np.float64), has_prev=has_prev, prev_torso_in=prev,
                    ctrl=d.ctrl.copy(), obs=obs, reward=float(reward),
                    reward_kind={float: 0, np.float64: 1, np.float32: 2}[type(reward)],
                    terminated=bool(term), truncated=bool(trunc), stance_out=env.stance_stability_time,
                    stats_out=np.array([env.episode_stats[k] for k in keys], np.float64),
                    has_prev_out=hasattr(env, "prev_torso_pos"),
                    prev_torso_out=env.prev_torso_pos.copy() if hasattr(env, "prev_torso_pos") else np.zeros(3))
        for k in out:
            out[k].append(vals[k])
    return {k: np.asarray(v) for k, v in out.items()}


def main_martial():
    env, xml = martial_env()
    os.makedirs(f"{HERE}/xml", exist_ok=True)
    with open(f"{HERE}/xml/humanoid_martial_arts.xml", "w") as f:
        f.write(xml)
    with open(f"{REPO}/mujoco_gymnasium_environments_amd/assets/humanoid_martial_arts.xml", "w") as f:
        f.write(xml)
    np.savez_compressed(f"{HERE}/martial_reset.npz", **martial_reset_vectors(env, list(range(0, 40)) + [31337]))
    np.savez_compressed(f"{HERE}/martial_envlogic.npz", **martial_envlogic_vectors(env, 600))


# ------------------------------------------------------------------------------- construction / assembly
class _Loaded(Exception):
    """Raised by the MjData stub once a constructor has handed its model to MuJoCo."""


def captured_model_xml(path, module_name, cls_name, **ctor_kw):
    """Run the reference constructor until it calls MjModel.from_xml_string / from_xml_path and
    return the MJCF it passes (the model input of the task, as MuJoCo would receive it)."""
    import contextlib
    import io
    import tempfile
    install_stubs()
    mj = sys.modules["mujoco"]
    seen = {}

    class MjModel:
        @staticmethod
        def from_xml_string(xml):
            seen["xml"] = xml
            return FakeModel(mjcf.compile_xml(xml))

        @staticmethod
        def from_xml_path(p):
            with open(p) as f:
                return MjModel.from_xml_string(f.read())

    def mjdata(m):
        raise _Loaded()
    mj.MjModel, mj.MjData = MjModel, mjdata
    mod = load_module(path, module_name)
    cls = getattr(mod, cls_name)
    if hasattr(cls, "_generate_xml_files"):
        # generators write next to the module; point them at a scratch directory instead
        d = tempfile.mkdtemp()
        gen = cls._generate_xml_files
        cls._load_xml_models = lambda self: (gen(self, d), setattr(
            self, "xml_string", open(os.path.join(d, "construction_site.xml")).read()))
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            cls(**ctor_kw)
    except _Loaded:
        pass
    return seen["xml"]


def main_models():
    """Composed models of the two tasks not simulated yet (construction: _generate_site_xml,
    construction_env.py:177-495; assembly: complete_model.xml loaded at assembly_env.py:46-54)."""
    os.makedirs(f"{HERE}/xml", exist_ok=True)
    xml = captured_model_xml(f"{REF}/humanoid_construction_env/construction_env.py", "ref_construction_env",
                             "HumanoidConstructionEnv", render_mode=None)
    with open(f"{HERE}/xml/humanoid_construction.xml", "w") as f:
        f.write(xml)
    xml = captured_model_xml(f"{REF}/robotic_arm_assembly_env/assembly_env.py", "ref_assembly_env",
                             "RoboticArmAssemblyEnv", render_mode=None)
    with open(f"{HERE}/xml/robotic_arm_assembly.xml", "w") as f:
        f.write(xml)


def assembly_env():
    """RoboticArmAssemblyEnv built by the reference constructor on the stubs (its reset() runs the
    10 settle mj_steps as stub no-ops), complete_model.xml read from the reference's assets."""
    import contextlib
    import io
    install_stubs()
    mj = sys.modules["mujoco"]

    class MjModel:
        @staticmethod
        def from_xml_path(p):
            with open(p) as f:
                return FakeModel(mjcf.compile_xml(f.read()))
    mj.MjModel = MjModel
    mod = load_module(f"{REF}/robotic_arm_assembly_env/assembly_env.py", "ref_assembly_env")
    with contextlib.redirect_stdout(io.StringIO()):
        env = mod.RoboticArmAssemblyEnv(render_mode=None)
    return env


def _assembly_site(c, xpos, xquat):
    """site_xpos of every site from body frames (xmat = quat2mat(xquat)); the logic only reads
    ee_site (assembly_env.py:437-439)."""
    out = np.zeros((len(c.site_names), 3))
    for s in range(len(c.site_names)):
        b = int(c.site_bodyid[s])
        R = mjcf.quat2mat(np.asarray(xquat[b], np.float64))
        out[s] = xpos[b] + R @ c.site_pos[s]
    return out


def assembly_reset_vectors(env):
    """reset() (assembly_env.py:162-218): mj_resetData, the home pose into qpos[0:7], every
    component at its bin position with an identity quaternion; tracking state cleared. The 10
    settle steps are stub no-ops here, so qpos is the state those steps start from."""
    env.data.qpos[:] = 7.0  # garbage that mj_resetData must clear
    obs, info = env.reset(seed=5)
    return dict(qpos=env.data.qpos.copy(), nstep=np.int64(getattr(env.data, "nstep", 0)),
                obs=obs, phase=np.int64(('idle', 'pickup', 'transport', 'align', 'insert').index(info['task_phase'])))


def assembly_envlogic_vectors(env, n, seed=8642, max_contacts=12):
    """Random synthetic states -> the reference's step() with mj_step stubbed out: clip, ctrl,
    gripper-contact task state, reward, termination, truncation, observation, tracking state."""
    c = env.model._c
    rng = np.random.default_rng(seed)
    seq = env.assembly_sequence
    status_names = ['in_bin', 'held', 'assembled', 'dropped']
    gnames = [c.id2name("geom", g) for g in range(c.ngeom)]
    pads = [g for g, nme in enumerate(gnames) if nme and 'gripper' in nme and 'pad' in nme]
    comp_geoms = [g for g, nme in enumerate(gnames) if nme and any(s in nme for s in seq)]
    other = [g for g in range(c.ngeom) if g not in pads and g not in comp_geoms]
    bodies = [c.name2id("body", s) for s in seq]
    targets = env.component_targets
    lo = np.array([-3.14, -2.36, -2.97, -3.14, -2.09, -3.14, -3.14])
    hi = np.array([3.14, 0.78, 2.97, 3.14, 2.09, 3.14, 3.14])
    cols = {k: [] for k in ("qpos", "qvel", "xpos", "xquat", "site_xpos", "ncon", "con_geom", "con_dist", "action",
                            "step_in", "held_in", "phase_in", "status_in", "progress_in", "cum_in", "ctrl", "obs",
                            "reward", "terminated", "truncated", "step_out", "held_out", "phase_out", "status_out",
                            "progress_out", "cum_out")}
    for i in range(n):
        d = env.data
        d.reset()
        scen = i % 8
        q = c.qpos0 + rng.normal(scale=0.3, size=c.nq)
        q[0:7] = rng.uniform(lo * 0.9, hi * 0.9)
        if scen == 0:  # one arm joint just past (or just inside) its 0.95 termination bound
            j = int(rng.integers(0, 7))
            q[j] = (hi[j] if rng.random() < 0.5 else lo[j]) * 0.95 * (1 + rng.choice([-1e-3, 1e-3]) * np.sign(hi[j]))
        d.qpos[:] = q
        d.qvel[:] = rng.normal(scale=rng.choice([0.01, 0.3, 3.0]), size=c.nv)
        xpos = rng.uniform(-1, 1, (c.nbody, 3))
        held_in = None if rng.random() < 0.4 else seq[int(rng.integers(0, 9))]
        if held_in is not None and scen in (1, 2, 3):
            # the held component near its target: inside the 2 mm assembly tolerance, inside
            # the 5 cm precision band, or just outside it
            r = {1: 0.0015, 2: 0.03, 3: 0.051}[scen] * rng.uniform(0.2, 1.0)
            v = rng.normal(size=3)
            xpos[bodies[seq.index(held_in)]] = np.asarray(targets[held_in]) + r * v / np.linalg.norm(v)
        d.xpos[:] = xpos
        qq = rng.normal(size=(c.nbody, 4))
        d.xquat[:] = qq / np.linalg.norm(qq, axis=1, keepdims=True)
        d.site_xpos = _assembly_site(c, d.xpos, d.xquat)
        nc = int(rng.integers(0, max_contacts + 1)) if scen != 4 else 0
        cons = []
        for k in range(nc):
            u = rng.random()
            if u < 0.35:
                g1, g2 = int(rng.choice(pads)), int(rng.choice(comp_geoms))
            elif u < 0.5:
                g1, g2 = int(rng.choice(pads)), int(rng.choice(other))
            else:
                g1, g2 = int(rng.integers(0, c.ngeom)), int(rng.integers(0, c.ngeom))
            if rng.random() < 0.5:
                g1, g2 = g2, g1
            dist = float(rng.choice([rng.uniform(-0.002, 0.001), rng.uniform(-0.02, 0), rng.uniform(-0.2, 0)]))
            cons.append(FakeContact(g1, g2, dist, [1, 0.5, 0.5]))
        if scen == 5 and cons:
            # one component only: the deterministic case of list(set(...))[0]
            cg = int(rng.choice(comp_geoms))
            for cn in cons:
                if cn.geom1 in comp_geoms and cn.geom2 in pads:
                    cn.geom1 = cg
                elif cn.geom2 in comp_geoms and cn.geom1 in pads:
                    cn.geom2 = cg
        # keep only states whose touched-component set has at most one member (quirk A3: with
        # two or more the reference's pick depends on PYTHONHASHSEED)
        touched = set()
        for cn in cons:
            for ga, gb in ((cn.geom1, cn.geom2), (cn.geom2, cn.geom1)):
                if ga in pads:
                    for s in seq:
                        if gnames[gb] and s in gnames[gb]:
                            touched.add(s)
                            break
                    break
        if len(touched) > 1:
            cons = [cn for cn in cons if not (cn.geom1 in pads or cn.geom2 in pads)]
        d.contact = cons
        d.ncon = len(cons)
        env.step_count = int(rng.choice([0, 1, 7, 149998, 149999, int(rng.integers(0, 200000))]))
        env.held_component = held_in
        env.task_phase = ('idle', 'pickup', 'transport', 'align', 'insert')[int(rng.integers(0, 5))]
        prog = [bool(rng.random() < (0.97 if scen == 6 else 0.3)) for _ in seq]
        env.assembly_progress = dict(zip(seq, prog))
        st = [status_names[int(rng.integers(0, 4))] for _ in seq]
        if held_in is not None:
            st[seq.index(held_in)] = 'held'
        env.component_status = dict(zip(seq, st))
        env.cumulative_reward = float(rng.choice([0.0, rng.normal(scale=1e4)]))
        action = (rng.uniform(-3, 3, 9) * np.array([1] * 7 + [50, 30])).astype(ACTION_DTYPE)
        snap = dict(qpos=d.qpos.copy(), qvel=d.qvel.copy(), xpos=d.xpos.copy(), xquat=d.xquat.copy(),
                    site_xpos=d.site_xpos.copy(), ncon=len(cons),
                    con_geom=_pad(np.array([[cn.geom1, cn.geom2] for cn in cons], np.int64).reshape(-1, 2),
                                  max_contacts, 2, -1),
                    con_dist=_pad(np.array([cn.dist for cn in cons]), max_contacts),
                    action=action, step_in=env.step_count,
                    held_in=-1 if held_in is None else seq.index(held_in),
                    phase_in=('idle', 'pickup', 'transport', 'align', 'insert').index(env.task_phase),
                    status_in=np.array([status_names.index(s) for s in st]), progress_in=np.array(prog),
                    cum_in=env.cumulative_reward)
        obs, reward, term, trunc, info = env.step(action)
        assert isinstance(reward, np.float64), type(reward)
        out = dict(ctrl=d.ctrl.copy(), obs=obs, reward=float(reward), terminated=bool(term), truncated=bool(trunc),
                   step_out=env.step_count,
                   held_out=-1 if env.held_component is None else seq.index(env.held_component),
                   phase_out=('idle', 'pickup', 'transport', 'align', 'insert').index(env.task_phase),
                   status_out=np.array([status_names.index(env.component_status[s]) for s in seq]),
                   progress_out=np.array([env.assembly_progress[s] for s in seq]),
                   cum_out=float(env.cumulative_reward))
        for k, v in {**snap, **out}.items():
            cols[k].append(v)
    return {k: np.asarray(v) for k, v in cols.items()}


def main_assembly():
    env = assembly_env()
    np.savez_compressed(f"{HERE}/assembly_reset.npz", **assembly_reset_vectors(env))
    np.savez_compressed(f"{HERE}/assembly_envlogic.npz", **assembly_envlogic_vectors(env, 600))


# ------------------------------------------------------------------------------- construction
def construction_env():
    """HumanoidConstructionEnv built by the reference constructor on the stubs, its scene being
    the composed construction_site.xml captured in tests/golden/xml (construction_env.py:135-175).
    gymnasium's Env.np_random is a property over _np_random (gymnasium/core.py); the stub gets
    the same property here so seed() and reset(seed=...) drive one generator, as in gymnasium."""
    import contextlib
    import io
    install_stubs()
    mod = load_module(f"{REF}/humanoid_construction_env/construction_env.py", "ref_construction_env")
    cls = mod.HumanoidConstructionEnv
    with open(f"{HERE}/xml/humanoid_construction.xml") as f:
        xml = f.read()
    cls._load_xml_models = lambda self: setattr(self, "xml_string", xml)
    cls.np_random = property(lambda self: self._np_random, lambda self, v: setattr(self, "_np_random", v))
    with contextlib.redirect_stdout(io.StringIO()):
        env = cls(render_mode=None)
    return env


CONSTRUCTION_TASKS = ('stack_blocks', 'operate_crane', 'transport_material', 'build_structure')


def construction_reset_vectors(env, seeds):
    """reset(seed) then an unseeded reset (construction_env.py:547-584): mj_resetData, the task
    choice and three weather draws from the env generator, the initial observation."""
    cols = {k: [] for k in ("seeds", "task", "weather", "obs", "task2", "weather2", "obs2")}
    for s in seeds:
        env.data.qpos[:] = 3.0  # garbage that mj_resetData must clear
        obs, info = env.reset(seed=int(s))
        w = [env.wind_strength, env.rain_intensity, env.temperature]
        obs2, info2 = env.reset()
        cols["seeds"].append(int(s))
        cols["task"].append(CONSTRUCTION_TASKS.index(info["task"]))
        cols["weather"].append(w)
        cols["obs"].append(obs)
        cols["task2"].append(CONSTRUCTION_TASKS.index(info2["task"]))
        cols["weather2"].append([env.wind_strength, env.rain_intensity, env.temperature])
        cols["obs2"].append(obs2)
    return {k: np.asarray(v) for k, v in cols.items()}


def construction_envlogic_vectors(env, n, seed=1357):
    """Random synthetic states -> the reference's step() with mj_step stubbed out: clip, ctrl,
    task progress, reward (numpy promotion: the float32 energy term makes it np.float32),
    termination (fall / task complete / safety), truncation at 3000, observation, stats."""
    c = env.model._c
    rng = np.random.default_rng(seed)
    hid = env.humanoid_id
    cols = {k: [] for k in ("qpos", "qvel", "torso_z", "task", "blocks", "violations", "weather", "step_in",
                            "progress_in", "completed_in", "total_in", "action", "ctrl", "obs", "reward",
                            "reward_kind", "terminated", "truncated", "step_out", "progress_out", "completed_out",
                            "total_out")}
    for i in range(n):
        d = env.data
        d.reset()
        d.qpos[:] = c.qpos0 + rng.normal(scale=0.5, size=c.nq)
        d.qvel[:] = rng.normal(scale=rng.choice([0.1, 2.0, 10.0]), size=c.nv)
        xpos = rng.uniform(-3, 3, (c.nbody, 3))
        z = float(rng.choice([rng.uniform(0.0, 0.5), 0.5, rng.uniform(0.5, 1.0), 1.0, rng.uniform(1.0, 2.0)]))
        xpos[hid, 2] = z
        d.xpos[:] = xpos
        task = int(rng.integers(0, 4))
        env.current_task = CONSTRUCTION_TASKS[task]
        env.blocks_placed = int(rng.choice([0, 1, 4, 5, 9, 10, 12, int(rng.integers(0, 20))]))
        env.safety_violations = int(rng.choice([0, 0, 1, 3, 4, 7]))
        env.wind_strength, env.rain_intensity, env.temperature = (float(rng.uniform(0, 5)), float(rng.uniform(0, 0.5)),
                                                                  float(rng.uniform(15, 35)))
        env.current_step = int(rng.choice([0, 1, 299, 300, 499, 500, 2998, 2999, 3000, int(rng.integers(0, 3500))]))
        env.task_progress = float(rng.uniform(0, 1))
        st = dict(env.episode_stats)
        st['tasks_completed'] = int(rng.integers(0, 3))
        st['total_reward'] = float(rng.choice([0.0, rng.normal(scale=1e4)]))
        env.episode_stats = st
        scale = rng.choice([1.0, 150.0, 400.0])
        action = rng.uniform(-scale, scale, c.nu).astype(ACTION_DTYPE)
        snap = dict(qpos=d.qpos.copy(), qvel=d.qvel.copy(), torso_z=z, task=task, blocks=env.blocks_placed,
                    violations=env.safety_violations,
                    weather=[env.wind_strength, env.rain_intensity, env.temperature], step_in=env.current_step,
                    progress_in=env.task_progress, completed_in=st['tasks_completed'], total_in=st['total_reward'],
                    action=action)
        obs, reward, term, trunc, info = env.step(action)
        out = dict(ctrl=d.ctrl.copy(), obs=obs, reward=float(reward),
                   reward_kind={float: 0, np.float64: 1, np.float32: 2}[type(reward)],
                   terminated=bool(term), truncated=bool(trunc), step_out=env.current_step,
                   progress_out=float(env.task_progress), completed_out=env.episode_stats['tasks_completed'],
                   total_out=float(env.episode_stats['total_reward']))
        for k, v in {**snap, **out}.items():
            cols[k].append(v)
    return {k: np.asarray(v) for k, v in cols.items()}


def main_construction():
    env = construction_env()
    np.savez_compressed(f"{HERE}/construction_reset.npz",
                        **construction_reset_vectors(env, list(range(0, 40)) + [2024]))
    np.savez_compressed(f"{HERE}/construction_envlogic.npz", **construction_envlogic_vectors(env, 800))


def main_dancing():
    install_stubs()
    denv = dancing_env()
    np.savez_compressed(f"{HERE}/dancing_reset.npz", **dancing_reset_vectors(denv, list(range(0, 40)) + [777]))
    np.savez_compressed(f"{HERE}/dancing_envlogic.npz", **dancing_envlogic_vectors(denv, 600))


def main_f64(n=200):
    """The env-logic vectors with float64 actions (the same synthetic states, actions not rounded to
    float32): the reference's np.clip keeps a float64 policy's dtype, so ctrl, the action terms of
    the reward and the numpy types downstream follow in float64 (<task>_envlogic_f64.npz)."""
    global ACTION_DTYPE
    install_stubs()
    ACTION_DTYPE = np.float64
    np.savez_compressed(f"{HERE}/soccer_envlogic_f64.npz", **soccer_envlogic_vectors(soccer_env(), n))
    np.savez_compressed(f"{HERE}/parkour_envlogic_f64.npz", **parkour_envlogic_vectors(parkour_env(), n))
    np.savez_compressed(f"{HERE}/bipedal_envlogic_f64.npz", **bipedal_envlogic_vectors(bipedal_env(), n))
    np.savez_compressed(f"{HERE}/dancing_envlogic_f64.npz", **dancing_envlogic_vectors(dancing_env(), n))
    np.savez_compressed(f"{HERE}/martial_envlogic_f64.npz", **martial_envlogic_vectors(martial_env()[0], n))
    np.savez_compressed(f"{HERE}/assembly_envlogic_f64.npz", **assembly_envlogic_vectors(assembly_env(), n))
    np.savez_compressed(f"{HERE}/construction_envlogic_f64.npz",
                        **construction_envlogic_vectors(construction_env(), n))
    ACTION_DTYPE = np.float32
    print("float64-action fixtures written to", HERE)


def main():
    install_stubs()
    dump_xml()
    env = soccer_env()
    np.savez_compressed(f"{HERE}/soccer_reset.npz", **soccer_reset_vectors(env, list(range(0, 40)) + [12345, 2**31 - 1]))
    np.savez_compressed(f"{HERE}/soccer_envlogic.npz", **soccer_envlogic_vectors(env, 400))
    penv = parkour_env()
    np.savez_compressed(f"{HERE}/parkour_reset.npz", **parkour_reset_vectors(penv, list(range(0, 40)) + [12345]))
    np.savez_compressed(f"{HERE}/parkour_envlogic.npz", **parkour_envlogic_vectors(penv, 500))
    benv = bipedal_env()
    np.savez_compressed(f"{HERE}/bipedal_reset.npz", **bipedal_reset_vectors(benv, list(range(0, 40)) + [4242]))
    np.savez_compressed(f"{HERE}/bipedal_envlogic.npz", **bipedal_envlogic_vectors(benv, 600))
    main_dancing()
    main_martial()
    main_assembly()
    main_construction()
    print("fixtures written to", HERE)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "dancing":
        main_dancing()
    elif len(sys.argv) > 1 and sys.argv[1] == "models":
        main_models()
    elif len(sys.argv) > 1 and sys.argv[1] == "martial":
        main_martial()
    elif len(sys.argv) > 1 and sys.argv[1] == "assembly":
        main_assembly()
    elif len(sys.argv) > 1 and sys.argv[1] == "construction":
        main_construction()
    elif len(sys.argv) > 1 and sys.argv[1] == "f64":
        main_f64()
    elif len(sys.argv) > 1 and sys.argv[1] == "soccer":
        install_stubs()
        np.savez_compressed(f"{HERE}/soccer_envlogic.npz", **soccer_envlogic_vectors(soccer_env(), 400))
    else:
        main()
