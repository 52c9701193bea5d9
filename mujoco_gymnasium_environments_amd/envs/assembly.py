"""robotic_arm_assembly_env on MI355X: a batched VectorEnv and a drop-in gymnasium-style Env.

Mirrors the reference interface robotic_arm_assembly_env/assembly_env.py:
  * ``RoboticArmAssemblyEnv`` — same constructor (``render_mode``, ``config``; it resets itself,
    :95) / ``reset(seed, options)`` / ``step(action)`` / spaces / ``metadata`` / ``render`` /
    ``close`` / info dict (:474-484), batch size 1.
  * ``AssemblyVectorEnv`` — N envs on one GPU, device tensors ``[N, ...]``, same-step autoreset.
Both run one fused HIP launch per env step (libmgx.so ``mgx_assembly_step``): clip, ctrl, the
10 mj_steps of one control period (Euler, Newton, 50 iterations, tolerance 1e-10), gripper-pad
contact task state, reward, termination, observation. reset() is deterministic in the reference
(home pose, components in their bins, 10 settle steps) and runs the same way on the device.

The model is the reference's complete_model.xml (assembly_env.py:53), compiled by mjcf.py:
nq 72, nv 63, nu 9, 28 bodies, 53 geoms (boxes and cylinders), 785 filtered candidate pairs +
18 explicit condim-6 pad pairs. Under random actions it holds up to ~70 contacts / ~310
constraint rows (oracle rollouts), hence the capacities below.

Precision: the scene runs in fp64 only. Its arm base is degenerate in the reference model
(base_plate and shoulder_pan_link interpenetrate coaxially: the contact's normal Jacobian is
zero, diagApprox is zero, so R sits at mjMINVAL = 1e-15 and the rows carry ~1e17 forces,
DESIGN.md §2). In fp32 the Newton Hessian I + D B B' with D = 1e15 overflows the factorisation
and every substep ends in a bad-state reset, so ``precision="f32"`` is refused.
"""
from __future__ import annotations

import ctypes as C
import functools
import os
from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch

from .. import cabi, mjcf
from ..batch import PhysicsBatch, _ptr, stream_handle
from ..native import check, lib
from ..spaces import Box, EnvBase, policy_action

ASSET = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets",
                     "robotic_arm_assembly.xml")
EFC_CAPACITY = 384
CON_CAPACITY = 96
OBS_DIM = 110
N_ACT = 9
MAX_EPISODE_STEPS = 150000       # assembly_env.py:36
SKIP_FRAMES = 10                 # :37-39 (500 Hz / 50 Hz)
SETTLE_STEPS = 10                # :186

# assembly_env.py:47-50, :77-87, :197-207, :340-353, :411-412, :150-151
SEQUENCE = ('pcb', 'screw1', 'screw2', 'screw3', 'screw4', 'cpu', 'battery', 'cable', 'cover')
TARGETS = {'pcb': (0, 0, 0.74), 'cpu': (0, 0, 0.76), 'screw1': (-0.08, -0.06, 0.735),
           'screw2': (0.08, -0.06, 0.735), 'screw3': (-0.08, 0.06, 0.735), 'screw4': (0.08, 0.06, 0.735),
           'battery': (0.05, 0, 0.77), 'cable': (-0.05, 0, 0.77), 'cover': (0, 0, 0.79)}
BINS = {'pcb': (-0.6, 0.3, 0.76), 'cpu': (-0.6, 0, 0.76), 'screw1': (-0.6, -0.3, 0.76),
        'screw2': (-0.58, -0.3, 0.76), 'screw3': (-0.62, -0.3, 0.76), 'screw4': (-0.6, -0.28, 0.76),
        'battery': (0.6, 0.3, 0.76), 'cable': (0.6, -0.3, 0.76), 'cover': (0.6, 0, 0.76)}
HOME = (0, -0.5, 0.5, 0, 0.5, 0, 0)
PLACE_REWARD = {'pcb': 2000, 'screw1': 500, 'screw2': 500, 'screw3': 500, 'screw4': 500, 'cpu': 2000,
                'battery': 1000, 'cable': 1000, 'cover': 1000}
JOINT_LOW = (-3.14, -2.36, -2.97, -3.14, -2.09, -3.14, -3.14)
JOINT_HIGH = (3.14, 0.78, 2.97, 3.14, 2.09, 3.14, 3.14)
ACTION_LOW = (-2, -2, -2, -2, -2, -2, -2, 0, 0)
ACTION_HIGH = (2, 2, 2, 2, 2, 2, 2, 100, 50)
PHASES = ('idle', 'pickup', 'transport', 'align', 'insert')
STATUS = ('in_bin', 'held', 'assembled', 'dropped', 'damaged')


@functools.lru_cache(maxsize=None)
def assembly_model() -> mjcf.Model:
    with open(ASSET) as f:
        m = mjcf.compile_xml(f.read())
    m.efc_capacity = EFC_CAPACITY
    m.con_capacity = CON_CAPACITY
    return m


def _observation_space() -> Box:
    """assembly_env.py:97-147 (the bounds arrays as the reference fills them, float32)."""
    lo, hi = np.full(OBS_DIM, -np.inf), np.full(OBS_DIM, np.inf)
    lo[0:7], hi[0:7] = JOINT_LOW, JOINT_HIGH
    lo[7:14], hi[7:14] = -5.0, 5.0
    lo[14:16], hi[14:16] = (0, 0), (0.1, 50)
    lo[16:19], hi[16:19] = (-2, -2, 0), (2, 2, 2)
    lo[19:23], hi[19:23] = -1.0, 1.0
    lo[23:79], hi[23:79] = np.tile([-2, -2, 0, -1, -1, -1, -1], 8), np.tile([2, 2, 2, 1, 1, 1, 1], 8)
    lo[79:87], hi[79:87] = 0, 1
    lo[87:89], hi[87:89] = (0, -1), (1, 8)
    lo[89:114], hi[89:114] = 0, 1
    lo[104:110], hi[104:110] = -100, 100
    lo[108], hi[108] = 0, 100
    lo[109], hi[109] = 0, 4
    return Box(low=lo, high=hi, dtype=np.float32)


class AssemblyTables:
    """The reference's name lookups resolved once: component bodies (:324-329), per-geom pad flag
    and component tag by substring in sequence order (:299-322), the ee_site frame (:437-439),
    and the reset qpos (:167-218)."""

    def __init__(self, m: mjcf.Model, max_episode_steps: int = MAX_EPISODE_STEPS):
        self.model = m
        self.max_episode_steps = max_episode_steps
        self.comp_body = [m.name2id("body", c) for c in SEQUENCE]
        names = [m.id2name("geom", g) or "" for g in range(m.ngeom)]
        self.geom_pad = [1 if ('gripper' in n and 'pad' in n) else 0 for n in names]
        self.geom_comp = [next((i for i, c in enumerate(SEQUENCE) if c in n), -1) if n else -1 for n in names]
        s = m.name2id("site", "ee_site")
        self.ee_body = int(m.site_bodyid[s])
        self.ee_pos = np.asarray(m.site_pos[s], np.float64)
        q = np.asarray(m.qpos0, np.float64).copy()
        q[0:7] = HOME
        for c in SEQUENCE:
            a = int(m.jnt_qposadr[m.body_jntadr[m.name2id("body", c)]])
            q[a:a + 3] = BINS[c]
            q[a + 3:a + 7] = (1, 0, 0, 0)
        self.reset_qpos = q

    def ids_struct(self) -> cabi.MgxAssemblyIds:
        m, s = self.model, cabi.MgxAssemblyIds()
        for i, b in enumerate(self.comp_body):
            s.comp_body[i] = b
            s.place_reward[i] = PLACE_REWARD[SEQUENCE[i]]
            for k in range(3):
                s.targets[3 * i + k] = TARGETS[SEQUENCE[i]][k]
        s.ee_body = self.ee_body
        s.n_geom = m.ngeom
        s.max_episode_steps = self.max_episode_steps
        s.substeps = SKIP_FRAMES
        s.settle_steps = SETTLE_STEPS
        for g in range(m.ngeom):
            s.geom_comp[g] = self.geom_comp[g]
            s.geom_pad[g] = self.geom_pad[g]
        for k in range(3):
            s.ee_pos[k] = float(self.ee_pos[k])
        jl, jh = np.array(JOINT_LOW) * 0.95, np.array(JOINT_HIGH) * 0.95  # float64, as :414
        for k in range(7):
            s.joint_low[k], s.joint_high[k] = float(jl[k]), float(jh[k])
        for k in range(9):
            s.action_low[k], s.action_high[k] = ACTION_LOW[k], ACTION_HIGH[k]
        return s


class AssemblyVectorEnv:
    """``num_envs`` robotic_arm_assembly envs stepping in lockstep on one GPU."""

    metadata = {'render_modes': [], 'render_fps': 50}

    def __init__(self, num_envs: int, device: str = "cuda:0", precision: str = "f64",
                 max_episode_steps: int = MAX_EPISODE_STEPS, autoreset: bool = True):
        if precision != "f64":
            raise ValueError("robotic_arm_assembly runs in fp64 only: its degenerate base contact (R = 1e-15, "
                             "~1e17 forces) breaks the fp32 Newton factorisation (module docstring)")
        self.num_envs = num_envs
        self.device = torch.device(device)
        self.model = assembly_model()
        self.tables = AssemblyTables(self.model, max_episode_steps)
        self.batch = PhysicsBatch(self.model, num_envs, precision=precision, device=device)
        self.native = self.batch.native
        self.autoreset = autoreset
        dev, N = self.device, num_envs
        self.ints = torch.zeros(N, 16, dtype=torch.int32, device=dev)
        self.ints[:, 1] = -1
        self.cumulative = torch.zeros(N, dtype=torch.float64, device=dev)
        self.episode = torch.zeros(N, dtype=torch.int32, device=dev)
        self.rollout = torch.zeros(N, 4, dtype=torch.float64, device=dev)
        self.reset_qpos = torch.as_tensor(self.tables.reset_qpos, dtype=torch.float64, device=dev)
        self.obs = torch.zeros(N, OBS_DIM, dtype=torch.float32, device=dev)
        self.final_obs = torch.zeros(N, OBS_DIM, dtype=torch.float32, device=dev)
        self.reward = torch.zeros(N, dtype=torch.float64, device=dev)
        self.terminated = torch.zeros(N, dtype=torch.uint8, device=dev)
        self.truncated = torch.zeros(N, dtype=torch.uint8, device=dev)
        self._env = cabi.MgxAssemblyEnv(*[t.data_ptr() for t in (self.ints, self.cumulative, self.episode,
                                                                   self.rollout, self.reset_qpos)])
        ids = self.tables.ids_struct()
        check(lib().mgx_assembly_configure(self.native.handle, C.byref(ids)), "mgx_assembly_configure")
        self.action_space = Box(low=np.array(ACTION_LOW, np.float32), high=np.array(ACTION_HIGH, np.float32),
                                dtype=np.float32)

    def reset(self, seed: Optional[int] = None, env_mask: Optional[torch.Tensor] = None,
              stream=None) -> Tuple[torch.Tensor, Dict[str, Any]]:
        """reset() for all (or masked) envs: deterministic (the seed only reseeds gymnasium's
        np_random, which the reference never draws from)."""
        if seed is not None:
            self.episode.zero_()
        check(lib().mgx_assembly_reset(self.native.handle, C.byref(self.batch.state), C.byref(self._env),
                                       _ptr(self.obs), self.num_envs, _ptr(env_mask), stream_handle(stream)),
              "mgx_assembly_reset")
        return self.obs, self.info()

    def step(self, actions: torch.Tensor, stream=None):
        """One env step (10 mj_steps) for every env. ``actions`` float32 [N, 9]: 7 joint
        commands, gripper opening (mm), grip force (unused by the reference, :252-265)."""
        # float32, or float64: the reference's np.clip keeps a float64 policy's dtype, so ctrl and the
        # action terms of the reward follow in float64 (include/mgx.h action_f64)
        dt = torch.float64 if actions.dtype == torch.float64 else torch.float32
        if actions.dtype != dt or not actions.is_contiguous() or actions.device != self.device:
            actions = actions.to(device=self.device, dtype=dt).contiguous()
        self._env.action_f64 = 1 if dt == torch.float64 else 0
        assert actions.shape == (self.num_envs, N_ACT), actions.shape
        check(lib().mgx_assembly_step(self.native.handle, C.byref(self.batch.state), C.byref(self._env),
                                      _ptr(actions), _ptr(self.obs), _ptr(self.reward), _ptr(self.terminated),
                                      _ptr(self.truncated), _ptr(self.final_obs) if self.autoreset else None,
                                      1 if self.autoreset else 0, self.num_envs, None, stream_handle(stream)),
              "mgx_assembly_step")
        return self.obs, self.reward, self.terminated, self.truncated, self.info()

    def info(self) -> Dict[str, Any]:
        """Device-tensor views of the reference's info dict (:474-484)."""
        return {
            'step_count': self.ints[:, 0],
            'held_component': self.ints[:, 1],
            'task_phase': self.ints[:, 2],
            'assembly_progress_mask': self.ints[:, 3],
            'component_status': self.ints[:, 4:13],
            'cumulative_reward': self.cumulative,
            'final_observation': self.final_obs,
            'episode': self.episode,
            'bad_state_resets': self.batch.warning,
        }

    def close(self):
        pass


class RoboticArmAssemblyEnv(EnvBase):
    """Drop-in for robotic_arm_assembly_env.assembly_env.RoboticArmAssemblyEnv on libmgx.
    Actions are taken as float32 (np.clip against the float32 action_space bounds keeps float32
    actions float32, so a[7] / 1000 is a float32 division, as in the reference for float32
    actions such as action_space.sample())."""

    metadata = {'render_modes': ['human', 'rgb_array'], 'render_fps': 50}

    def __init__(self, render_mode: Optional[str] = None, config: Optional[Dict] = None, device: str = "cuda:0",
                 precision: str = "f64"):
        super().__init__()
        self.render_mode = render_mode
        self.config = config or {}
        self.max_episode_steps = MAX_EPISODE_STEPS
        self.control_frequency = 50
        self.simulation_frequency = 500
        self.skip_frames = SKIP_FRAMES
        self.assembly_tolerance = 0.002
        self.force_threshold = 50.0
        self.gentle_force_threshold = 10.0
        self.assembly_sequence = list(SEQUENCE)
        self.component_targets = {k: np.array(v) for k, v in TARGETS.items()}
        self._vec = AssemblyVectorEnv(1, device=device, precision=precision, autoreset=False,
                                      max_episode_steps=self.max_episode_steps)
        self.model = self._vec.model
        self.observation_space = _observation_space()
        self.action_space = Box(low=np.array(ACTION_LOW, np.float32), high=np.array(ACTION_HIGH, np.float32),
                                dtype=np.float32)
        self.viewer = None
        self.np_random = None
        self.reset()

    def reset(self, seed: Optional[int] = None, options: Optional[Dict] = None):
        obs, _ = self._vec.reset(seed=seed)
        torch.cuda.synchronize(self._vec.device)
        return obs[0].cpu().numpy().copy(), self._get_info()

    def step(self, action: np.ndarray):
        a = torch.from_numpy(policy_action(action).reshape(1, -1)).to(self._vec.device)
        obs, rew, term, trunc, _ = self._vec.step(a)
        torch.cuda.synchronize(self._vec.device)
        return obs[0].cpu().numpy().copy(), float(rew[0]), bool(term[0]), bool(trunc[0]), self._get_info()

    # reference attribute names, read back from the device state
    @property
    def step_count(self) -> int:
        return int(self._vec.ints[0, 0])

    @property
    def held_component(self) -> Optional[str]:
        h = int(self._vec.ints[0, 1])
        return SEQUENCE[h] if h >= 0 else None

    @property
    def task_phase(self) -> str:
        return PHASES[int(self._vec.ints[0, 2])]

    @property
    def assembly_progress(self) -> Dict[str, bool]:
        mask = int(self._vec.ints[0, 3])
        return {c: bool((mask >> i) & 1) for i, c in enumerate(SEQUENCE)}

    @property
    def component_status(self) -> Dict[str, str]:
        st = self._vec.ints[0, 4:13].cpu().tolist()
        return {c: STATUS[s] for c, s in zip(SEQUENCE, st)}

    @property
    def cumulative_reward(self) -> float:
        return float(self._vec.cumulative[0])

    def _get_info(self) -> Dict[str, Any]:
        """:474-484."""
        prog = self.assembly_progress
        return {'step_count': self.step_count, 'assembly_progress': prog.copy(),
                'component_status': self.component_status, 'task_phase': self.task_phase,
                'held_component': self.held_component, 'cumulative_reward': self.cumulative_reward,
                'success': all(prog.values())}

    def render(self):
        if self.render_mode == "rgb_array":
            return np.zeros((480, 640, 3), dtype=np.uint8)  # :494-497
        return None

    def close(self):
        self.viewer = None
