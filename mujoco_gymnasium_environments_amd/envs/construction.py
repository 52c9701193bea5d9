"""humanoid_construction_env on MI355X: a batched VectorEnv and a drop-in gymnasium-style Env.

Mirrors the reference interface humanoid_construction_env/construction_env.py:
  * ``HumanoidConstructionEnv`` — same constructor / ``reset(seed, options)`` / ``step(action)`` /
    spaces / ``metadata`` / ``render`` / ``close`` surface (construction_env.py:24-768), batch size
    1, gymnasium seeding (PCG64 over SeedSequence) and the same draws per reset (task, then wind /
    rain / temperature, :560, :574-576).
  * ``ConstructionVectorEnv`` — N envs on one GPU, device tensors ``[N, ...]``, same-step autoreset
    with Philox reset draws keyed by (seed, global env index, episode).
Both run one fused HIP launch per env step (libmgx.so ``mgx_construction_step``): clip, ctrl =
action, one RK4 mj_step with MuJoCo's default Newton solver (construction_site.xml:10) on the wide
kernels (nv = 99: two dofs per lane, mgx_wide.h), progress / reward / termination / observation.

Quirks reproduced (oracle/construction_logic.py): the 135-float observation against the declared
125 (C1), the np.float32 reward and running total (C2), progress only from the step counter for
operate_crane / transport_material (C3), reset leaves MuJoCo's qpos0 pose and runs no forward
pass (C4).
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
from ..seeding import np_random
from ..spaces import Box, EnvBase, policy_action

ASSET = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets",
                     "humanoid_construction.xml")
OBS_DIM = 135                  # what _get_observation returns (quirk C1)
DECLARED_OBS_DIM = 125         # observation_space (construction_env.py:527)
MAX_EPISODE_STEPS = 3000       # construction_env.py:38
ACTION_LIMIT = 200.0           # construction_env.py:522-523
TASKS = ('stack_blocks', 'operate_crane', 'transport_material', 'build_structure')   # :73
STAT_KEYS = ('blocks_placed', 'materials_transported', 'crane_operations', 'safety_violations',
             'tasks_completed', 'total_reward')


@functools.lru_cache(maxsize=None)
def construction_model() -> mjcf.Model:
    """construction_site.xml as the reference's _generate_xml_files writes it (construction_env.py:
    179-494); nv = 99 > 64, so it runs on the wide kernels with rows in global scratch."""
    with open(ASSET) as f:
        m = mjcf.compile_xml(f.read())
    m.layout_flags = cabi.MGX_ROWS_IN_SCRATCH
    # ten free blocks resting on the floor / foundation / platform plus the humanoid: up to ~100
    # contacts; rows beyond the capacities are dropped with a counter (mgx_state.overflow)
    m.con_capacity = 128
    m.efc_capacity = 512
    return m


class ConstructionTables:
    """Index tables looked up as _get_model_indices does (construction_env.py:511-516)."""

    def __init__(self, m: mjcf.Model, max_episode_steps: int = MAX_EPISODE_STEPS):
        self.model = m
        self.humanoid = m.name2id("body", "humanoid")
        self.crane = m.name2id("body", "crane_base")
        self.max_episode_steps = max_episode_steps

    def ids_struct(self) -> cabi.MgxConstructionIds:
        s = cabi.MgxConstructionIds()
        s.humanoid = self.humanoid
        s.n_act = self.model.nu
        s.max_episode_steps = self.max_episode_steps
        s.action_limit = ACTION_LIMIT
        return s

    @staticmethod
    def reset_draws(rng: np.random.Generator) -> np.ndarray:
        """The draws of one reset, in reference order (construction_env.py:560, :574-576): the task
        (np_random.choice over the 4 task names), wind, rain, temperature."""
        task = TASKS.index(str(rng.choice(TASKS)))
        return np.array([task, rng.uniform(0, 5), rng.uniform(0, 0.5), rng.uniform(15, 35)], dtype=np.float64)


class ConstructionVectorEnv:
    """``num_envs`` humanoid_construction envs stepping in lockstep on one GPU."""

    metadata = {'render_modes': [], 'render_fps': 50}

    def __init__(self, num_envs: int, device: str = "cuda:0", precision: str = "f64", seed: int = 0,
                 max_episode_steps: int = MAX_EPISODE_STEPS, autoreset: bool = True, env_offset: int = 0):
        self.num_envs = num_envs
        self.device = torch.device(device)
        self.model = construction_model()
        self.tables = ConstructionTables(self.model, max_episode_steps)
        self.batch = PhysicsBatch(self.model, num_envs, precision=precision, device=device)
        self.native = self.batch.native
        self.autoreset = autoreset
        self.seed_value = int(seed) & ((1 << 64) - 1)
        self.env_offset = env_offset
        dev, N = self.device, num_envs
        self.scal = torch.zeros(N, 4, dtype=torch.float64, device=dev)   # progress, wind, rain, temperature
        self.ints = torch.zeros(N, 5, dtype=torch.int32, device=dev)     # task, step, blocks, violations, completed
        # episode_stats['total_reward']: a float32 value (NEP 50 keeps it np.float32 for float32 actions)
        # or float64 once a float64 action's reward was added; total_kind records which (include/mgx.h)
        self.total_reward = torch.zeros(N, dtype=torch.float64, device=dev)
        self.total_kind = torch.zeros(N, dtype=torch.uint8, device=dev)
        self.episode = torch.zeros(N, dtype=torch.int32, device=dev)
        self.rollout = torch.zeros(N, 4, dtype=torch.float64, device=dev)
        self.obs = torch.zeros(N, OBS_DIM, dtype=torch.float32, device=dev)
        self.final_obs = torch.zeros(N, OBS_DIM, dtype=torch.float32, device=dev)
        self.reward = torch.zeros(N, dtype=torch.float64, device=dev)
        self.terminated = torch.zeros(N, dtype=torch.uint8, device=dev)
        self.truncated = torch.zeros(N, dtype=torch.uint8, device=dev)
        self._env = cabi.MgxConstructionEnv(*[t.data_ptr() for t in (self.scal, self.ints, self.total_reward,
                                                                      self.episode, self.rollout)])
        self._env.total_kind = self.total_kind.data_ptr()
        ids = self.tables.ids_struct()
        check(lib().mgx_construction_configure(self.native.handle, C.byref(ids)), "mgx_construction_configure")
        self.action_space = Box(low=-ACTION_LIMIT, high=ACTION_LIMIT, shape=(self.model.nu,), dtype=np.float32)

    def reset(self, seed: Optional[int] = None, env_mask: Optional[torch.Tensor] = None,
              draws: Optional[np.ndarray] = None, stream=None) -> Tuple[torch.Tensor, Dict[str, Any]]:
        """reset() for all (or masked) envs. ``draws`` [N,4] (host, reference order) gives exact
        gymnasium seeding; otherwise device Philox draws keyed by (seed, env, episode)."""
        if seed is not None:
            self.seed_value = int(seed) & ((1 << 64) - 1)
            self.episode.zero_()
        d = None
        if draws is not None:
            d = torch.as_tensor(np.asarray(draws).reshape(self.num_envs, 4), dtype=self.batch.dtype).to(self.device)
        check(lib().mgx_construction_reset(self.native.handle, C.byref(self.batch.state), C.byref(self._env), _ptr(d),
                                           _ptr(self.obs), self.seed_value, self.env_offset, self.num_envs,
                                           _ptr(env_mask), stream_handle(stream)), "mgx_construction_reset")
        return self.obs, self.info()

    def step(self, actions: torch.Tensor, stream=None):
        """One env step for every env. ``actions`` [N, nu] float32 or float64 (clipped to +-200)."""
        # float32, or float64: the reference's np.clip keeps a float64 policy's dtype, so ctrl and the
        # action terms of the reward follow in float64 (include/mgx.h action_f64)
        dt = torch.float64 if actions.dtype == torch.float64 else torch.float32
        if actions.dtype != dt or not actions.is_contiguous() or actions.device != self.device:
            actions = actions.to(device=self.device, dtype=dt).contiguous()
        self._env.action_f64 = 1 if dt == torch.float64 else 0
        assert actions.shape == (self.num_envs, self.model.nu), actions.shape
        check(lib().mgx_construction_step(self.native.handle, C.byref(self.batch.state), C.byref(self._env),
                                          _ptr(actions), _ptr(self.obs), _ptr(self.reward), _ptr(self.terminated),
                                          _ptr(self.truncated), _ptr(self.final_obs) if self.autoreset else None,
                                          1 if self.autoreset else 0, self.seed_value, self.env_offset,
                                          self.num_envs, None, stream_handle(stream)), "mgx_construction_step")
        return self.obs, self.reward, self.terminated, self.truncated, self.info()

    def info(self) -> Dict[str, Any]:
        """Device-tensor views of the reference's info dict (construction_env.py:739-752)."""
        return {
            'task': self.ints[:, 0],
            'task_progress': self.scal[:, 0],
            'blocks_placed': self.ints[:, 2],
            'safety_violations': self.ints[:, 3],
            'tasks_completed': self.ints[:, 4],
            'total_reward': self.total_reward,
            'weather': self.scal[:, 1:4],
            'current_step': self.ints[:, 1],
            'final_observation': self.final_obs,
            'episode': self.episode,
            'bad_state_resets': self.batch.warning,
        }

    def close(self):
        pass


class HumanoidConstructionEnv(EnvBase):
    """Drop-in for humanoid_construction_env.construction_env.HumanoidConstructionEnv on libmgx.
    A float32 action (``action_space.sample()``, float32 policies) is clipped against the float32
    bounds in float32, and the reward is np.float32; a float64 action (or a list of floats) stays
    float64 through the clip, ``ctrl`` and the energy term, and the reward is np.float64, as in the
    reference (construction_env.py:589-592, :691).

    ``info['episode_stats']['total_reward']`` is the running total *before* this step's reward:
    the reference copies ``episode_stats`` into ``info`` (construction_env.py:613-614, :746) and
    only then adds the reward (:617). It is a Python 0.0 until the first reward has been added,
    np.float32 after (NEP 50: Python float + np.float32 stays float32)."""

    metadata = {'render_modes': ['human', 'rgb_array'], 'render_fps': 50}

    def __init__(self, render_mode: Optional[str] = None, device: str = "cuda:0", precision: str = "f64", **kwargs):
        super().__init__()
        self.dt = 0.02
        self.max_episode_steps = MAX_EPISODE_STEPS
        self.current_step = 0
        self.render_mode = render_mode
        self._vec = ConstructionVectorEnv(1, device=device, precision=precision, autoreset=False,
                                          max_episode_steps=self.max_episode_steps)
        self.model = self._vec.model
        self.num_joints = self.model.nu
        self.task_types = list(TASKS)
        self.current_task = None
        self.action_space = Box(low=-ACTION_LIMIT * np.ones(self.num_joints), high=ACTION_LIMIT * np.ones(self.num_joints),
                                dtype=np.float32)
        self.observation_space = Box(low=-np.inf, high=np.inf, shape=(DECLARED_OBS_DIM,), dtype=np.float32)
        self.viewer = None
        self.np_random = None
        self.seed()

    def seed(self, seed: Optional[int] = None) -> list:
        self.np_random, seed = np_random(seed)
        return [seed]

    def reset(self, *, seed: Optional[int] = None, options: Optional[Dict[str, Any]] = None):
        if seed is not None:
            self.seed(seed)
        draws = self._vec.tables.reset_draws(self.np_random)[None]
        obs, _ = self._vec.reset(draws=draws)
        torch.cuda.synchronize(self._vec.device)
        self.current_step = 0
        self._total_before = 0.0
        return obs[0].cpu().numpy().copy(), self._info()

    def step(self, action: np.ndarray):
        act = policy_action(action)
        a = torch.from_numpy(act.reshape(1, -1)).to(self._vec.device)
        obs, rew, term, trunc, _ = self._vec.step(a)
        torch.cuda.synchronize(self._vec.device)
        self.current_step = int(self._vec.ints[0, 1])
        info = self._info()  # the total as it was before this step's reward (construction_env.py:614-617)
        kind = int(self._vec.total_kind[0])
        self._total_before = (np.float64 if kind == 1 else np.float32)(self._vec.total_reward[0].item())
        rtype = np.float64 if act.dtype == np.float64 else np.float32
        return obs[0].cpu().numpy().copy(), rtype(rew[0].item()), bool(term[0]), bool(trunc[0]), info

    def _info(self) -> Dict[str, Any]:
        v = self._vec
        sc = v.scal[0].cpu().numpy()
        it = v.ints[0].cpu().numpy()
        self.current_task = TASKS[int(it[0])]
        stats = dict(zip(STAT_KEYS, [0, 0, 0, 0, int(it[4]), getattr(self, '_total_before', 0.0)]))
        return {'task': self.current_task, 'task_progress': float(sc[0]), 'blocks_placed': int(it[2]),
                'safety_violations': int(it[3]), 'episode_stats': stats,
                'weather': {'wind': float(sc[1]), 'rain': float(sc[2]), 'temperature': float(sc[3])}}

    def render(self):
        return None  # no viewer on a headless GPU node

    def close(self):
        self.viewer = None
