"""humanoid_martial_arts_env on MI355X: a batched VectorEnv and a drop-in gymnasium-style Env.

Mirrors the reference interface humanoid_martial_arts_env/martial_arts_env.py:
  * ``HumanoidMartialArtsEnv`` — same constructor / ``reset(seed, options)`` / ``step(action)`` /
    spaces / ``metadata`` / ``render`` / ``close`` surface (martial_arts_env.py:23-651), batch
    size 1, gymnasium seeding (PCG64 over SeedSequence) and the same two draws per reset (:460-463).
  * ``MartialArtsVectorEnv`` — N envs on one GPU, device tensors ``[N, ...]``, same-step autoreset
    with Philox reset draws keyed by (seed, global env index, episode).
Both run one fused HIP launch per env step (libmgx.so ``mgx_martial_step``): clip, ctrl =
action x ctrlrange, one mj_step with the Newton solver (martial_arts_scene.xml:163), observation /
reward / termination / statistics for every env.
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
                     "humanoid_martial_arts.xml")
OBS_DIM = 113                 # what _get_observation returns (quirk M2)
DECLARED_OBS_DIM = 85         # observation_space (:408-420): 29 + 2 * nu
MAX_EPISODE_STEPS = 6000      # martial_arts_env.py:46
STAT_KEYS = ('techniques_performed', 'successful_combos', 'balance_maintained', 'max_power_generated',
             'total_distance_moved', 'falls')


def martial_model(rows_in_scratch: Optional[bool] = None) -> mjcf.Model:
    """The compiled model; rows_in_scratch None = the MGX_MARTIAL_ROWS_LDS environment variable, read at
    each call (not once per process), and part of the cache key."""
    if rows_in_scratch is None:
        rows_in_scratch = os.environ.get("MGX_MARTIAL_ROWS_LDS", "0") != "1"
    return _martial_model(bool(rows_in_scratch))


CON_CAPACITY = 96
EFC_CAPACITY = 384


@functools.lru_cache(maxsize=None)
def _martial_model(rows_in_scratch: bool) -> mjcf.Model:
    """The scene the reference's _generate_xml_files writes (martial_arts_env.py:150-381)."""
    with open(ASSET) as f:
        m = mjcf.compile_xml(f.read())
    m.layout_flags = cabi.MGX_KEEP_CVEL  # the observation and reward read cvel (:536-589)
    # contact / row capacity: the oracle census at the bench's U(-1, 1) actions
    # (tools/capacity_census.py --task martial: 128 envs x 1000 env steps, autoreset) peaks at 75
    # contacts / 320 rows, p99 208 rows — above the 64 / 192 default on ~1.5% of steps. MuJoCo keeps
    # them all; 96 / 384 holds the census maximum (Capacity).
    m.con_capacity = CON_CAPACITY
    m.efc_capacity = EFC_CAPACITY
    # constraint rows in per-env global scratch: the env's LDS drops from 65 to 30 KiB (fp32),
    # five envs per CU instead of two; MGX_MARTIAL_ROWS_LDS=1 keeps them in LDS
    if rows_in_scratch:
        m.layout_flags |= cabi.MGX_ROWS_IN_SCRATCH
    return m


class MartialTables:
    """Index tables looked up exactly as _get_model_indices does (martial_arts_env.py:383-395)."""

    def __init__(self, m: mjcf.Model, max_episode_steps: int = MAX_EPISODE_STEPS):
        self.model = m
        self.torso = m.name2id("body", "torso")
        self.right_hand = m.name2id("body", "right_hand")
        self.left_hand = m.name2id("body", "left_hand")
        self.right_foot = m.name2id("body", "right_ankle")
        self.left_foot = m.name2id("body", "left_ankle")
        self.dummy1 = m.name2id("body", "dummy1")
        self.dummy2 = m.name2id("body", "dummy2")
        self.max_episode_steps = max_episode_steps

    def ids_struct(self) -> cabi.MgxMartialIds:
        m = self.model
        s = cabi.MgxMartialIds()
        s.torso, s.right_hand, s.left_hand = self.torso, self.right_hand, self.left_hand
        s.right_foot, s.left_foot, s.dummy1, s.dummy2 = self.right_foot, self.left_foot, self.dummy1, self.dummy2
        s.n_act = m.nu
        s.max_episode_steps = self.max_episode_steps
        for u in range(m.nu):
            s.ctrl_scale[u] = float(m.actuator_ctrlrange[u][1])
        return s

    @staticmethod
    def reset_draws(rng: np.random.Generator) -> np.ndarray:
        """The 2 uniform draws of one reset, in reference order (martial_arts_env.py:462-463)."""
        return np.array([rng.uniform(-0.5, 0.5), rng.uniform(-0.5, 0.5)])


class MartialArtsVectorEnv:
    """``num_envs`` humanoid_martial_arts envs stepping in lockstep on one GPU."""

    metadata = {'render_modes': [], 'render_fps': 60}

    def __init__(self, num_envs: int, device: str = "cuda:0", precision: str = "f64", seed: int = 0,
                 max_episode_steps: int = MAX_EPISODE_STEPS, autoreset: bool = True, env_offset: int = 0,
                 rows_in_scratch: Optional[bool] = None):
        self.num_envs = num_envs
        self.device = torch.device(device)
        self.model = martial_model(rows_in_scratch)
        self.tables = MartialTables(self.model, max_episode_steps)
        self.batch = PhysicsBatch(self.model, num_envs, precision=precision, device=device)
        self.native = self.batch.native
        self.autoreset = autoreset
        self.seed_value = int(seed) & ((1 << 64) - 1)
        self.env_offset = env_offset
        dev, N = self.device, num_envs
        # stance_stability_time, total_distance_moved, prev_torso_pos[3] (fp64)
        self.scal = torch.zeros(N, 5, dtype=torch.float64, device=dev)
        # current_step, techniques_performed, falls, has prev_torso_pos
        self.ints = torch.zeros(N, 4, dtype=torch.int32, device=dev)
        self.episode = torch.zeros(N, dtype=torch.int32, device=dev)
        self.rollout = torch.zeros(N, 4, dtype=torch.float64, device=dev)
        self.obs = torch.zeros(N, OBS_DIM, dtype=torch.float32, device=dev)
        self.final_obs = torch.zeros(N, OBS_DIM, dtype=torch.float32, device=dev)
        self.reward = torch.zeros(N, dtype=torch.float64, device=dev)
        self.terminated = torch.zeros(N, dtype=torch.uint8, device=dev)
        self.truncated = torch.zeros(N, dtype=torch.uint8, device=dev)
        self._env = cabi.MgxMartialEnv(*[t.data_ptr() for t in (self.scal, self.ints, self.episode, self.rollout)])
        ids = self.tables.ids_struct()
        check(lib().mgx_martial_configure(self.native.handle, C.byref(ids)), "mgx_martial_configure")
        self.action_space = Box(low=-1.0, high=1.0, shape=(self.model.nu,), dtype=np.float32)

    def reset(self, seed: Optional[int] = None, env_mask: Optional[torch.Tensor] = None,
              draws: Optional[np.ndarray] = None, stream=None) -> Tuple[torch.Tensor, Dict[str, Any]]:
        """reset() for all (or masked) envs. ``draws`` [N,2] (host, reference order) gives exact
        gymnasium seeding; otherwise device Philox draws keyed by (seed, env, episode)."""
        if seed is not None:
            self.seed_value = int(seed) & ((1 << 64) - 1)
            self.episode.zero_()
        d = None
        if draws is not None:
            d = torch.as_tensor(np.asarray(draws).reshape(self.num_envs, 2), dtype=self.batch.dtype).to(self.device)
        check(lib().mgx_martial_reset(self.native.handle, C.byref(self.batch.state), C.byref(self._env), _ptr(d),
                                      _ptr(self.obs), self.seed_value, self.env_offset, self.num_envs, _ptr(env_mask),
                                      stream_handle(stream)), "mgx_martial_reset")
        return self.obs, self.info()

    def step(self, actions: torch.Tensor, stream=None):
        """One env step for every env. ``actions`` float32 [N, nu] in [-1, 1] (clipped)."""
        # float32, or float64: the reference's np.clip keeps a float64 policy's dtype, so ctrl and the
        # action terms of the reward follow in float64 (include/mgx.h action_f64)
        dt = torch.float64 if actions.dtype == torch.float64 else torch.float32
        if actions.dtype != dt or not actions.is_contiguous() or actions.device != self.device:
            actions = actions.to(device=self.device, dtype=dt).contiguous()
        self._env.action_f64 = 1 if dt == torch.float64 else 0
        assert actions.shape == (self.num_envs, self.model.nu), actions.shape
        check(lib().mgx_martial_step(self.native.handle, C.byref(self.batch.state), C.byref(self._env),
                                     _ptr(actions), _ptr(self.obs), _ptr(self.reward), _ptr(self.terminated),
                                     _ptr(self.truncated), _ptr(self.final_obs) if self.autoreset else None,
                                     1 if self.autoreset else 0, self.seed_value, self.env_offset, self.num_envs,
                                     None, stream_handle(stream)), "mgx_martial_step")
        return self.obs, self.reward, self.terminated, self.truncated, self.info()

    def info(self) -> Dict[str, Any]:
        """Device-tensor views of the reference's info dict (martial_arts_env.py:623-630)."""
        return {
            'stance_stability': self.scal[:, 0],
            'total_distance_moved': self.scal[:, 1],
            'current_step': self.ints[:, 0],
            'techniques_performed': self.ints[:, 1],
            'falls': self.ints[:, 2],
            'final_observation': self.final_obs,
            'episode': self.episode,
            'bad_state_resets': self.batch.warning,
        }

    def close(self):
        pass


class HumanoidMartialArtsEnv(EnvBase):
    """Drop-in for humanoid_martial_arts_env.martial_arts_env.HumanoidMartialArtsEnv on libmgx.
    Actions are taken as float32 (the reference keeps the caller's dtype through np.clip; its
    energy term is float32 for float32 actions, e.g. action_space.sample())."""

    metadata = {'render_modes': ['human', 'rgb_array', 'depth_array'], 'render_fps': 60}

    def __init__(self, render_mode: Optional[str] = None, device: str = "cuda:0", precision: str = "f64", **kwargs):
        super().__init__()
        self.dt = 0.01667
        self.max_episode_steps = MAX_EPISODE_STEPS
        self.current_step = 0
        self.render_mode = render_mode
        self._vec = MartialArtsVectorEnv(1, device=device, precision=precision, autoreset=False,
                                         max_episode_steps=self.max_episode_steps)
        self.model = self._vec.model
        self.num_joints = self.model.nu
        self.combo_chain = []
        self.action_space = Box(low=-1.0, high=1.0, shape=(self.num_joints,), dtype=np.float32)
        self.observation_space = Box(low=-np.inf, high=np.inf, shape=(DECLARED_OBS_DIM,), dtype=np.float32)
        self.viewer = None
        self.np_random = None
        self.seed()

    def seed(self, seed: Optional[int] = None) -> list:
        self.np_random, seed = np_random(seed)
        return [seed]

    def reset(self, seed: Optional[int] = None, options: Optional[dict] = None):
        if seed is not None:
            self.seed(seed)
        draws = self._vec.tables.reset_draws(self.np_random)[None]
        obs, _ = self._vec.reset(draws=draws)
        torch.cuda.synchronize(self._vec.device)
        self.current_step = 0
        return obs[0].cpu().numpy().copy(), self._info()

    def step(self, action: np.ndarray):
        a = torch.from_numpy(policy_action(action).reshape(1, -1)).to(self._vec.device)
        obs, rew, term, trunc, _ = self._vec.step(a)
        torch.cuda.synchronize(self._vec.device)
        self.current_step = int(self._vec.ints[0, 0])
        return obs[0].cpu().numpy().copy(), float(rew[0]), bool(term[0]), bool(trunc[0]), self._info()

    def _info(self) -> Dict[str, Any]:
        v = self._vec
        sc = v.scal[0].cpu().numpy()
        it = v.ints[0].cpu().numpy()
        stats = dict(zip(STAT_KEYS, [int(it[1]), 0, 0, 0, float(sc[1]), int(it[2])]))
        return {'episode_stats': stats, 'combo_chain': [], 'stance_stability': float(sc[0]),
                'current_step': int(it[0])}

    def render(self):
        return None  # no viewer on a headless GPU node

    def close(self):
        self.viewer = None
