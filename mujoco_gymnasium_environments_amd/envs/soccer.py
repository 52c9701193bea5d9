"""humanoid_soccer_env on MI355X: a batched VectorEnv and a drop-in gymnasium-style Env.

Mirrors the reference interface humanoid_soccer_env/soccer_env.py:
  * ``HumanoidSoccerEnv`` — same constructor/``reset(seed, options)``/``step(action)``/spaces/
    ``metadata``/``render``/``close`` surface as ``HumanoidSoccerEnv`` (soccer_env.py:19-855),
    batch size 1, same gymnasium seeding (PCG64 over SeedSequence) and same 36 reset draws.
  * ``SoccerVectorEnv`` — N envs on one GPU, device tensors ``[N, ...]``, same-step autoreset
    with counter-based (Philox) reset draws keyed by (seed, global env index, episode).
Both run the fused HIP kernel (libmgx.so ``mgx_soccer_step``/``mgx_soccer_reset``):
goalkeeper + wind + mj_step + observation/reward/termination for every env in one launch.
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
from ..native import NativeError, check, lib
from ..seeding import np_random
from ..spaces import Box, EnvBase
from .sharded import StreamShardedEnv

ASSET = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets", "humanoid_soccer.xml")

# soccer_env.py:226-232
JOINT_NAMES = [
    'abdomen_y', 'abdomen_z', 'abdomen_x', 'neck_x', 'neck_y',
    'right_shoulder1', 'right_shoulder2', 'right_elbow', 'right_wrist_y', 'right_wrist_x', 'right_wrist_z',
    'left_shoulder1', 'left_shoulder2', 'left_elbow', 'left_wrist_y', 'left_wrist_x', 'left_wrist_z',
    'right_hip_x', 'right_hip_z', 'right_hip_y', 'right_knee', 'right_ankle_y', 'right_ankle_x',
    'left_hip_x', 'left_hip_z', 'left_hip_y', 'left_knee', 'left_ankle_y', 'left_ankle_x']
# soccer_env.py:799-800
BODY_PARTS = ['foot', 'shin', 'thigh', 'torso', 'head', 'hand', 'arm']
OBS_DIM = 80
MAX_EPISODE_STEPS = 5000          # soccer_env.py:38 (class value governs `truncated`)
REGISTERED_MAX_EPISODE_STEPS = 2500  # humanoid_soccer_env/__init__.py:21 (TimeLimit)


# Contact / row capacity. MuJoCo allocates contacts from its arena and keeps them all. The
# staged step (the default) holds 96 contacts / 384 rows per env — no overflow at bench
# conditions (measured maximum ~230 rows) — so the timed path computes mj_step's physics on every
# env step. full_capacity=False keeps the round-1 capacity of 64 contacts / 192 rows and counts
# the rare env step beyond it (mgx_state.overflow, MuJoCo's mjWARN_CONTACTFULL / CNSTRFULL
# semantics: drop in row order); the monolithic kernel (staged=False) always holds 64 / 192
# (Capacity). The drop-in HumanoidSoccerEnv runs the staged step at full capacity.
CON_CAPACITY = 96
EFC_CAPACITY = 384


@functools.lru_cache(maxsize=None)
def soccer_model(full_capacity: bool = False) -> mjcf.Model:
    with open(ASSET) as f:
        m = mjcf.compile_xml(f.read())
    if full_capacity:
        m.con_capacity = CON_CAPACITY
        m.efc_capacity = EFC_CAPACITY
    return m


class SoccerTables:
    """Index tables the env logic needs, looked up exactly as soccer_env.py:222-263 does."""

    def __init__(self, m: mjcf.Model, max_episode_steps: int = MAX_EPISODE_STEPS):
        self.joint_indices = [m.name2id("joint", n) for n in JOINT_NAMES]
        self.torso = m.name2id("body", "torso")
        self.ball = m.name2id("body", "ball")
        self.goalkeeper = m.name2id("body", "opponent_goalkeeper")
        self.ball_geom = m.name2id("geom", "ball_geom")
        self.right_foot = m.name2id("geom", "right_foot")
        self.left_foot = m.name2id("geom", "left_foot")
        ball_joint = m.name2id("joint", "ball_joint")
        gk_joint = m.name2id("joint", "goalkeeper_y")
        self.ball_qposadr = int(m.jnt_qposadr[ball_joint])
        self.ball_dofadr = int(m.jnt_dofadr[ball_joint])
        self.gk_qposadr = int(m.jnt_qposadr[gk_joint])
        # the reference indexes qfrc_applied with the JOINT id (soccer_env.py:523-524)
        self.gk_qfrc_index = gk_joint
        self.max_episode_steps = max_episode_steps
        nobs = min(m.nu, 25)
        self.obs_joints = [j for j in self.joint_indices[:nobs]]
        # reset noise joints: those with a valid range (soccer_env.py:480-488)
        self.noise_joints = [j for j in self.joint_indices
                             if j < m.nq and m.jnt_range[j][0] < m.jnt_range[j][1]]
        self.root_qposadr = int(m.jnt_qposadr[0])
        mask = 0
        for g, name in enumerate(m.geom_names):
            if name and any(p in name for p in BODY_PARTS):
                mask |= 1 << g
        self.robot_geom_mask = mask
        self.model = m

    def ids_struct(self) -> cabi.MgxSoccerIds:
        m = self.model
        s = cabi.MgxSoccerIds()
        s.torso, s.ball, s.goalkeeper = self.torso, self.ball, self.goalkeeper
        s.ball_geom, s.right_foot, s.left_foot, s.field_geom = self.ball_geom, self.right_foot, self.left_foot, 0
        s.ball_qposadr, s.ball_dofadr, s.gk_qposadr = self.ball_qposadr, self.ball_dofadr, self.gk_qposadr
        s.gk_dofadr = self.gk_qfrc_index
        s.max_episode_steps = self.max_episode_steps
        for i in range(25):
            if i < len(self.obs_joints):
                j = self.obs_joints[i]
                s.obs_jnt_qposadr[i] = int(m.jnt_qposadr[j])
                s.obs_jnt_dofadr[i] = int(m.jnt_dofadr[j])
                s.obs_jnt_range[2 * i] = float(m.jnt_range[j][0])
                s.obs_jnt_range[2 * i + 1] = float(m.jnt_range[j][1])
            else:  # unused slot: lo == hi -> observation 0
                s.obs_jnt_qposadr[i] = 0
                s.obs_jnt_dofadr[i] = 0
        s.robot_geom_mask_lo = self.robot_geom_mask & ((1 << 64) - 1)
        s.robot_geom_mask_hi = self.robot_geom_mask >> 64
        return s

    def reset_draws(self, rng: np.random.Generator) -> np.ndarray:
        """The 36 uniform draws of one reset, in reference order (soccer_env.py:458-504)."""
        d = [rng.uniform(-15.0, -5.0), rng.uniform(-10.0, 10.0), rng.uniform(-0.5, 0.5)]
        d += [rng.uniform(-0.1, 0.1) for _ in self.noise_joints]
        d += [rng.uniform(-2.0, 2.0), rng.uniform(0.0, 2.0), rng.uniform(0, 2 * np.pi), rng.uniform(0.05, 0.15)]
        out = np.zeros(36)
        out[:len(d)] = d
        return out


class SoccerVectorEnv:
    """``num_envs`` humanoid_soccer envs stepping in lockstep on one GPU."""

    metadata = {'render_modes': [], 'render_fps': 50}

    def __init__(self, num_envs: int, device: str = "cuda:0", precision: str = "f64", seed: int = 0,
                 max_episode_steps: int = MAX_EPISODE_STEPS, autoreset: bool = True, env_offset: int = 0,
                 staged: bool = True, banks: int = 3, full_capacity: Optional[bool] = None):
        """``staged`` selects the row-builder / lane-group PGS / finisher kernels
        with ``banks`` precomputed resets per env; ``staged=False`` runs one monolithic wave per
        env. Both compute the same step (parity-tested against each other and the oracle).
        ``full_capacity`` (default: the staged step's) holds 96 contacts / 384 rows instead of
        64 / 192 (see soccer_model)."""
        if full_capacity is None:
            full_capacity = staged
        if full_capacity and not staged:
            # the monolithic layout holds 64 contacts / 192 rows whatever the model's capacity
            raise ValueError("full_capacity needs the staged pipeline (staged=True)")
        self.num_envs = num_envs
        self.device = torch.device(device)
        self.model = soccer_model(full_capacity)
        self.tables = SoccerTables(self.model, max_episode_steps)
        self.batch = PhysicsBatch(self.model, num_envs, precision=precision, device=device)
        self.native = self.batch.native
        self.autoreset = autoreset
        self.seed_value = int(seed) & ((1 << 64) - 1)
        self.env_offset = env_offset
        dt, dev, N = self.batch.dtype, self.device, num_envs
        self.prev_ball_pos = torch.zeros(N, 3, dtype=dt, device=dev)
        self.prev_robot_pos = torch.zeros(N, 3, dtype=dt, device=dev)
        self.wind = torch.zeros(N, 3, dtype=dt, device=dev)
        self.step_count = torch.zeros(N, dtype=torch.int32, device=dev)
        self.goal_scored = torch.zeros(N, dtype=torch.uint8, device=dev)
        self.stats = torch.zeros(N, 5, dtype=dt, device=dev)
        self.episode = torch.zeros(N, dtype=torch.int32, device=dev)
        self.flags = torch.zeros(N, 2, dtype=torch.uint8, device=dev)
        # running sums: reward, terminated, truncated, steps, nefc, PGS sweeps, nefc^2,
        # sweeps * nefc^2 (include/mgx.h mgx_soccer_env.rollout)
        self.rollout = torch.zeros(N, 8, dtype=torch.float64, device=dev)
        self.obs = torch.zeros(N, OBS_DIM, dtype=torch.float32, device=dev)
        self.final_obs = torch.zeros(N, OBS_DIM, dtype=torch.float32, device=dev)
        self.reward = torch.zeros(N, dtype=torch.float64, device=dev)
        self.terminated = torch.zeros(N, dtype=torch.uint8, device=dev)
        self.truncated = torch.zeros(N, dtype=torch.uint8, device=dev)
        self._env = cabi.MgxSoccerEnv(*[t.data_ptr() for t in (self.prev_ball_pos, self.prev_robot_pos, self.wind,
                                                               self.step_count, self.goal_scored, self.stats,
                                                               self.episode, self.flags, self.rollout)])
        self.staged = staged
        self.workspace = None
        if staged:
            nb = int(lib().mgx_soccer_workspace_bytes(self.native.handle, N, banks))
            if nb <= 0:
                raise NativeError(f"mgx_soccer_workspace_bytes: {lib().mgx_last_error().decode()}")
            self.workspace = torch.empty(nb, dtype=torch.uint8, device=dev)
            check(lib().mgx_soccer_workspace_init(self.native.handle, _ptr(self.workspace), nb, N, banks, None),
                  "mgx_soccer_workspace_init")
            self._env.workspace = self.workspace.data_ptr()
            self._env.workspace_bytes = nb
            self._env.banks = banks
        ids = self.tables.ids_struct()
        check(lib().mgx_soccer_configure(self.native.handle, C.byref(ids)), "mgx_soccer_configure")
        nq = np.array([int(self.model.jnt_qposadr[j]) for j in self.tables.noise_joints], dtype=np.int32)
        nr = np.array([self.model.jnt_range[j] for j in self.tables.noise_joints], dtype=np.float64).reshape(-1)
        check(lib().mgx_soccer_configure_reset(self.native.handle, self.tables.root_qposadr, len(nq),
                                               nq.ctypes.data_as(C.POINTER(C.c_int32)),
                                               nr.ctypes.data_as(C.POINTER(C.c_double))), "configure_reset")
        self.action_space = Box(low=-150.0, high=150.0, shape=(self.model.nu,), dtype=np.float32)

    # ------------------------------------------------------------------ API
    def reset(self, seed: Optional[int] = None, env_mask: Optional[torch.Tensor] = None,
              draws: Optional[np.ndarray] = None, stream=None) -> Tuple[torch.Tensor, Dict[str, Any]]:
        """reset() for all (or masked) envs. ``draws`` [N,36] (host, reference order) gives exact
        gymnasium seeding; otherwise device Philox draws keyed by (seed, env, episode)."""
        if seed is not None:
            self.seed_value = int(seed) & ((1 << 64) - 1)
            self.episode.zero_()
        d = None
        if draws is not None:
            d = torch.as_tensor(np.asarray(draws).reshape(self.num_envs, 36), dtype=self.batch.dtype).to(self.device)
        check(lib().mgx_soccer_reset(self.native.handle, C.byref(self.batch.state), C.byref(self._env), _ptr(d),
                                     _ptr(self.obs), self.seed_value, self.env_offset, self.num_envs, _ptr(env_mask),
                                     stream_handle(stream)), "mgx_soccer_reset")
        return self.obs, self.info()

    def step(self, actions: torch.Tensor, stream=None):
        """One env step for every env. ``actions`` [N, nu] on the device: float32, or float64 — a
        float64 action is clipped and applied in float64 and its energy term summed in float64,
        as the reference's np.clip keeps a float64 policy's dtype (soccer_env.py:401-405, :674)."""
        dt = torch.float64 if actions.dtype == torch.float64 else torch.float32
        if actions.dtype != dt or not actions.is_contiguous() or actions.device != self.device:
            actions = actions.to(device=self.device, dtype=dt).contiguous()
        assert actions.shape == (self.num_envs, self.model.nu), actions.shape
        self._env.action_f64 = 1 if dt == torch.float64 else 0
        check(lib().mgx_soccer_step(self.native.handle, C.byref(self.batch.state), C.byref(self._env),
                                    _ptr(actions), _ptr(self.obs), _ptr(self.reward), _ptr(self.terminated),
                                    _ptr(self.truncated), _ptr(self.final_obs) if self.autoreset else None,
                                    1 if self.autoreset else 0, self.seed_value, self.env_offset, self.num_envs,
                                    None, stream_handle(stream)), "mgx_soccer_step")
        return self.obs, self.reward, self.terminated, self.truncated, self.info()

    def info(self) -> Dict[str, Any]:
        """Device-tensor views of the reference's info dict fields (soccer_env.py:433-441)."""
        return {
            'episode_stats': self.stats,  # goals, contacts, distance, time_upright, max_ball_speed
            'ball_position': self.prev_ball_pos,
            'robot_position': self.prev_robot_pos,
            'ball_contact': self.flags[:, 0],
            'robot_upright': self.flags[:, 1],
            'goal_scored': self.goal_scored,
            'final_observation': self.final_obs,
            'episode': self.episode,
            'bad_state_resets': self.batch.warning,
        }

    def close(self):
        pass


class StreamShardedSoccerEnv(StreamShardedEnv):
    """``num_envs`` soccer envs as ``n_streams`` contiguous shards, each its own staged pipeline
    (SoccerVectorEnv, own workspace) on its own HIP stream (envs/sharded.py). One step launches
    every shard's rows -> PGS -> finish chain on its stream, so one shard's row builder
    (LDS-limited) overlaps another's solver (under one wave per SIMD) and the solver's heavy-slot
    tail. Trajectories are the ones a single SoccerVectorEnv over all envs produces
    (tests/test_gpu_staged.py)."""

    def __init__(self, num_envs: int, n_streams: int = 2, device: str = "cuda:0", precision: str = "f64",
                 seed: int = 0, max_episode_steps: int = MAX_EPISODE_STEPS, autoreset: bool = True,
                 env_offset: int = 0, staged: bool = True, banks: int = 3):
        super().__init__(lambda n, off: SoccerVectorEnv(n, device=device, precision=precision, seed=seed,
                                                        max_episode_steps=max_episode_steps, autoreset=autoreset,
                                                        env_offset=env_offset + off, staged=staged, banks=banks),
                         num_envs, n_streams, device)


def _obs_bounds(num_joints: int):
    # soccer_env.py:276-340
    n = min(num_joints, 25)
    low = np.array([*[-1.0] * n, *[-1.0] * n, *[-1.0] * 4, *[-1.0] * 3, *[-1.0] * 3, *[-1.0] * 3, *[-1.0] * 3,
                    *[-1.0] * 3, *[-1.0] * 4, *[-1.0] * 3, 0.0, 0.0, *[-1.0] * 2], dtype=np.float32)
    high = np.array([*[1.0] * n, *[1.0] * n, *[1.0] * 4, *[1.0] * 3, *[1.0] * 3, *[1.0] * 3, *[1.0] * 3,
                     *[1.0] * 3, *[1.0] * 4, *[1.0] * 3, 1.0, 1.0, *[1.0] * 2], dtype=np.float32)
    return low, high


class HumanoidSoccerEnv(EnvBase):
    """Drop-in for humanoid_soccer_env.soccer_env.HumanoidSoccerEnv, simulated by libmgx."""

    metadata = {'render_modes': ['human', 'rgb_array', 'depth_array'], 'render_fps': 50}

    def __init__(self, render_mode: Optional[str] = None, device: str = "cuda:0", precision: str = "f64", **kwargs):
        super().__init__()
        self.dt = 0.02
        self.max_episode_steps = MAX_EPISODE_STEPS
        self.render_mode = render_mode
        # one env on the staged pipeline at MuJoCo's full arena (96 contacts / 384 rows: no row is
        # ever dropped at bench conditions, DESIGN.md §3 Capacity), reset() settled by the same
        # stages (k_soccer_settle) from the gymnasium-seeded host draws; no reset banks (the
        # caller resets). The monolithic kernel holds 64 / 192 and is not used here.
        self._vec = SoccerVectorEnv(1, device=device, precision=precision, autoreset=False,
                                    max_episode_steps=self.max_episode_steps, staged=True, banks=0,
                                    full_capacity=True)
        self.model = self._vec.model
        self.num_joints = self.model.nu
        self.action_space = Box(low=-150.0, high=150.0, shape=(self.num_joints,), dtype=np.float32)
        low, high = _obs_bounds(self.num_joints)
        self.observation_space = Box(low=low, high=high, dtype=np.float32)
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
        return obs[0].cpu().numpy().copy(), self._info(False)

    def step(self, action: np.ndarray):
        # np.clip against the float32 bounds keeps a float64 action float64 (soccer_env.py:401-405)
        action = np.clip(np.asarray(action), self.action_space.low, self.action_space.high)
        action = action.astype(np.float64 if action.dtype == np.float64 else np.float32, copy=False)
        a = torch.from_numpy(np.ascontiguousarray(action.reshape(1, -1))).to(self._vec.device)
        obs, rew, term, trunc, _ = self._vec.step(a)
        torch.cuda.synchronize(self._vec.device)
        self.current_step = int(self._vec.step_count[0])
        return (obs[0].cpu().numpy().copy(), float(rew[0]), bool(term[0]), bool(trunc[0]), self._info(True))

    def _info(self, stepped: bool) -> Dict[str, Any]:
        v = self._vec
        st = v.stats[0].double().cpu().numpy()
        robot = v.prev_robot_pos[0].double().cpu().numpy()
        info = {
            'episode_stats': {'goals_scored': int(st[0]), 'ball_contacts': int(st[1]), 'distance_traveled': float(st[2]),
                              'time_upright': float(st[3]), 'max_ball_speed': float(st[4])},
            'ball_position': v.prev_ball_pos[0].double().cpu().numpy(),
            'robot_position': robot,
            'goal_distance': float(np.linalg.norm(robot - np.array([24.5, 0.0, 0.0]))),
        }
        if stepped:
            fl = v.flags[0].cpu().numpy()
            info.update({'ball_contact': bool(fl[0]), 'robot_upright': bool(fl[1]),
                         'goal_scored': bool(v.goal_scored[0])})
        return info

    def render(self):
        return None  # no viewer on a headless GPU node

    def close(self):
        self.viewer = None


def register_envs() -> bool:
    """Register 'HumanoidSoccer-v0' with gymnasium when it is installed (__init__.py:18-26)."""
    try:
        import gymnasium as gym  # type: ignore
    except Exception:  # noqa: BLE001
        return False
    try:
        gym.register(id='HumanoidSoccer-v0',
                     entry_point='mujoco_gymnasium_environments_amd.envs.soccer:HumanoidSoccerEnv',
                     max_episode_steps=REGISTERED_MAX_EPISODE_STEPS, reward_threshold=8000.0,
                     kwargs={'render_mode': None})
    except Exception:  # noqa: BLE001 - already registered
        pass
    return True
