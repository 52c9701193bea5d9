"""numpy restatement of the humanoid_construction env logic (TEST INFRASTRUCTURE ONLY).

Follows humanoid_construction_env/construction_env.py line by line: step :586-623 (clip :589,
ctrl = action :592, one mj_step :595), task progress :702-719, reward :661-700, termination
:721-737, observation :625-659, reset :547-584. Pinned against the golden vectors produced by
the reference's own methods (tests/golden/construction_envlogic.npz, construction_reset.npz;
tests/test_oracle_construction.py). The physics of this task (RK4 + Newton, nv 99) is not on
the device yet.

Quirks reproduced, not fixed:
  C1  the observation is 135 floats while observation_space declares 125 (:527).
  C2  the energy term -0.2 * np.sum(np.abs(action)) is np.float32 (float32 action), so the reward
      and, through `total_reward += reward`, the episode's total reward are float32 from the
      first step on (NumPy 2 promotion: Python floats are weak scalars).
  C3  blocks_placed and safety_violations never change inside an episode, so stack_blocks and
      build_structure make no progress; the task-completion path only fires for operate_crane
      (step 500) and transport_material (step 300).
  C4  reset() draws the task and the weather from the env generator but never touches qpos:
      mj_resetData leaves the model's qpos0 pose.
"""
from __future__ import annotations

import numpy as np

TASKS = ('stack_blocks', 'operate_crane', 'transport_material', 'build_structure')   # :73
MAX_EPISODE_STEPS = 3000       # :38
MAX_BLOCKS = 20                # :53
BLOCK_PLACED_REWARD = 500.0    # :78
MATERIAL_TRANSPORTED_REWARD = 300.0   # :79
CRANE_OPERATION_REWARD = 200.0        # :80
SAFETY_BONUS = 100.0           # :81
STABILITY_REWARD = 50.0        # :82
ENERGY_PENALTY = -0.2          # :83
FALL_PENALTY = -2000.0         # :85
ACTION_LIMIT = 200.0           # :522-523
OBS_DIM = 135


class ConstructionState:
    """The per-env Python state of HumanoidConstructionEnv between steps."""

    def __init__(self):
        self.task = 0
        self.task_progress = 0.0
        self.blocks_placed = 0
        self.safety_violations = 0
        self.current_step = 0
        self.wind = 0.0
        self.rain = 0.0
        self.temperature = 20.0
        self.hard_hat_on = True
        self.tasks_completed = 0
        self.total_reward = 0.0


class ConstructionLogic:
    def __init__(self, humanoid_body: int, nu: int, max_episode_steps: int = MAX_EPISODE_STEPS):
        self.hid = humanoid_body   # _get_model_indices :513
        self.nu = nu
        self.max_episode_steps = max_episode_steps
        self.low = np.full(nu, -ACTION_LIMIT, dtype=np.float32)
        self.high = np.full(nu, ACTION_LIMIT, dtype=np.float32)

    # -------------------------------------------------------------- reset (:547-584)
    @staticmethod
    def reset(rng: np.random.Generator) -> ConstructionState:
        s = ConstructionState()
        s.task = TASKS.index(str(rng.choice(TASKS)))
        s.wind = rng.uniform(0, 5)
        s.rain = rng.uniform(0, 0.5)
        s.temperature = rng.uniform(15, 35)
        return s

    # -------------------------------------------------------------- step (:586-623)
    def pre(self, action: np.ndarray) -> np.ndarray:
        """The clipped action; it is also data.ctrl (:589-592)."""
        return np.clip(action, self.low, self.high)

    def post(self, s: ConstructionState, action: np.ndarray, qpos: np.ndarray, qvel: np.ndarray,
             xpos: np.ndarray):
        """After mj_step: step counter, progress, reward, flags, observation, total reward."""
        s.current_step += 1
        self.update_progress(s)
        reward = self.reward(s, action, xpos)
        terminated = self.terminated(s, xpos)
        truncated = s.current_step >= self.max_episode_steps
        obs = self.observation(s, qpos, qvel)
        s.total_reward += reward
        return obs, reward, terminated, truncated

    @staticmethod
    def update_progress(s: ConstructionState) -> None:
        t = TASKS[s.task]
        if t == 'stack_blocks':
            s.task_progress = min(1.0, s.blocks_placed / 5)
        elif t == 'operate_crane':
            s.task_progress = min(1.0, s.current_step / 500)
        elif t == 'transport_material':
            s.task_progress = min(1.0, s.current_step / 300)
        elif t == 'build_structure':
            s.task_progress = min(1.0, s.blocks_placed / 10)

    def reward(self, s: ConstructionState, action: np.ndarray, xpos: np.ndarray):
        t = TASKS[s.task]
        r = 0.0
        if t == 'stack_blocks':
            r += s.task_progress * BLOCK_PLACED_REWARD
        elif t == 'operate_crane':
            r += CRANE_OPERATION_REWARD * 0.1
        elif t == 'transport_material':
            r += MATERIAL_TRANSPORTED_REWARD * 0.1
        elif t == 'build_structure':
            r += s.task_progress * 100
        if s.hard_hat_on:
            r += SAFETY_BONUS * 0.01
        r -= s.safety_violations * 100
        r += ENERGY_PENALTY * np.sum(np.abs(action))      # C2: float32 from here on
        if xpos[self.hid][2] > 1.0:
            r += STABILITY_REWARD * 0.1
        else:
            r += FALL_PENALTY
        return r

    def terminated(self, s: ConstructionState, xpos: np.ndarray) -> bool:
        if xpos[self.hid][2] < 0.5:
            return True
        if s.task_progress >= 1.0:
            s.tasks_completed += 1
            return True
        return s.safety_violations > 3

    @staticmethod
    def observation(s: ConstructionState, qpos: np.ndarray, qvel: np.ndarray) -> np.ndarray:
        o = np.zeros(OBS_DIM, dtype=np.float32)
        o[0:30] = qpos[:30]
        o[30:60] = qvel[:30]
        # 60:90 object placeholders
        o[90 + s.task] = 1.0
        o[94] = s.task_progress
        # 95:100 task parameters
        o[100] = s.wind / 10.0
        o[101] = s.rain
        o[102] = s.temperature / 50.0
        # 103:110 environment features
        o[110] = float(s.hard_hat_on)
        o[111] = float(s.safety_violations) / 10.0
        # 112:115 safety features
        o[115] = float(s.blocks_placed) / MAX_BLOCKS
        return o
