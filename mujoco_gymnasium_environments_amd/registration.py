"""Environment ids and ``make`` with gymnasium's TimeLimit semantics.

The reference registers its tasks with gymnasium (humanoid_soccer_env/__init__.py:18-26,
quadruped_parkour_env/__init__.py:16-34, bipedal_rescue_env/rescue_env.py:803-814,
humanoid_dancing_env/dancing_env.py:1308-1319); ``gym.make(id)`` then wraps the env in a
``TimeLimit`` whose ``max_episode_steps`` can be shorter than the class's own counter (soccer:
registered 2500, class 5000, soccer_env.py:38,427). gymnasium is not installed here, so ``make``
applies the same wrapper itself; ``register_all()`` registers the ids with gymnasium when it is
importable, and ``gym.make`` then builds the same wrapped env.

TimeLimit (gymnasium/wrappers/common.py): ``step`` counts elapsed steps and sets
``truncated = True`` once ``elapsed >= max_episode_steps``, leaving ``terminated`` as the env
returned it; ``reset`` zeroes the count. The inner env's own truncation still applies.
"""
from __future__ import annotations

import importlib
from typing import Any, Dict, Optional

# id -> (entry point "module:Class", max_episode_steps, reward_threshold, kwargs)
REGISTRY: Dict[str, tuple] = {
    'HumanoidSoccer-v0': ('mujoco_gymnasium_environments_amd.envs.soccer:HumanoidSoccerEnv', 2500, 8000.0,
                          {'render_mode': None}),
    'QuadrupedParkour-v0': ('mujoco_gymnasium_environments_amd.envs.parkour:QuadrupedParkourEnv', 6000, 8000.0,
                            {'render_mode': None}),
    'QuadrupedParkour-v1': ('mujoco_gymnasium_environments_amd.envs.parkour:QuadrupedParkourEnv', 6000, 10000.0,
                            {'render_mode': 'human'}),
    'BipedalRescue-v0': ('mujoco_gymnasium_environments_amd.envs.bipedal:BipedalRescueEnv', 10000, 20000.0, {}),
    'HumanoidDancing-v0': ('mujoco_gymnasium_environments_amd.envs.dancing:HumanoidDancingEnv', 3600, 5000.0, {}),
    'RoboticArmAssembly-v0': ('mujoco_gymnasium_environments_amd.envs.assembly:RoboticArmAssemblyEnv', 150000, 8000.0,
                              {}),   # robotic_arm_assembly_env/__init__.py:12-17
    'HumanoidConstruction-v0': ('mujoco_gymnasium_environments_amd.envs.construction:HumanoidConstructionEnv', 3000,
                                10000.0, {'render_mode': None}),   # humanoid_construction_env/__init__.py:18-26
    # martial arts registers nothing in the reference (humanoid_martial_arts_env/__init__.py)
}


class TimeLimit:
    """gymnasium's TimeLimit wrapper: truncates at ``max_episode_steps`` env steps."""

    def __init__(self, env, max_episode_steps: int):
        self.env = env
        self._max_episode_steps = int(max_episode_steps)
        self._elapsed_steps: Optional[int] = None

    def __getattr__(self, name):
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        return getattr(self.env, 'unwrapped', self.env)

    def reset(self, *, seed: Optional[int] = None, options: Optional[dict] = None):
        self._elapsed_steps = 0
        return self.env.reset(seed=seed, options=options)

    def step(self, action):
        if self._elapsed_steps is None:  # gym.make's OrderEnforcing wrapper raises here
            raise ResetNeeded("Cannot call env.step() before calling env.reset()")
        obs, reward, terminated, truncated, info = self.env.step(action)
        self._elapsed_steps += 1
        if self._elapsed_steps >= self._max_episode_steps:
            truncated = True
        return obs, reward, terminated, truncated, info


try:  # gymnasium.error.ResetNeeded when gymnasium is importable, else a local stand-in
    from gymnasium.error import ResetNeeded  # type: ignore
except Exception:  # noqa: BLE001
    class ResetNeeded(RuntimeError):
        """step() before reset() (gymnasium.error.ResetNeeded)."""


def _load(entry: str):
    mod, cls = entry.split(':')
    return getattr(importlib.import_module(mod), cls)


def make(env_id: str, max_episode_steps: Optional[int] = None, **kwargs: Any):
    """``gym.make(env_id, **kwargs)`` for the registered ids: the env wrapped in TimeLimit."""
    if env_id not in REGISTRY:
        raise KeyError(f"unknown environment id {env_id!r}; registered: {sorted(REGISTRY)}")
    entry, steps, _, defaults = REGISTRY[env_id]
    env = _load(entry)(**{**defaults, **kwargs})
    return TimeLimit(env, steps if max_episode_steps is None else max_episode_steps)


def register_all() -> bool:
    """Register every id with gymnasium when it is importable (False otherwise)."""
    try:
        import gymnasium as gym  # type: ignore
    except Exception:  # noqa: BLE001
        return False
    for env_id, (entry, steps, thr, kw) in REGISTRY.items():
        try:
            gym.register(id=env_id, entry_point=entry, max_episode_steps=steps, reward_threshold=thr, kwargs=kw)
        except Exception:  # noqa: BLE001 - already registered
            pass
    return True
