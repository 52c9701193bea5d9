"""gymnasium.spaces.Box when gymnasium is installed; a minimal compatible Box otherwise.

gymnasium is not installed in this image; the envs only need Box's
low/high/shape/dtype/contains/sample surface (soccer_env.py:269-274, :336-340).
"""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - exercised only where gymnasium exists
    from gymnasium.spaces import Box  # type: ignore
    HAVE_GYMNASIUM = True
except Exception:  # noqa: BLE001
    HAVE_GYMNASIUM = False

    class Box:  # type: ignore[no-redef]
        def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
            self.dtype = np.dtype(dtype)
            if shape is not None:
                self.low = np.full(shape, low, dtype=self.dtype)
                self.high = np.full(shape, high, dtype=self.dtype)
            else:
                self.low = np.asarray(low, dtype=self.dtype)
                self.high = np.asarray(high, dtype=self.dtype)
            self.shape = self.low.shape
            self._rng = np.random.default_rng(seed)

        def seed(self, seed=None):
            self._rng = np.random.default_rng(seed)
            return [seed]

        def sample(self):
            return self._rng.uniform(self.low, self.high).astype(self.dtype)

        def contains(self, x) -> bool:
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"

try:  # pragma: no cover
    import gymnasium as _gym  # type: ignore
    EnvBase = _gym.Env
except Exception:  # noqa: BLE001
    class EnvBase:  # type: ignore[no-redef]
        """Stand-in for gymnasium.Env (metadata / render_mode / np_random attributes)."""
        metadata: dict = {}
        render_mode = None
        spec = None

        @property
        def unwrapped(self):
            return self


def policy_action(action) -> np.ndarray:
    """A policy's action as the reference's np.clip against float32 bounds would type it: float32
    when numpy promotes the action with float32 to float32 (float32 / float16 arrays), float64
    otherwise (float64 arrays, Python lists of floats, integer arrays). Contiguous, unclipped: the
    device kernels clip in that dtype."""
    a = np.asarray(action)
    dt = np.float64 if np.result_type(a.dtype, np.float32) == np.float64 else np.float32
    return np.ascontiguousarray(a, dtype=dt)
