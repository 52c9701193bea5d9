"""gymnasium.utils.seeding.np_random restated (used by soccer_env.py:342-345).

gymnasium >= 0.26: Generator(PCG64(SeedSequence(seed))); returns (rng, entropy).
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np


def np_random(seed: Optional[int] = None) -> Tuple[np.random.Generator, int]:
    if seed is not None and not (isinstance(seed, (int, np.integer)) and seed >= 0):
        raise ValueError(f"Seed must be a non-negative python integer, got {seed!r}")
    ss = np.random.SeedSequence(None if seed is None else int(seed))
    return np.random.Generator(np.random.PCG64(ss)), ss.entropy
