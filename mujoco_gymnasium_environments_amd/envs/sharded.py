"""Stream shards: one batch of envs stepped as several contiguous shards, each its own staged
pipeline (own VectorEnv, own workspace) on its own HIP stream (shard 0 on the caller's).

Why: a staged step is a chain of launches per substep (rows -> lane-group PGS -> finish). The
solver launch ends with a tail in which a few waves run the heaviest slots' Gauss–Seidel chains
(parkour's exploding pre-reset states reach 338 rows, DESIGN.md §3 Capacity) while most CUs sit
idle; a second shard's row builder or solver on another stream fills them. Shard i owns global
envs [env_offset + start_i, ...): draws and device Philox streams are keyed by the global env
index, so the trajectories are the ones one VectorEnv over all envs produces
(tests/test_gpu_staged.py, tests/test_gpu_parkour.py). The outputs (obs, reward, flags,
final_obs) are one tensor each; the shards write into row slices of them.
"""
from __future__ import annotations

from collections.abc import Mapping
from typing import Any, Callable, Dict, Optional

import numpy as np
import torch


class _CatInfo(Mapping):
    """info() of a stream-sharded batch: each field is the shards' device views concatenated on
    first access (no kernels are launched for fields the caller never reads). A read-only
    Mapping, so get / items / values / `in` all go through __getitem__ and agree with the
    single-batch VectorEnv.info() dict."""

    def __init__(self, shards):
        self._shards = shards
        self._keys = list(shards[0].info().keys())
        self._cache: Dict[str, Any] = {}

    def __getitem__(self, k):
        if k not in self._cache:
            if k not in self._keys:
                raise KeyError(k)
            self._cache[k] = torch.cat([s.info()[k] for s in self._shards])
        return self._cache[k]

    def __iter__(self):
        return iter(self._keys)

    def __len__(self):
        return len(self._keys)


def shard_bounds(num_envs: int, n_streams: int):
    """contiguous [a, b) ranges, the first num_envs % n_streams one env larger"""
    if n_streams < 1 or n_streams > num_envs:
        raise ValueError("need 1 <= n_streams <= num_envs")
    base, extra = divmod(num_envs, n_streams)
    out, a = [], 0
    for i in range(n_streams):
        b = a + base + (1 if i < extra else 0)
        out.append((a, b))
        a = b
    return out


class StreamShardedEnv:
    """``num_envs`` envs of one task as ``n_streams`` shards; ``make_shard(n, offset)`` builds
    the VectorEnv of one shard (n envs, global env offset ``offset`` added to the caller's)."""

    _OUTPUTS = ("obs", "final_obs", "reward", "terminated", "truncated")

    def __init__(self, make_shard: Callable[[int, int], Any], num_envs: int, n_streams: int = 2,
                 device: str = "cuda:0", serial: bool = False):
        """``serial``: the shards run one after another on the caller's stream (sub-batches:
        each shard's whole step — every substep / RK4 stage — before the next shard's, so one
        shard's constraint rows B, written once per stage and re-read every PGS sweep, are the
        only B live in the 256 MiB Infinity Cache at a time)."""
        self.num_envs = num_envs
        self.device = torch.device(device)
        self.bounds = shard_bounds(num_envs, n_streams)
        self.shards = [make_shard(b - a, a) for a, b in self.bounds]
        s0 = self.shards[0]
        self.model, self.tables, self.action_space = s0.model, s0.tables, s0.action_space
        self.nu = int(np.prod(s0.action_space.shape))
        for name in self._OUTPUTS:
            t = getattr(s0, name)
            full = torch.zeros((num_envs,) + tuple(t.shape[1:]), dtype=t.dtype, device=self.device)
            setattr(self, name, full)
            for (a, b), s in zip(self.bounds, self.shards):  # row slices: contiguous
                setattr(s, name, full[a:b])
        self.serial = serial
        # shard 0 runs on the caller's stream, shards 1.. on streams of their own: K shards take K
        # HIP streams, so up to 4 fit the box's 4 hardware queues (GPU_MAX_HW_QUEUES) without a
        # shard's kernels queueing behind the caller stream's wait for all of them
        self.streams = [] if serial else [torch.cuda.Stream(device=self.device) for _ in self.shards[1:]]

    def _fan_out(self, stream, fn):
        cs = stream if stream is not None else torch.cuda.current_stream(self.device)
        if self.serial:
            for (a, b), s in zip(self.bounds, self.shards):
                fn(a, b, s, cs)
            return
        for st in self.streams:
            st.wait_stream(cs)
        for (a, b), s, st in zip(self.bounds, self.shards, [cs] + self.streams):
            fn(a, b, s, st)
        for st in self.streams:
            cs.wait_stream(st)

    def reset(self, seed: Optional[int] = None, env_mask: Optional[torch.Tensor] = None,
              draws: Optional[np.ndarray] = None, stream=None):
        """reset over every shard (mask / draws sliced per shard)."""
        d = None if draws is None else np.asarray(draws).reshape(self.num_envs, -1)
        self._fan_out(stream, lambda a, b, s, st: s.reset(seed=seed, env_mask=None if env_mask is None else env_mask[a:b],
                                                           draws=None if d is None else d[a:b], stream=st))
        return self.obs, self.info()

    def step(self, actions: torch.Tensor, stream=None):
        """One env step for every env; actions float32 or float64 [N, nu] on the device."""
        dt = torch.float64 if actions.dtype == torch.float64 else torch.float32
        if actions.dtype != dt or not actions.is_contiguous() or actions.device != self.device:
            actions = actions.to(device=self.device, dtype=dt).contiguous()
        assert actions.shape == (self.num_envs, self.nu), actions.shape
        self._fan_out(stream, lambda a, b, s, st: s.step(actions[a:b], stream=st))
        return self.obs, self.reward, self.terminated, self.truncated, self.info()

    def info(self) -> Dict[str, Any]:
        return _CatInfo(self.shards)

    @property
    def episode(self) -> torch.Tensor:
        return torch.cat([s.episode for s in self.shards])

    @property
    def rollout(self) -> torch.Tensor:
        return torch.cat([s.rollout for s in self.shards])

    def close(self):
        pass
