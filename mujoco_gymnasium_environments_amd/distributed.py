"""Env-batch data parallelism across GPUs.

Envs are independent, so rank r of k owns the global env indices [r*N, (r+1)*N): its reset
draws are keyed by the global index (Philox in mgx_soccer_step/reset), so trajectories are
identical for any k. The only collective is one end-of-rollout all-reduce of a small metric
vector (RCCL over xGMI via torch.distributed "nccl"; gloo on CPU for tests).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch

METRICS = ("env_steps", "episodes", "reward_sum", "terminated", "truncated", "bad_state_resets")


def env_offset(rank: int, envs_per_rank: int) -> int:
    return rank * envs_per_rank


def world_from_env() -> Tuple[int, int, int]:
    """(world_size, rank, local_rank) from torchrun's environment (defaults: single process)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def reduce_rollout(metrics: torch.Tensor, elapsed_s: float, group: Optional[object] = None) -> Tuple[torch.Tensor, float]:
    """All-reduce rollout metrics (SUM) and wall time (MAX). No-op without a process group."""
    import torch.distributed as dist
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=metrics.device)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(metrics, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return metrics, float(t.item())
