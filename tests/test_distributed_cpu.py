"""CPU: the N>1 path's collective (end-of-rollout metric all-reduce, max wall time) and the
env sharding arithmetic, with torch.distributed gloo at world_size 2 (127.0.0.1)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mujoco_gymnasium_environments_amd.distributed import env_offset, reduce_rollout
    n = 4096
    off = env_offset(rank, n)
    m = torch.tensor([n * 10.0, 3.0 + rank, -5.0 * (rank + 1), rank, 0.0, 2.0], dtype=torch.float64)
    m, t = reduce_rollout(m, elapsed_s=1.0 + rank)
    q.put((rank, off, m.tolist(), t))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_metric_allreduce():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, off0, m0, t0), (r1, off1, m1, t1) = out
    assert (off0, off1) == (0, 4096)
    assert m0 == m1 == [2 * 40960.0, 7.0, -15.0, 1.0, 0.0, 4.0]
    assert t0 == t1 == 2.0


def test_single_process_noop():
    from mujoco_gymnasium_environments_amd.distributed import reduce_rollout
    m, t = reduce_rollout(torch.ones(6, dtype=torch.float64), 3.5)
    assert m.tolist() == [1.0] * 6 and t == 3.5
