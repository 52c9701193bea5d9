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


def test_bench_gpus2_spawns_its_own_ranks():
    """`bench.py --gpus 2` with no outer launcher starts two rank processes itself (the CPU
    harness: gloo + the oracle soccer env in place of RCCL + the GPU step) and rank 0 prints one
    JSON line covering both shards."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--harness", "cpu",
                        "--envs", "2", "--steps", "3", "--warmup", "1"], env=env, cwd=root,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 2 * 2
    assert out["config"]["env_steps_total"] == 2 * 2 * 3 and out["value"] > 0


def test_bench_gpus_must_match_world():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--harness", "cpu"],
                       env=env, cwd=root, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def _bench_worker(rank, world, port, q):
    """One rank of bench.py's harness (timed_region + whole_job_value, the code every bench line
    runs) over its env shard of the oracle soccer env, gloo standing in for RCCL."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import time

    import numpy as np

    import bench
    from mujoco_gymnasium_environments_amd.distributed import env_offset
    n, steps = 2, 4
    envs = [bench.OracleSoccerEnv(env_offset(rank, n) + i, seed=5) for i in range(n)]
    acts = np.random.default_rng(0).uniform(-150, 150, (steps, envs[0].m.nu)).astype(np.float32)
    acc = torch.zeros(6, dtype=torch.float64)

    def step(k):
        for e in envs:
            r, term, trunc = e.step(acts[k])
            acc[0] += 1
            acc[2] += r
            acc[3] += term
            acc[4] += trunc
        time.sleep(0.05 * rank)  # rank 1 is the slow one: the value uses its time

    own = bench.timed_region(step, steps, lambda: None, dist)
    red, elapsed, value = bench.whole_job_value(acc, own)
    q.put((rank, own, elapsed, value, red.tolist()))
    dist.destroy_process_group()


def test_gloo_world2_bench_harness_env_shards():
    """bench.py's N>1 path on CPU: barrier + timed region per rank, SUM of the metrics and MAX of
    the time over ranks, value = all ranks' env steps / slowest time; and the env shards (global
    index = env_offset + local) reproduce a single-process run over all envs."""
    import numpy as np

    import bench
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, own0, el0, v0, red0), (_, own1, el1, v1, red1) = out
    assert red0 == red1, (red0, red1)
    # the closing barrier holds the fast rank until the slow one (4 x 50 ms of sleeps) is done
    assert el0 == el1 == max(own0, own1) and min(own0, own1) >= 4 * 0.05, (own0, own1, el0, el1)
    assert red0[0] == 2 * 2 * 4 and v0 == v1 == red0[0] / el0
    # one process over the 4 global envs: the same totals
    envs = [bench.OracleSoccerEnv(g, seed=5) for g in range(4)]
    acts = np.random.default_rng(0).uniform(-150, 150, (4, envs[0].m.nu)).astype(np.float32)
    rew, term, trunc = 0.0, 0, 0
    for k in range(4):
        for e in envs:
            r, t1, t2 = e.step(acts[k])
            rew, term, trunc = rew + r, term + t1, trunc + t2
    assert abs(red0[2] - rew) <= 1e-9 * abs(rew) and (red0[3], red0[4]) == (term, trunc)


def test_shard_bounds_partition():
    """Stream shards / sub-batches (envs/sharded.py) and rank shards partition envs the same way:
    contiguous, covering, the first num_envs % k shards one env larger, refusing k > num_envs."""
    import pytest as _pytest

    from mujoco_gymnasium_environments_amd.envs.sharded import shard_bounds
    for n, k in ((4096, 3), (190, 3), (101, 2), (7, 7), (5, 1)):
        b = shard_bounds(n, k)
        assert b[0][0] == 0 and b[-1][1] == n and len(b) == k
        assert all(b[i][1] == b[i + 1][0] for i in range(k - 1))
        sizes = [y - x for x, y in b]
        assert max(sizes) - min(sizes) <= 1 and sizes == sorted(sizes, reverse=True)
    with _pytest.raises(ValueError):
        shard_bounds(3, 4)
