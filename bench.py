#!/usr/bin/env python3
"""Headline benchmark: env steps/sec (whole node), humanoid_soccer, 4096 envs per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs 4096]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

`--gpus N` alone (no WORLD_SIZE in the environment) starts the N rank processes itself, one per
GPU, before any GPU call (spawn_ranks); under a launcher, --gpus must equal WORLD_SIZE.

One "step" = one SoccerVectorEnv.step over all envs of a rank: action clip, goalkeeper, wind,
mj_step (kinematics .. PGS .. Euler) and observation/reward/termination for every env, with
same-step autoreset — mgx_soccer_step, the staged kernels k_soccer_rows -> k_pgs_groups ->
k_soccer_bank_finish -> k_soccer_finish -> k_soccer_settle (the resets whose bank was not ready)
on one stream (--mono: one fused kernel). Reset settle steps of the precomputed
reset banks run as extra slots of the same launches. Actions are
synthetic U(-150, 150)^33 float32 drawn before the timed region and resident in HBM.
Ranks shard envs (global index = rank * envs + i); the only collective is the end-of-rollout
metric all-reduce over RCCL. Rank 0 prints ONE JSON line.

--task parkour benchmarks BASELINE configs[1] instead (quadruped_parkour, 4096 envs/GPU, staged per substep; --mono: one wave per env): one
step = ParkourVectorEnv.step = mgx_parkour_step (clip, 10 mj_step's of 1 ms, obstacle motors,
obs/reward/termination, same-step autoreset), actions U(-lim, lim) per joint (80/80/60/40).

--task mixed benchmarks BASELINE configs[4], all seven tasks (soccer, parkour, bipedal, dancing,
martial arts, assembly, construction): 1024 envs per task on one GPU, each task's fused step on its
own HIP stream so the ragged models overlap on the chip; one step = one env step of every task;
value = all tasks' env steps / wall time.

--task bipedal benchmarks BASELINE configs[3] (bipedal_rescue, 8192 envs/GPU by default): one
step = BipedalVectorEnv.step = mgx_bipedal_step (clip, float32 energy, one RK4 mj_step with the
constraint rows in per-env global scratch, victim interactions, obs/reward/termination/stats,
same-step autoreset), actions U(-100, 100)^26.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env steps/sec (whole node), humanoid_soccer 4096 envs/GPU at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
VALU_PEAK_TFLOPS = {"f32": 157.3, "f64": 78.6}  # MI355X_MICROARCH.md: FP32 vector peak; FP64 vector = 1/2
# latest tools/profile_round.sh summaries of the soccer step (HBM traffic per step), per precision
PMC_PROFILE = {"f64": "r06_final2_head_pmc.json", "f32": "r03_f32_pmc.json"}
PMC_PROFILE_BIPEDAL = "r06_final_bipedal_pmc.json"
PMC_PROFILE_ASSEMBLY = "r05_assembly_pmc.json"
PMC_PROFILE_PARKOUR = "r06_parkour_pmc.json"
PMC_PROFILE_CONSTRUCTION = "r05_construction_pmc.json"
PMC_PROFILE_MIXED = "r06_final_mixed_pmc.json"
# algorithmic HBM bytes per env step: r/w qpos 41 + qvel 40 +
# qacc_warmstart 40 (fp32), read action 33, r/w goalkeeper qfrc 1 + ball xfrc 2, r/w 11 task
# scalars, write obs 80 (fp32), reward (fp64), terminated + truncated (u8)
ALG_BYTES_PER_ENV_STEP = 4 * (2 * 121 + 33 + 2 * 3 + 2 * 11 + 80) + 8 + 2
# the same in the parity precision: state, goalkeeper / wind forces and task scalars in fp64
ALG_BYTES_PER_ENV_STEP_F64 = 8 * (2 * 121 + 2 * 3 + 2 * 11) + 4 * (33 + 80) + 8 + 2
# parkour: r/w qpos 38 + qvel 37 + qacc_warmstart 37, r/w the 2 obstacle-motor
# ctrl, read action 16, r/w last_position 3 + max_progress 1 (fp32), r/w episode_reward (fp64)
# + er_kind (u8) + reached/fall/stuck/step (int32), write obs 95, reward (fp64), flags (u8)
PARKOUR_ALG_BYTES = 4 * (2 * 112 + 2 * 2 + 16 + 2 * 4 + 95) + 2 * 8 + 2 + 2 * 16 + 8 + 2
# fp64 (the default precision): the physics state, the motor ctrl and last_position / max_progress
# in 8 bytes
PARKOUR_ALG_BYTES_F64 = 8 * (2 * 112 + 2 * 2 + 2 * 4) + 4 * (16 + 95) + 2 * 8 + 2 + 2 * 16 + 8 + 2
PARKOUR_METRIC = "env steps/sec (whole node), quadruped_parkour 4096 envs/GPU (BASELINE configs[1])"
# bipedal: r/w qpos 63 + qvel 63 + qacc_warmstart 63 and ctrl 26 (fp32), read
# action 26, r/w nine int32 task scalars, energy + energy_used (fp32), carrying (u8), closest,
# prev_sz, distance, prev_robot_pos[3] (fp64), read ttfr (fp64), write obs 102 (fp32), reward
# (fp64), flags (u8)
BIPEDAL_ALG_BYTES = 4 * (2 * 189 + 2 * 26 + 26 + 2 * 9 + 2 * 2 + 102) + 2 + 8 * (2 * 6 + 1 + 1) + 2
# fp64 (the parity precision): the same state / task I/O with the physics reals in 8 bytes
BIPEDAL_ALG_BYTES_F64 = 8 * (2 * 189 + 2 * 26) + 4 * (26 + 2 * 9 + 2 * 2 + 102) + 2 + 8 * (2 * 6 + 1 + 1) + 2
BIPEDAL_METRIC = "env steps/sec (whole node), bipedal_rescue 8192 envs/GPU (BASELINE configs[3])"
# dancing: r/w qpos/qvel/qacc_warmstart 29 each and ctrl 29 (fp32), action 29, r/w 18 fp64 + 8
# int32 task scalars + 3 hist, prev_jvel 23 (fp64), read the 20-move sequence (int32 + fp64),
# obs 94, reward, flags
DANCING_ALG_BYTES = 4 * (2 * 87 + 2 * 29 + 29 + 2 * 8 + 2 * 3 + 20 + 94) + 8 * (2 * 18 + 2 * 23 + 20 + 1) + 2
DANCING_ALG_BYTES_F64 = 8 * (2 * 87 + 2 * 29) + 4 * (29 + 2 * 8 + 2 * 3 + 20 + 94) + 8 * (2 * 18 + 2 * 23 + 20 + 1) + 2
# martial arts: r/w qpos 50 + qvel 47 + qacc_warmstart 47 and ctrl 28 (fp32), action 28, r/w 5 fp64
# + 4 int32 task scalars, obs 113, reward, flags
MARTIAL_ALG_BYTES = 4 * (2 * 144 + 2 * 28 + 28 + 2 * 4 + 113) + 8 * (2 * 5 + 1) + 2
MARTIAL_ALG_BYTES_F64 = 8 * (2 * 144 + 2 * 28) + 4 * (28 + 2 * 4 + 113) + 8 * (2 * 5 + 1) + 2
# assembly (fp64 only): r/w qpos 72 + qvel 63 + qacc_warmstart 63 and ctrl 9 (fp64), action 9,
# r/w 16 int32 task words + cumulative reward (fp64), obs 110 (fp32), reward, flags
ASSEMBLY_ALG_BYTES = 8 * (2 * 198 + 2 * 9) + 4 * (9 + 2 * 16 + 110) + 8 * (2 + 1) + 2
# construction (fp64): r/w qpos 110 + qvel 99 + qacc_warmstart 99 and ctrl 33, action 33 (fp32), r/w
# 4 fp64 + 5 int32 task scalars and the fp32 total, obs 135, reward, flags
CONSTRUCTION_ALG_BYTES = 8 * (2 * 308 + 2 * 33 + 2 * 4 + 1) + 4 * (33 + 2 * 5 + 2 + 135) + 2
ASSEMBLY_METRIC = "env steps/sec (whole node), robotic_arm_assembly 1024 envs/GPU (10 Newton substeps per env step)"
MIXED_METRIC = "env steps/sec (whole node), all tasks mixed, 1024 envs each on 1 MI355X (BASELINE configs[4])"


def _pmc_traffic(name: str, envs: int, precision: str, mode: str):
    """HBM bytes per step from a committed tools/profile_round.sh summary of the same config."""
    path = os.path.join(ROOT, "profiles", name)
    try:
        with open(path) as f:
            p = json.load(f)
        if p.get("envs") == envs and p.get("precision") == precision and p.get("mode") == mode:
            return p.get("hbm_bytes_per_step")
    except Exception:  # noqa: BLE001
        pass
    return None


def _finite(x: float):
    """JSON-safe mean: the bipedal approach term is +inf on the first step after a reset
    (rescue_env.py:632-635), which makes a rollout's reward sum infinite."""
    return round(x, 3) if np.isfinite(x) else None


def timed_region(step, steps: int, sync, dist=None) -> float:
    """The timed region of every bench line: a barrier and a device sync on both sides of exactly
    `steps` calls of step(k); returns this rank's wall seconds."""
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(steps):
        step(k)
    sync()
    if dist:
        dist.barrier()
    return time.perf_counter() - t0


def whole_job_value(acc, elapsed: float):
    """End-of-rollout reduction (SUM of the metric vector, MAX of the wall time over ranks) and
    the whole-job value: env steps of all ranks / the slowest rank's time."""
    from mujoco_gymnasium_environments_amd.distributed import reduce_rollout
    acc, elapsed = reduce_rollout(acc, elapsed)
    return acc, elapsed, acc[0].item() / elapsed


class OracleSoccerEnv:
    """One humanoid_soccer env on the oracle (mjref fp64 physics + the numpy logic oracle), reset
    draws keyed by the GLOBAL env index like the device's (seed + global_env), same-step autoreset.
    The CPU baseline and the gloo test of the bench harness step it."""

    _shared = None  # (model, tables, logic, packed model): built once per process

    def __init__(self, global_env: int, seed: int = 0):
        from mujoco_gymnasium_environments_amd.seeding import np_random
        from oracle.mjref import RefSim
        if OracleSoccerEnv._shared is None:
            from mujoco_gymnasium_environments_amd import cabi
            from mujoco_gymnasium_environments_amd.envs.soccer import SoccerTables, soccer_model
            from oracle.soccer_logic import SoccerLogic
            m = soccer_model()
            tb = SoccerTables(m)
            OracleSoccerEnv._shared = (m, tb, SoccerLogic(tb), cabi.pack_model(m))
        self.m, self.tb, self.L, pk = OracleSoccerEnv._shared
        m = self.m
        self.sim = RefSim(pk)
        self.draws = self.tb.reset_draws(np_random(seed + global_env)[0])
        nn = len(self.tb.noise_joints)
        d = self.draws
        self.s = dict(wind_strength=d[4 + nn], wind_direction=np.array([np.cos(d[5 + nn]), np.sin(d[5 + nn])]))
        self.reset()

    def reset(self):
        m, tb, sim, d = self.m, self.tb, self.sim, self.draws
        sim.reset()
        q = sim.qpos
        a0 = tb.root_qposadr
        q[a0:a0 + 3] = [d[0], d[1], 1.4]
        q[a0 + 3:a0 + 7] = [np.cos(d[2] / 2), 0, 0, np.sin(d[2] / 2)]
        q[tb.ball_qposadr:tb.ball_qposadr + 3] = [d[0] + 2, d[1], 0.15]
        for k, j in enumerate(tb.noise_joints):
            lo, hi = m.jnt_range[j]
            q[m.jnt_qposadr[j]] = np.clip((lo + hi) / 2 + d[3 + k], lo, hi)
        q[tb.gk_qposadr] = d[3 + len(tb.noise_joints)]
        sim.step(10)
        self.view()
        self.s.update(goal_scored=False, stats=np.zeros(5), prev_ball_pos=self.s["xpos"][tb.ball].copy(),
                      prev_robot_pos=self.s["xpos"][tb.torso].copy())
        self.nstep = 0

    def view(self):
        m, sim = self.m, self.sim
        c = sim.contacts()
        self.s.update(qpos=sim.qpos, qvel=sim.qvel, xpos=sim.xpos.reshape(-1, 3), xquat=sim.xquat.reshape(-1, 4),
                      subtree_com=sim.subtree_com.reshape(-1, 3), con_geom=c["geom"], con_dist=c["dist"],
                      con_mu=np.array([np.linalg.norm(m.pair_friction[p][:2]) for p in c["pair"]]), ctrl=sim.ctrl,
                      qfrc_applied=sim.qfrc_applied, xfrc_applied=sim.xfrc_applied.reshape(-1, 6))

    def step(self, action):
        """-> (reward, terminated, truncated); an ended episode is reset in the same call."""
        a = self.L.pre(self.s, action)
        self.sim.step()
        self.view()
        self.nstep += 1
        _, reward, term, trunc, _, _ = self.L.post(self.s, a, self.nstep)
        if term or trunc:
            self.reset()
        return float(reward), bool(term), bool(trunc)


def cpu_baseline_task(task: str, n_envs: int, n_steps: int, seed: int = 0) -> dict:
    """Oracle port on one host core (oracle/envs.py: mjref C fp64 physics + the task's numpy
    logic), n_envs envs one after another, n_steps env steps each with autoreset, at the bench's
    action distribution. Besides the rate it reports the oracle's own termination and bad-state
    (MuJoCo's auto-reset) rates at these actions, to read next to the device line's."""
    from mujoco_gymnasium_environments_amd.seeding import np_random
    from oracle.envs import ORACLES, task_setup
    packed, tb, draws_fn, acts_fn = task_setup(task)
    acts = acts_fn(np.random.default_rng(seed), 64)
    total = terms = bad = 0
    t0 = time.perf_counter()
    for e in range(n_envs):
        rng = np_random(seed + e)[0]
        env = ORACLES[task](packed, tb)
        env.reset(draws_fn(rng))
        for k in range(n_steps):
            _, _, te, tr = env.step(acts[k % 64])
            total += 1
            terms += te
            if te or tr:
                env.reset(draws_fn(rng))
        bad += env.bad_states
    dt = time.perf_counter() - t0
    what = {"soccer": "humanoid_soccer, U(-150,150) actions",
            "parkour": "quadruped_parkour (10 substeps each), U(-lim, lim) actions",
            "bipedal": "bipedal_rescue (RK4), U(-100,100) actions"}[task]
    return {"value": total / dt, "unit": "env_steps/s", "cores": 1, "kind": "port",
            "sample": f"{n_envs} envs x {n_steps} steps (autoreset) of {what}, oracle/mjref.c fp64 physics + "
                      f"oracle/{task}_logic.py; CPU MuJoCo unavailable (not installed)",
            "seconds": round(dt, 2), "host_cpu": platform.processor() or platform.machine(),
            "oracle_termination_rate": round(terms / max(total, 1), 5),
            "oracle_bad_state_rate": round(bad / max(total, 1), 5)}


def cpu_baseline(n_envs: int, n_steps: int, seed: int = 0) -> dict:
    return cpu_baseline_task("soccer", n_envs, n_steps, seed)


def cpu_baseline_parkour(n_envs: int, n_steps: int, seed: int = 0) -> dict:
    return cpu_baseline_task("parkour", n_envs, n_steps, seed)


def cpu_baseline_bipedal(n_envs: int, n_steps: int, seed: int = 0) -> dict:
    return cpu_baseline_task("bipedal", n_envs, n_steps, seed)


def cpu_baseline_assembly(n_envs: int, n_steps: int, seed: int = 0) -> dict:
    """Oracle port on one host core: mjref (C, fp64, Newton) physics + numpy assembly logic."""
    from mujoco_gymnasium_environments_amd import cabi
    from mujoco_gymnasium_environments_amd.envs.assembly import AssemblyTables, assembly_model
    from oracle.assembly_logic import AssemblyLogic, AssemblyTables as OTables
    from oracle.mjref import RefSim
    m = assembly_model()
    pk = cabi.pack_model(m)
    tb = AssemblyTables(m)
    L = AssemblyLogic(OTables(m))
    rng = np.random.default_rng(seed)
    lo = np.array([-2.0] * 7 + [0, 0])
    hi = np.array([2.0] * 7 + [100, 50])
    total = 0
    t0 = time.perf_counter()
    for e in range(n_envs):
        sim = RefSim(pk)

        def reset():
            sim.reset()
            sim.qpos[:] = tb.reset_qpos
            sim.step(10)
            return L.new_state()
        s = reset()
        for _ in range(n_steps):
            a = rng.uniform(lo, hi).astype(np.float32)
            _, ctrl = L.pre(a)
            sim.ctrl[:] = ctrl
            sim.step(10)
            c = sim.contacts()
            nc = int(sim.ncon[0])
            _, _, term, trunc = L.post(s, sim.qpos, sim.qvel, sim.xpos.reshape(-1, 3), sim.xmat.reshape(-1, 9),
                                       c["geom"][:nc], c["dist"][:nc])
            total += 1
            if term or trunc:
                s = reset()
    dt = time.perf_counter() - t0
    return {"value": total / dt, "unit": "env_steps/s", "cores": 1, "kind": "port",
            "sample": f"{n_envs} envs x {n_steps} steps (autoreset) of robotic_arm_assembly, uniform actions, "
                      f"oracle/mjref.c fp64 Newton physics (10 substeps) + oracle/assembly_logic.py; CPU MuJoCo "
                      f"unavailable (not installed)",
            "seconds": round(dt, 2), "host_cpu": platform.processor() or platform.machine()}


# round 5 (assembly now the longest stream): soccer beside construction, dancing beside bipedal —
# 125.8k / 126.0k / 126.5k against 125.0k / 124.5k / 124.6k env-steps/s for the round-4 grouping
# (construction alone; bipedal + soccer; parkour + martial arts + dancing), alternating runs on one box
# Round 6 (parkour at MuJoCo's full arena, 96 contacts / 384 rows): parkour's stream alone, martial
# arts beside construction and soccer — 112.8k -> 128.8k env-steps/s against the round-5 grouping
# (parkour with martial arts), one box, profiles/r06_mixed_groups_ab.json
MIXED_GROUPS = [["humanoid_construction", "humanoid_soccer", "humanoid_martial_arts"], ["robotic_arm_assembly"],
                ["bipedal_rescue", "humanoid_dancing"], ["quadruped_parkour"]]
# MGX_MIX_GROUPS (A/B hook): another grouping, groups separated by ';', tasks by ',' (group 0 is
# the high-priority one)
if os.environ.get("MGX_MIX_GROUPS"):
    MIXED_GROUPS = [g.split(",") for g in os.environ["MGX_MIX_GROUPS"].split(";")]


def sharded(args, N, dev, make):
    """the task's VectorEnv, or --streams > 1 of them as stream shards (envs/sharded.py)"""
    from mujoco_gymnasium_environments_amd.envs.sharded import StreamShardedEnv
    if args.sub_batches > 1:
        return StreamShardedEnv(make, N, args.sub_batches, device=str(dev), serial=True)
    if args.streams <= 1:
        return make(N, 0)
    return StreamShardedEnv(make, N, args.streams, device=str(dev))


def _with_hooks(kv: dict, make):
    """make() with the MGX_* hooks in kv set in the environment (libmgx reads them when a model is
    created), the previous values restored after"""
    old = {k: os.environ.get(k) for k in kv}
    os.environ.update(kv)
    try:
        return make()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def mix_parkour_hooks() -> dict:
    """A/B hook MGX_MIX_PK_PRIO_ROWS: in the mixed run, parkour's solver waves raise their wave
    priority above this many rows (MGX_PGS_PRIO_ROWS for the parkour model only)"""
    v = os.environ.get("MGX_MIX_PK_PRIO_ROWS")
    return {"MGX_PGS_PRIO_ROWS": v} if v else {}


def mixed_side_streams(n_tasks: int, mix_streams: int) -> None:
    """The grouped layout runs without the staged tasks' side streams (MGX_SIDE_STREAM=0, a hook
    libmgx reads when a model is created: call this before the envs are built)."""
    if mix_streams < n_tasks:
        os.environ["MGX_SIDE_STREAM"] = "0"


def mixed_streams(tasks, mix_streams: int, mix_priority: int, dev):
    """The mixed run's HIP streams per task (tests/test_gpu_mixed.py steps the same layout).

    HIP streams map onto GPU_MAX_HW_QUEUES hardware queues (4 on the box): with a stream per
    task (7, plus the staged tasks' side streams) unrelated tasks share queues and wait on each
    other's kernels. Four streams instead: construction (with soccer and martial arts) and assembly,
    the long Newton steps, each on a stream of their own, bipedal with dancing, and parkour (its
    heavy-slot solver chains) alone; no side streams
    (MGX_SIDE_STREAM=0, mixed_side_streams). Construction's stream runs at high priority
    (mix_priority 1, measured 73.2k -> 75.5k env-steps/s in round 4; in round 5 group 0 alone is
    still best: 122.7k against 119.4k with assembly's group, 118.9k with both). mix_streams 7: one
    stream per task (67.3k)."""
    if mix_streams >= len(tasks):
        return {k: torch.cuda.Stream(device=dev) for k in tasks}
    # (dancing with parkour and martial arts: 75.5 / 76.7k against 74.9 / 75.0k with dancing
    # beside bipedal and soccer, two A/B pairs on one box)
    # MGX_MIX_PRIO_GROUPS (A/B hook): which groups run at high priority; 0 / 0,1 / 1 measured
    # within noise of each other (75.3k - 75.9k, profiles/r04_mixed_priority_ab.json)
    # round 6: construction's group and parkour's stream at high priority (130.1k -> 132.0k
    # env-steps/s mean of two interleaved pairs, profiles/r06_mixed_priority_ab.json)
    hi = {int(x) for x in os.environ.get("MGX_MIX_PRIO_GROUPS", "0,3").split(",") if x} if mix_priority else set()
    gs = [torch.cuda.Stream(device=dev, priority=-1 if i in hi else 0) for i in range(len(MIXED_GROUPS))]
    return {k: gs[i] for i, grp in enumerate(MIXED_GROUPS) for k in grp if k in tasks}


def bench_mixed(args, dev, world, rank, dist):
    """BASELINE configs[4]: every built task, N envs each, one HIP stream per task."""
    from mujoco_gymnasium_environments_amd.distributed import env_offset, reduce_rollout
    from mujoco_gymnasium_environments_amd.envs.assembly import AssemblyVectorEnv
    from mujoco_gymnasium_environments_amd.envs.bipedal import BipedalVectorEnv
    from mujoco_gymnasium_environments_amd.envs.construction import ConstructionVectorEnv
    from mujoco_gymnasium_environments_amd.envs.dancing import DancingVectorEnv
    from mujoco_gymnasium_environments_amd.envs.martial import MartialArtsVectorEnv
    from mujoco_gymnasium_environments_amd.envs.parkour import ParkourVectorEnv, action_limits
    from mujoco_gymnasium_environments_amd.envs.soccer import SoccerVectorEnv
    N = args.envs
    off = env_offset(rank, N)
    f64 = args.precision == "f64"
    g = torch.Generator(device=dev)
    g.manual_seed(2000 + rank)
    plim = torch.as_tensor(action_limits(), dtype=torch.float32, device=dev)
    # assembly action_space: [-2, 2]^7 joint commands, [0, 100] opening, [0, 50] force (:150-151)
    alo = torch.tensor([-2.0] * 7 + [0.0, 0.0], device=dev)
    alim = torch.tensor([4.0] * 7 + [100.0, 50.0], device=dev)
    mixed_side_streams(7, args.mix_streams)
    tasks = {
        "humanoid_soccer": (SoccerVectorEnv(N, device=str(dev), precision=args.precision, seed=11, env_offset=off,
                                            banks=args.banks), lambda: torch.rand(N, 33, device=dev, generator=g) * 300 - 150,
                            ALG_BYTES_PER_ENV_STEP_F64 if f64 else ALG_BYTES_PER_ENV_STEP),
        "quadruped_parkour": (_with_hooks(mix_parkour_hooks(), lambda: ParkourVectorEnv(
                                  N, device=str(dev), precision=args.precision, seed=12, env_offset=off,
                                  staged=bool(args.mix_staged))),
                              lambda: (torch.rand(N, 16, device=dev, generator=g) * 2 - 1) * plim,
                              PARKOUR_ALG_BYTES_F64 if f64 else PARKOUR_ALG_BYTES),
        "bipedal_rescue": (BipedalVectorEnv(N, device=str(dev), precision=args.precision, seed=13, env_offset=off,
                                            staged=bool(args.mix_staged)),
                           lambda: (torch.rand(N, 26, device=dev, generator=g) * 2 - 1) * 100.0,
                           BIPEDAL_ALG_BYTES_F64 if f64 else BIPEDAL_ALG_BYTES),
        "humanoid_dancing": (DancingVectorEnv(N, device=str(dev), precision=args.precision, seed=14, env_offset=off),
                             lambda: (torch.rand(N, 29, device=dev, generator=g) * 2 - 1) * 200.0,
                             DANCING_ALG_BYTES_F64 if f64 else DANCING_ALG_BYTES),
        "humanoid_martial_arts": (MartialArtsVectorEnv(N, device=str(dev), precision=args.precision, seed=15,
                                                       env_offset=off),
                                  lambda: torch.rand(N, 28, device=dev, generator=g) * 2 - 1,
                                  MARTIAL_ALG_BYTES_F64 if f64 else MARTIAL_ALG_BYTES),
        # assembly's reset is deterministic (assembly_env.py:162-218): no seed; fp64 only (its
        # degenerate base contact breaks the fp32 Newton factorisation, envs/assembly.py)
        "robotic_arm_assembly": (AssemblyVectorEnv(N, device=str(dev), precision="f64"),
                                 lambda: torch.rand(N, 9, device=dev, generator=g) * alim + alo, ASSEMBLY_ALG_BYTES),
        # construction: fp64 like assembly (RK4 + Newton on the wide kernels, nv 99; its parity
        # tests run in fp64, tests/test_gpu_construction.py)
        "humanoid_construction": (ConstructionVectorEnv(N, device=str(dev), precision="f64", seed=17, env_offset=off),
                                  lambda: (torch.rand(N, 33, device=dev, generator=g) * 2 - 1) * 200.0,
                                  CONSTRUCTION_ALG_BYTES),
    }
    streams = mixed_streams(list(tasks), args.mix_streams, args.mix_priority, dev)
    pools = {k: [f().contiguous() for _ in range(8)] for k, (_, f, _) in tasks.items()}
    for k, (env, _, _) in tasks.items():
        env.reset()
    torch.cuda.synchronize(dev)

    def one_step(i, ev=None):
        for k, (env, _, _) in tasks.items():
            with torch.cuda.stream(streams[k]):
                if ev is not None:
                    ev[k][0].record(streams[k])
                env.step(pools[k][i % 8], stream=streams[k])
                if ev is not None:
                    ev[k][1].record(streams[k])
    for i in range(args.warmup):
        one_step(i)
    torch.cuda.synchronize(dev)
    for env, _, _ in tasks.values():
        env.rollout.zero_()
        env.batch.overflow.zero_()
    warn0 = {k: int(env.batch.warning.sum().item()) for k, (env, _, _) in tasks.items()}
    evs = [{k: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for k in tasks}
           for _ in range(args.steps)]
    elapsed = timed_region(lambda i: one_step(i, evs[i]), args.steps, lambda: torch.cuda.synchronize(dev), dist)
    per = {k: float(np.mean([e[k][0].elapsed_time(e[k][1]) for e in evs])) for k in tasks}
    acc = torch.zeros(6, dtype=torch.float64, device=dev)
    # per task, over the timed region: MuJoCo's bad-state auto-resets and the env steps whose
    # contacts / rows exceeded the task's capacity (0 when every row MuJoCo keeps was kept)
    bad = {k: int(env.batch.warning.sum().item()) - warn0[k] for k, (env, _, _) in tasks.items()}
    ovf = {k: int(env.batch.overflow.sum().item()) for k, (env, _, _) in tasks.items()}
    for k, (env, _, _) in tasks.items():
        ro = env.rollout.double().sum(0)
        acc[0] += ro[3]
        acc[2] += ro[0] if torch.isfinite(ro[0]) else 0.0
        acc[3] += ro[1]
        acc[4] += ro[2]
        acc[5] += bad[k]
    acc, elapsed, _ = whole_job_value(acc, elapsed)
    total = acc[0].item()
    if rank == 0:
        # roofline of the whole mixed step: every task's algorithmic bytes over the step's wall
        # time (the seven steps overlap on four streams); traffic = the PMC bytes of every step
        # kernel per step (tools/profile_round.sh with --task mixed)
        dom = max(per, key=per.get)
        bytes_all = sum(t[2] for t in tasks.values()) * N
        step_s = elapsed / args.steps
        achieved = bytes_all / step_s / 1e9
        out = {
            "metric": MIXED_METRIC, "value": round(total / elapsed, 1), "unit": "env_steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "data": "synthetic (uniform actions within each task's action_space, Philox reset draws)",
            "config": {"workload": "all tasks mixed, 1024 envs each on 1 GPU (BASELINE configs[4])",
                       "tasks": list(tasks), "tasks_missing": [],
                       "envs_per_task": N, "global_batch": N * len(tasks) * world,
                       "parallelism": f"dp{world} (env shards), {len(set(map(id, streams.values())))} HIP streams",
                       "autoreset": "same-step", "task_launch_ms": {k: round(v, 4) for k, v in per.items()},
                       "task_dtype": {k: ("f64" if k in ("robotic_arm_assembly", "humanoid_construction")
                                          else args.precision) for k in tasks},
                       "bad_state_resets": int(acc[5].item()), "bad_state_resets_per_task": bad,
                       "capacity_overflow_steps": sum(ovf.values()), "capacity_overflow_steps_per_task": ovf},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": _pmc_traffic(PMC_PROFILE_MIXED, N, args.precision, "mixed"),
                         "profile": f"profiles/{PMC_PROFILE_MIXED}",
                         "kernel": f"all seven tasks' step launches (longest stream: {dom})",
                         "alg_bytes_per_step": bytes_all, "launch_ms": round(step_s * 1e3, 4)},
        }
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


def soccer_flops(ro: torch.Tensor, nv: int) -> dict:
    """SURVEY 8(d) algorithmic FLOPs of the soccer step from the in-kernel sums (dense-equivalent
    count of the constraint phase: A = J M^-1 J' costs 2 nefc^2 nv, PGS 2 sweeps nefc^2; the
    kinematics / CRB / RNE rest ~ 300 nbody is added as a constant)."""
    steps = float(ro[3])
    a = 2.0 * float(ro[6]) * nv
    pgs = 2.0 * float(ro[7])
    rest = 300.0 * 20 * steps
    return {"flops_per_env_step": (a + pgs + rest) / max(steps, 1.0), "nefc_mean": float(ro[4]) / max(steps, 1.0),
            "pgs_sweeps_mean": float(ro[5]) / max(steps, 1.0)}


def bipedal_other_line(args, dev, N, g, precision: str) -> dict:
    """configs[3] in the other precision (a short timed run after the headline's timed region).
    fp64 is the parity precision; fp32 is compared with it by distribution
    (tests/test_gpu_bipedal.py::test_bipedal_f32_distribution_matches_f64)."""
    from mujoco_gymnasium_environments_amd.envs.bipedal import BipedalVectorEnv
    env = BipedalVectorEnv(N, device=str(dev), precision=precision, seed=1234, staged=not args.mono,
                           banks=min(args.banks, 1) if args.banks > 0 else 0)
    pool = [((torch.rand(N, 26, device=dev, generator=g) * 2 - 1) * 100.0).contiguous() for _ in range(4)]
    env.reset()
    for k in range(3):
        env.step(pool[k % 4])
    torch.cuda.synchronize(dev)
    steps = 10
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record()
    for k in range(steps):
        env.step(pool[k % 4])
    b.record()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    return {"value": round(N * steps / el, 1), "unit": "env_steps/s", "ms_per_step": round(el / steps * 1e3, 4),
            "launch_ms": round(a.elapsed_time(b) / steps, 4), "steps": steps, "dtype": precision,
            "step_kernels": "mono" if args.mono else "staged"}


def other_precision_line(args, dev, N, g, precision: str) -> dict:
    """The same staged step in the other precision (SURVEY §7 'report both'): a short timed run
    after the headline's timed region. fp64 is the parity precision (tests/test_gpu_f32_staged.py:
    1000-step drift vs the oracle < 1e-4); fp32 is faster but misses that bar (median drift 3e-4
    at step 1000), so it is reported here and never as the headline."""
    from mujoco_gymnasium_environments_amd.envs.soccer import SoccerVectorEnv
    env = SoccerVectorEnv(N, device=str(dev), precision=precision, seed=1234, staged=True, banks=args.banks)
    pool = [(torch.rand(N, env.model.nu, device=dev, generator=g) * 300.0 - 150.0).contiguous() for _ in range(4)]
    env.reset()
    for k in range(5):
        env.step(pool[k % 4])
    torch.cuda.synchronize(dev)
    steps = 20
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record()
    for k in range(steps):
        env.step(pool[k % 4])
    b.record()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    note = ("parity precision (tests/test_gpu_f32_staged.py: 1000-step drift vs the oracle < 1e-4)"
            if precision == "f64" else
            "fast precision; misses the north_star 1e-4 drift bar over 1000 steps (median 3e-4, DESIGN.md §2)")
    return {"value": round(N * steps / el, 1), "unit": "env_steps/s", "ms_per_step": round(el / steps * 1e3, 4),
            "launch_ms": round(a.elapsed_time(b) / steps, 4), "steps": steps, "dtype": precision, "note": note}


def spawn_ranks(n: int, argv) -> int:
    """``--gpus N`` without an outer launcher: start N rank processes of this script, one per GPU
    (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1), the way
    ``torch.distributed.run --nproc-per-node N`` would, and wait for them. Called before anything
    touches the GPU (the parent never initialises HIP); rank 0 prints the one JSON line. Returns
    the first non-zero exit status of the ranks (0 when every rank succeeded)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def cpu_harness(args, world: int, rank: int, dist) -> None:
    """``--harness cpu``: bench.py's multi-rank machinery (spawn, rendezvous, env shards, timed
    region, SUM / MAX reduction, rank-0 JSON line) with gloo and the oracle soccer env standing in
    for RCCL and the GPU step, so the N-rank path is testable on a CPU-only host
    (tests/test_distributed_cpu.py). Not a benchmark: the line says so in its `data` field."""
    from mujoco_gymnasium_environments_amd.distributed import env_offset
    n = args.envs
    envs = [OracleSoccerEnv(env_offset(rank, n) + i, seed=5) for i in range(n)]
    acts = np.random.default_rng(0).uniform(-150, 150, (max(1, args.steps + args.warmup), envs[0].m.nu))
    acts = acts.astype(np.float32)
    acc = torch.zeros(6, dtype=torch.float64)

    def step(k):
        for e in envs:
            r, term, trunc = e.step(acts[k])
            acc[0] += 1
            acc[2] += r
            acc[3] += term
            acc[4] += trunc
    for k in range(args.warmup):
        step(k)
    acc.zero_()
    elapsed = timed_region(lambda k: step(args.warmup + k), args.steps, lambda: None, dist)
    acc, elapsed, value = whole_job_value(acc, elapsed)
    if rank == 0:
        print(json.dumps({
            "metric": METRIC, "value": round(value, 3), "unit": "env_steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / max(args.steps, 1) * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "cpu harness: oracle soccer env, gloo (tests only, not a measurement)",
            "config": {"workload": "harness", "envs_per_gpu": n, "global_batch": n * world,
                       "parallelism": f"dp{world} (env shards)", "env_steps_total": int(acc[0].item())}}))
    if dist:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without an outer torch.distributed.run, bench.py starts them itself")
    ap.add_argument("--harness", default="gpu", choices=["gpu", "cpu"], help=argparse.SUPPRESS)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--envs", type=int, default=0, help="envs per GPU (default 4096; 8192 for bipedal)")
    # soccer's headline precision is fp64: the precision that meets the north_star accuracy bar
    # (qpos drift < 1e-4 over 1000 steps vs the fp64 oracle); fp32 rides along as an extra key
    ap.add_argument("--precision", default=None, choices=["f32", "f64"],
                    help="default: f64 (MuJoCo's mjtNum, the parity precision) for every task")
    ap.add_argument("--cpu-envs", type=int, default=16)
    ap.add_argument("--cpu-steps", type=int, default=2000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mono", action="store_true", help="monolithic one-wave-per-env kernel instead of the staged step")
    ap.add_argument("--banks", type=int, default=3, help="reset banks per env (3: measured fastest, DESIGN.md §4)")
    ap.add_argument("--full-capacity", action="store_true",
                    help="soccer: 96 contacts / 384 rows per env (the default since round 5; kept for old scripts)")
    ap.add_argument("--reduced-capacity", action="store_true",
                    help="soccer: the round-1 capacity, 64 contacts / 192 rows, rows beyond it dropped and counted")
    ap.add_argument("--streams", type=int, default=None,
                    help="soccer / parkour / bipedal: split the rank's envs into this many stream shards, each "
                         "its own staged pipeline on its own HIP stream (envs/sharded.py); default 4 for "
                         "parkour (145.9k -> 159.6k env-steps/s), 2 for bipedal (206.6k -> 243.4k; "
                         "profiles/r06_stream_shards_ab.json), else 1")
    ap.add_argument("--sub-batches", type=int, default=1,
                    help="parkour / bipedal: step the rank's envs as this many sub-batches one after another "
                         "on one stream (envs/sharded.py serial shards: one sub-batch's B live in the "
                         "Infinity Cache at a time)")
    ap.add_argument("--no-f64-line", "--no-other-line", dest="no_f64_line", action="store_true",
                    help="skip the other-precision soccer line (fp32 when the headline is fp64)")
    ap.add_argument("--mix-streams", type=int, default=4, help="mixed: 4 grouped streams (default) or 7 (one per task)")
    ap.add_argument("--mix-priority", type=int, default=1, help="mixed: construction's stream at high priority (1)")
    ap.add_argument("--mix-staged", type=int, default=1,
                    help="mixed: parkour and bipedal on their staged pipelines (1) or one wave per env (0)")
    ap.add_argument("--task", default="soccer", choices=["soccer", "parkour", "bipedal", "mixed", "assembly",
                                                          "construction"])
    args = ap.parse_args()
    if args.streams is None:
        args.streams = {"parkour": 4, "bipedal": 2}.get(args.task, 1) if args.sub_batches <= 1 else 1
    from mujoco_gymnasium_environments_amd.distributed import env_offset, reduce_rollout, world_from_env
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        # no outer launcher: one child process per GPU, started before any GPU call
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world, rank, local = world_from_env()
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (launch one rank per GPU)")
    if args.harness == "cpu":
        dist = None
        if world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo")
        args.envs = args.envs if args.envs > 0 else 2
        return cpu_harness(args, world, rank, dist)
    if args.task not in ("soccer", "bipedal", "parkour"):
        args.mono = True  # one fused wave-per-env launch per step
    if args.precision is None:
        args.precision = "f64"
    if args.envs <= 0:
        args.envs = {"bipedal": 8192, "mixed": 1024, "assembly": 1024, "construction": 1024}.get(args.task, 4096)

    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    N = args.envs
    if args.task == "mixed":
        return bench_mixed(args, dev, world, rank, dist)
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    if args.task == "parkour":
        from mujoco_gymnasium_environments_amd.envs.parkour import ParkourVectorEnv, action_limits
        env = sharded(args, N, dev, lambda n, off: ParkourVectorEnv(
            n, device=str(dev), precision=args.precision, seed=1234, env_offset=env_offset(rank, N) + off,
            staged=not args.mono, banks=min(args.banks, 1) if args.banks > 0 else 0))
        lim = torch.as_tensor(action_limits(), dtype=torch.float32, device=dev)
        pool = [((torch.rand(N, 16, device=dev, generator=g) * 2 - 1) * lim).contiguous() for _ in range(16)]
    elif args.task == "bipedal":
        from mujoco_gymnasium_environments_amd.envs.bipedal import BipedalVectorEnv
        env = sharded(args, N, dev, lambda n, off: BipedalVectorEnv(
            n, device=str(dev), precision=args.precision, seed=1234, env_offset=env_offset(rank, N) + off,
            staged=not args.mono, banks=min(args.banks, 1) if args.banks > 0 else 0))
        pool = [((torch.rand(N, 26, device=dev, generator=g) * 2 - 1) * 100.0).contiguous() for _ in range(16)]
    elif args.task == "assembly":
        from mujoco_gymnasium_environments_amd.envs.assembly import AssemblyVectorEnv
        args.precision = "f64"  # fp64 only (envs/assembly.py)
        env = AssemblyVectorEnv(N, device=str(dev), precision="f64")
        alo = torch.tensor([-2.0] * 7 + [0.0, 0.0], device=dev)
        alim = torch.tensor([4.0] * 7 + [100.0, 50.0], device=dev)
        pool = [(torch.rand(N, 9, device=dev, generator=g) * alim + alo).contiguous() for _ in range(16)]
    elif args.task == "construction":
        from mujoco_gymnasium_environments_amd.envs.construction import ConstructionVectorEnv
        args.precision = "f64"  # fp64 (its parity tests and the mixed run use fp64)
        env = ConstructionVectorEnv(N, device=str(dev), precision="f64", seed=1234, env_offset=env_offset(rank, N))
        pool = [((torch.rand(N, 33, device=dev, generator=g) * 2 - 1) * 200.0).contiguous() for _ in range(16)]
    else:
        from mujoco_gymnasium_environments_amd.envs.soccer import SoccerVectorEnv
        if args.streams > 1:
            from mujoco_gymnasium_environments_amd.envs.soccer import StreamShardedSoccerEnv
            env = StreamShardedSoccerEnv(N, args.streams, device=str(dev), precision=args.precision, seed=1234,
                                         env_offset=env_offset(rank, N), staged=not args.mono, banks=args.banks)
        else:
            env = SoccerVectorEnv(N, device=str(dev), precision=args.precision, seed=1234,
                                  env_offset=env_offset(rank, N), staged=not args.mono, banks=args.banks,
                                  full_capacity=not (args.reduced_capacity or args.mono))
        pool = [(torch.rand(N, env.model.nu, device=dev, generator=g) * 300.0 - 150.0).contiguous() for _ in range(16)]
    env.reset()
    for k in range(args.warmup):
        env.step(pool[k % len(pool)])
    torch.cuda.synchronize(dev)
    # rollout metrics accumulate inside the kernel (env.rollout); read once after the timed region
    acc = torch.zeros(6, dtype=torch.float64, device=dev)  # env_steps, episodes, reward, term, trunc, bad
    shards = getattr(env, "shards", [env])  # StreamShardedSoccerEnv: per-shard metric buffers
    for e in shards:
        e.rollout.zero_()
        e.batch.overflow.zero_()
    ep0 = sum(int(e.episode.sum().item()) for e in shards)
    warn0 = sum(int(e.batch.warning.sum().item()) for e in shards)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    def one_step(k):
        ev[k][0].record()
        env.step(pool[k % len(pool)])
        ev[k][1].record()
    elapsed = timed_region(one_step, args.steps, lambda: torch.cuda.synchronize(dev), dist)
    launch_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    ro = torch.cat([e.rollout for e in shards]).double().sum(0)
    acc[0] = ro[3]
    acc[1] = float(sum(int(e.episode.sum().item()) for e in shards) - ep0)
    acc[2], acc[3], acc[4] = ro[0], ro[1], ro[2]
    acc[5] = float(sum(int(e.batch.warning.sum().item()) for e in shards) - warn0)  # over the timed region
    overflow_steps = sum(int(e.batch.overflow.sum().item()) for e in shards)
    acc, elapsed, value = whole_job_value(acc, elapsed)  # end-of-rollout metric all-reduce (RCCL), max time
    total_steps = acc[0].item()
    if rank == 0 and args.task == "bipedal":
        bytes_per_launch = (BIPEDAL_ALG_BYTES_F64 if args.precision == "f64" else BIPEDAL_ALG_BYTES) * N
        bmode = "mono" if args.mono else "staged"
        achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
        out = {
            "metric": BIPEDAL_METRIC, "value": round(value, 1), "unit": "env_steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "data": "synthetic (U(-100,100) actions, Philox reset draws)",
            "config": {"workload": "bipedal_rescue_env, 8192 envs/GPU (BASELINE configs[3])", "envs_per_gpu": N,
                       "global_batch": N * world, "parallelism": f"dp{world} (env shards)", "autoreset": "same-step",
                       "integrator": "RK4", "step_kernels": bmode, "stream_shards": args.streams,
                       "sub_batches": args.sub_batches,
                       "episodes_started": int(acc[1].item()),
                       "terminated_total": int(acc[3].item()), "bad_state_resets": int(acc[5].item()),
                       "termination_rate": round(acc[3].item() / total_steps, 5),
                       "bad_state_rate": round(acc[5].item() / total_steps, 5),
                       "capacity_overflow_steps": overflow_steps,
                       "mean_reward": _finite(acc[2].item() / total_steps)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": _pmc_traffic(PMC_PROFILE_BIPEDAL, N, args.precision,
                                                                                  bmode),
                         "kernel": ("mgx_bipedal_step = 4 x (k_rk_rows + k_pgs_groups + k_rk_finish) + k_rk_settle"
                                    if bmode == "staged" else "mgx_bipedal_step = k_bipedal<T,0,GB>"),
                         "alg_bytes_per_step": bytes_per_launch, "launch_ms": round(launch_ms, 4)},
        }
        if not args.no_f64_line:
            other = "f32" if args.precision == "f64" else "f64"
            out[f"{other}_line"] = bipedal_other_line(args, dev, N, g, other)
        if not args.no_cpu_baseline and world == 1:  # the CPU leg: rank 0 at N = 1 only
            out["cpu_baseline"] = cpu_baseline_bipedal(max(1, args.cpu_envs // 8), args.cpu_steps // 10)
        print(json.dumps(out))
    elif rank == 0 and args.task == "assembly":
        bytes_per_launch = ASSEMBLY_ALG_BYTES * N
        achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
        out = {
            "metric": ASSEMBLY_METRIC, "value": round(value, 1), "unit": "env_steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "data": "synthetic (uniform actions over action_space; deterministic reset)",
            "config": {"workload": "robotic_arm_assembly_env, 1024 envs/GPU (BASELINE configs[4] task)",
                       "envs_per_gpu": N, "global_batch": N * world, "parallelism": f"dp{world} (env shards)",
                       "autoreset": "same-step (10 settle steps)", "substeps_per_step": 10, "solver": "Newton",
                       "step_kernels": "mono",
                       "episodes_started": int(acc[1].item()), "terminated_total": int(acc[3].item()),
                       "bad_state_resets": int(acc[5].item()), "capacity_overflow_steps": overflow_steps,
                       "mean_reward": _finite(acc[2].item() / total_steps)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": _pmc_traffic(PMC_PROFILE_ASSEMBLY, N, args.precision, "mono"),
                         "kernel": "mgx_assembly_step = k_assembly<T,0,GB>", "alg_bytes_per_step": bytes_per_launch,
                         "launch_ms": round(launch_ms, 4)},
        }
        if not args.no_cpu_baseline and world == 1:  # the CPU leg: rank 0 at N = 1 only
            out["cpu_baseline"] = cpu_baseline_assembly(2, max(5, args.cpu_steps // 2))
        print(json.dumps(out))
    elif rank == 0 and args.task == "construction":
        bytes_per_launch = CONSTRUCTION_ALG_BYTES * N
        achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
        out = {
            "metric": "env steps/sec (whole node), humanoid_construction 1024 envs/GPU (RK4 + Newton, nv 99)",
            "value": round(value, 1), "unit": "env_steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (U(-200,200) actions, Philox task / weather draws)",
            "config": {"workload": "humanoid_construction_env, 1024 envs/GPU (BASELINE configs[4] task)",
                       "envs_per_gpu": N, "global_batch": N * world, "parallelism": f"dp{world} (env shards)",
                       "autoreset": "same-step", "integrator": "RK4", "solver": "Newton",
                       "step_kernels": "wide (two dofs per lane)",
                       "episodes_started": int(acc[1].item()), "terminated_total": int(acc[3].item()),
                       "bad_state_resets": int(acc[5].item()), "capacity_overflow_steps": overflow_steps,
                       "mean_reward": _finite(acc[2].item() / total_steps)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": _pmc_traffic(PMC_PROFILE_CONSTRUCTION, N, "f64", "wide (two dofs per lane)"),
                         "profile": f"profiles/{PMC_PROFILE_CONSTRUCTION}",
                         "kernel": "mgx_construction_step = k_construction<double,0>",
                         "alg_bytes_per_step": bytes_per_launch, "launch_ms": round(launch_ms, 4)},
        }
        print(json.dumps(out))
    elif rank == 0 and args.task == "parkour":
        bytes_per_launch = (PARKOUR_ALG_BYTES_F64 if args.precision == "f64" else PARKOUR_ALG_BYTES) * N
        achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
        out = {
            "metric": PARKOUR_METRIC, "value": round(value, 1), "unit": "env_steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "data": "synthetic (U(-lim,lim) actions per joint, Philox reset draws)",
            "config": {"workload": "quadruped_parkour_env, 4096 envs/GPU (BASELINE configs[1])", "envs_per_gpu": N,
                       "global_batch": N * world, "parallelism": f"dp{world} (env shards)", "autoreset": "same-step",
                       "substeps_per_step": 10, "step_kernels": "mono" if args.mono else "staged",
                       "stream_shards": args.streams, "sub_batches": args.sub_batches,
                       "episodes_started": int(acc[1].item()),
                       "terminated_total": int(acc[3].item()), "bad_state_resets": int(acc[5].item()),
                       "termination_rate": round(acc[3].item() / total_steps, 5),
                       "bad_state_rate": round(acc[5].item() / total_steps, 5),
                       "capacity": "96 contacts / 384 rows", "capacity_overflow_steps": overflow_steps,
                       "mean_reward": _finite(acc[2].item() / total_steps)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": _pmc_traffic(PMC_PROFILE_PARKOUR, N, args.precision, "mono" if args.mono else "staged"),
                         "kernel": ("mgx_parkour_step = k_parkour<T,0,GB>" if args.mono else
                                    "mgx_parkour_step = 10 x (k_pk_rows + k_pgs_groups + k_pk_bank_finish + k_pk_finish)"
                                    " + k_pk_settle (fixups)"),
                         "alg_bytes_per_step": bytes_per_launch,
                         "launch_ms": round(launch_ms, 4)},
        }
        if not args.no_cpu_baseline and world == 1:  # the CPU leg: rank 0 at N = 1 only
            out["cpu_baseline"] = cpu_baseline_parkour(max(1, args.cpu_envs // 4), args.cpu_steps // 4)
        print(json.dumps(out))
    elif rank == 0:
        alg = ALG_BYTES_PER_ENV_STEP_F64 if args.precision == "f64" else ALG_BYTES_PER_ENV_STEP
        bytes_per_launch = alg * N
        achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
        mode = "mono" if args.mono else "staged"
        traffic = _pmc_traffic(PMC_PROFILE[args.precision], N, args.precision, mode)
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "env_steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "data": "synthetic (U(-150,150) actions, Philox reset draws)",
            "config": {"workload": "humanoid_soccer_env, 4096 envs/GPU (BASELINE configs[2])",
                       "envs_per_gpu": N, "global_batch": N * world, "parallelism": f"dp{world} (env shards)",
                       "autoreset": "same-step", "step_kernels": mode, "reset_banks": 0 if args.mono else args.banks,
                       "stream_shards": args.streams,
                       "episodes_started": int(acc[1].item()),
                       "terminated_total": int(acc[3].item()), "bad_state_resets": int(acc[5].item()),
                       "termination_rate": round(acc[3].item() / total_steps, 5),
                       "bad_state_rate": round(acc[5].item() / total_steps, 5),
                       "capacity_overflow_steps": overflow_steps,
                       "capacity": "64 contacts / 192 rows" if (args.reduced_capacity or args.mono) else "96 contacts / 384 rows",
                       "mean_reward": _finite(acc[2].item() / total_steps)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": ("mgx_soccer_step = k_soccer_rows + k_pgs_groups + k_soccer_bank_finish + "
                                    "k_soccer_finish + k_soccer_settle (fixups)" if mode == "staged" else "mgx_soccer_step = k_soccer<T,0>"),
                         "profile": f"profiles/{PMC_PROFILE[args.precision]}",
                         "alg_bytes_per_step": bytes_per_launch, "launch_ms": round(launch_ms, 4),
                         "note": "achieved = algorithmic bytes of one env step x envs / HIP-event time of the "
                                 "step's launches; traffic = PMC HBM bytes of those launches per step"},
        }
        fl = soccer_flops(ro.cpu(), env.model.nv)
        tf = fl["flops_per_env_step"] * N / (launch_ms * 1e-3) / 1e12
        out["roofline_flops"] = {"bound": "valu", "achieved": round(tf, 4), "peak": VALU_PEAK_TFLOPS[args.precision],
                                 "unit": "TFLOP/s", "frac": tf / VALU_PEAK_TFLOPS[args.precision],
                                 "flops_per_env_step": round(fl["flops_per_env_step"]),
                                 "nefc_mean": round(fl["nefc_mean"], 2), "pgs_sweeps_mean": round(fl["pgs_sweeps_mean"], 2),
                                 "definition": "SURVEY 8(d) dense-equivalent: 2 nefc^2 nv (A) + 2 sweeps nefc^2 (PGS) "
                                               "+ 300 nbody, summed per env step in the kernel"}
        if not args.no_f64_line and world == 1 and not args.mono and args.streams == 1:
            other = "f32" if args.precision == "f64" else "f64"
            out[f"{other}_line"] = other_precision_line(args, dev, N, g, other)
        if not args.no_cpu_baseline and world == 1:  # the CPU leg: rank 0 at N = 1 only
            out["cpu_baseline"] = cpu_baseline(args.cpu_envs, args.cpu_steps)
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
