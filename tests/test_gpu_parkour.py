"""GPU: the fused quadruped_parkour kernel (10 physics substeps + env logic) against the
reference golden vectors and the CPU oracle (mjref physics + oracle/parkour_logic.py).

Bars: logic kernel fp64 — obs, reward, episode reward, flags, counters and reached-mask
bit-exact against the reference's own step() outputs, obstacle-motor ctrl to 1 ulp (device
sin vs numpy sin); fp32 — obs atol 2e-5, reward rtol 1e-5
+ 0.5, flags exact. End-to-end fp64 (reset with numpy-seeded draws + 40 steps = 400 substeps):
obs atol 1e-5, reward atol 1e-3 and identical terminated/truncated flags per step.
"""
import ctypes as C

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _t(x, dtype, dev="cuda:0"):
    return torch.as_tensor(np.ascontiguousarray(x)).to(device=dev, dtype=dtype).contiguous()


@pytest.mark.parametrize("prec", ["f64", "f32", "f64_actions"])
def test_parkour_logic_kernel_matches_reference(parkour_model, prec):
    from mujoco_gymnasium_environments_amd import cabi
    from mujoco_gymnasium_environments_amd.envs.parkour import ParkourVectorEnv
    from mujoco_gymnasium_environments_amd.native import check, lib
    # f64_actions: the fp64 kernel on the float64-action vectors (make_fixtures.py main_f64),
    # mgx_parkour_env.action_f64 = 1 — the reference keeps a float64 action float64 through np.clip
    act64 = prec == "f64_actions"
    prec = "f64" if act64 else prec
    g = dict(np.load("tests/golden/parkour_envlogic" + ("_f64" if act64 else "") + ".npz"))
    n = g["obs"].shape[0]
    env = ParkourVectorEnv(n, precision=prec, autoreset=False)
    dt = env.batch.dtype
    mc = g["con_geom"].shape[1]
    env.last_position.copy_(_t(g["last_position_in"], dt))
    env.max_progress.copy_(_t(g["max_progress_in"], dt))
    env.episode_reward.copy_(_t(g["episode_reward_in"], torch.float64))
    env.er_kind.zero_()
    env.reached.copy_(_t(g["reached_in"], torch.int32))
    env.fall_count.copy_(_t(g["fall_count_in"], torch.int32))
    env.stuck.copy_(_t(g["stuck_in"], torch.int32))
    env.step_count.copy_(_t(g["step_count_in"], torch.int32))
    T = dict(qpos=_t(g["qpos"], dt), qvel=_t(g["qvel"], dt), xpos=_t(g["xpos"], dt),
             ncon=_t(g["ncon"], torch.int32), con_geom=_t(np.maximum(g["con_geom"], -1), torch.int32),
             ctrl=_t(g["ctrl_in"], dt), action=_t(g["action"], torch.float64 if act64 else torch.float32),
             obs=torch.zeros(n, 95, dtype=torch.float32, device="cuda:0"),
             reward=torch.zeros(n, dtype=torch.float64, device="cuda:0"),
             term=torch.zeros(n, dtype=torch.uint8, device="cuda:0"),
             trunc=torch.zeros(n, dtype=torch.uint8, device="cuda:0"))
    io = cabi.MgxParkourLogicIO(T["qpos"].data_ptr(), T["qvel"].data_ptr(), T["xpos"].data_ptr(),
                                T["ncon"].data_ptr(), T["con_geom"].data_ptr(), mc, 0, T["ctrl"].data_ptr(),
                                T["action"].data_ptr(), T["obs"].data_ptr(), T["reward"].data_ptr(),
                                T["term"].data_ptr(), T["trunc"].data_ptr())
    env._env.action_f64 = 1 if act64 else 0
    check(lib().mgx_parkour_logic_test(env.native.handle, C.byref(io), C.byref(env._env), n, None), "logic_test")
    torch.cuda.synchronize()
    obs, rew = T["obs"].cpu().numpy(), T["reward"].cpu().numpy()
    np.testing.assert_array_equal(T["term"].cpu().numpy().astype(bool), g["terminated"])
    np.testing.assert_array_equal(T["trunc"].cpu().numpy().astype(bool), g["truncated"])
    np.testing.assert_array_equal(env.reached.cpu().numpy(), g["reached_out"])
    np.testing.assert_array_equal(env.fall_count.cpu().numpy(), g["fall_count_out"])
    np.testing.assert_array_equal(env.stuck.cpu().numpy(), g["stuck_out"])
    np.testing.assert_array_equal(env.step_count.cpu().numpy(), g["step_count_out"])
    if prec == "f64":
        np.testing.assert_array_equal(obs, g["obs"])
        np.testing.assert_array_equal(rew, g["reward"])
        np.testing.assert_array_equal(env.episode_reward.cpu().numpy(), g["episode_reward_out"])
        # obstacle motors 50 sin(0.5 t): the device sin may differ from numpy's by 1 ulp
        np.testing.assert_allclose(T["ctrl"].cpu().numpy(), g["ctrl_out"], rtol=1e-15, atol=1e-13)
        np.testing.assert_array_equal(env.max_progress.cpu().numpy(), g["max_progress_out"])
        np.testing.assert_array_equal(env.last_position.cpu().numpy(), g["last_position_out"])
    else:
        np.testing.assert_allclose(obs, g["obs"], atol=2e-5, rtol=1e-6)
        np.testing.assert_allclose(rew, g["reward"], rtol=1e-5, atol=0.5)
        np.testing.assert_allclose(T["ctrl"].cpu().numpy(), g["ctrl_out"], rtol=1e-6, atol=1e-5)


class _OracleParkour:
    """CPU oracle of one parkour env: mjref physics + numpy logic, reset from explicit draws."""

    def __init__(self, packed, tables, draws):
        from oracle.mjref import RefSim
        from oracle.parkour_logic import ParkourLogic, ParkourTables
        self.sim = RefSim(packed)
        self.L = ParkourLogic(ParkourTables(packed.model))
        self.s = {}
        self.reset(draws)

    def view(self):
        sim, s = self.sim, self.s
        c = sim.contacts()
        s.update(qpos=sim.qpos, qvel=sim.qvel, ctrl=sim.ctrl, xpos=sim.xpos.reshape(-1, 3),
                 con_geom=c["geom"], ncon=int(sim.ncon[0]))

    def reset(self, draws):
        self.sim.reset()
        self.view()
        self.L.apply_reset(self.s, draws)
        self.sim.step(10)
        self.view()
        return self.L.obs(self.s)

    def step(self, action):
        a = self.L.pre(self.s, action)
        self.sim.step(10)
        self.view()
        return self.L.post(self.s, a)


@pytest.mark.parametrize("staged", [True, False])
def test_parkour_end_to_end_f64_matches_oracle(parkour_model, staged):
    """staged=True (the default): per substep row builder -> lane-group PGS -> finisher, the reset
    settled by the same stages; staged=False: one wave per env for the whole env step."""
    from mujoco_gymnasium_environments_amd import cabi
    from mujoco_gymnasium_environments_amd.envs.parkour import ParkourVectorEnv, action_limits
    from mujoco_gymnasium_environments_amd.seeding import np_random
    n = 4
    env = ParkourVectorEnv(n, precision="f64", autoreset=False, staged=staged)
    draws = np.stack([env.tables.reset_draws(np_random(100 + i)[0]) for i in range(n)])
    obs, _ = env.reset(draws=draws)
    packed = cabi.pack_model(parkour_model)
    oracles = [_OracleParkour(packed, env.tables, draws[i]) for i in range(n)]
    o0 = obs.cpu().numpy()
    for i in range(n):
        np.testing.assert_allclose(o0[i], oracles[i].L.obs(oracles[i].s), atol=1e-6, err_msg=f"reset obs env {i}")
    rng = np.random.default_rng(5)
    lim = action_limits()
    for k in range(40):
        act = (rng.uniform(-1, 1, (n, 16)) * lim * 0.05).astype(np.float32)
        obs, rew, term, trunc, _ = env.step(_t(act, torch.float32))
        torch.cuda.synchronize()
        ob, rw = obs.cpu().numpy(), rew.cpu().numpy()
        te, tr = term.cpu().numpy().astype(bool), trunc.cpu().numpy().astype(bool)
        for i in range(n):
            o, r, t1, t2 = oracles[i].step(act[i])
            np.testing.assert_allclose(ob[i], o, atol=1e-5, err_msg=f"obs env {i} step {k}")
            assert abs(rw[i] - r) < 1e-3, (i, k, rw[i], r)
            assert te[i] == t1 and tr[i] == t2, (i, k)


def test_parkour_autoreset_and_sharding_invariance():
    """Global env index keys the reset draws: a 2-env shard at offset 2 reproduces envs 2..3
    of a 4-env run bit for bit, through terminations and same-step autoresets."""
    from mujoco_gymnasium_environments_amd.envs.parkour import ParkourVectorEnv, action_limits
    full = ParkourVectorEnv(4, precision="f32", seed=9, max_episode_steps=7)
    shard = ParkourVectorEnv(2, precision="f32", seed=9, max_episode_steps=7, env_offset=2)
    full.reset()
    shard.reset()
    rng = np.random.default_rng(3)
    lim = action_limits()
    ends = 0
    for k in range(20):
        act = (rng.uniform(-1, 1, (4, 16)) * lim).astype(np.float32)
        fo, fr, ft, fu, _ = full.step(_t(act, torch.float32))
        so, sr, st, su, _ = shard.step(_t(act[2:], torch.float32))
        torch.cuda.synchronize()
        assert torch.equal(fo[2:], so) and torch.equal(fr[2:], sr)
        assert torch.equal(ft[2:], st) and torch.equal(fu[2:], su)
        ends += int((fu | ft).sum())
    assert ends >= 8  # truncation at 7 steps forces same-step autoresets
    assert int(full.episode.min()) >= 3
    assert torch.isfinite(full.obs).all()


def test_parkour_f32_rollout_finite_and_counted():
    from mujoco_gymnasium_environments_amd.envs.parkour import ParkourVectorEnv, action_limits
    n = 256
    env = ParkourVectorEnv(n, precision="f32", seed=1)
    env.reset()
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0)
    lim = torch.as_tensor(action_limits(), dtype=torch.float32, device="cuda:0")
    for _ in range(50):
        a = (torch.rand(n, 16, device="cuda:0", generator=g) * 2 - 1) * lim
        env.step(a)
    torch.cuda.synchronize()
    assert torch.isfinite(env.obs).all() and torch.isfinite(env.reward).all()
    assert int(env.rollout[:, 3].sum()) == 50 * n


def _pk_trajectory(n, banks, steps, staged=True, max_steps=3, seed=9):
    from mujoco_gymnasium_environments_amd.envs.parkour import ParkourVectorEnv, action_limits
    env = ParkourVectorEnv(n, precision="f64", seed=seed, max_episode_steps=max_steps, staged=staged, banks=banks)
    o, _ = env.reset()
    out = [o.cpu().numpy().copy()]
    lim = torch.as_tensor(action_limits(), dtype=torch.float32, device="cuda:0")
    g = torch.Generator(device="cuda:0")
    g.manual_seed(5)
    for _ in range(steps):
        a = ((torch.rand(n, 16, device="cuda:0", generator=g) * 2 - 1) * lim).contiguous()
        obs, rew, term, trunc, _ = env.step(a)
        out.append(np.concatenate([obs.cpu().numpy().ravel(), rew.cpu().numpy().ravel(),
                                   term.cpu().numpy().ravel().astype(np.float64),
                                   trunc.cpu().numpy().ravel().astype(np.float64),
                                   env.batch.qpos.cpu().numpy().ravel()]))
    torch.cuda.synchronize()
    return out, env.episode.cpu().numpy().copy(), int(env.batch.warning.sum())


@pytest.mark.parametrize("banks", [1, 2])
def test_parkour_bank_count_does_not_change_trajectories(banks):
    """Staged step: the bank count is a performance knob only. banks = 0 (every autoreset settled
    by k_pk_settle in one wave) and banks = R (settled banks installed; with 3-step episodes every
    env resets every third step) give the same trajectories bit for bit."""
    ref, e0, w0 = _pk_trajectory(8, 0, 12)
    got, e1, w1 = _pk_trajectory(8, banks, 12)
    assert int(e0.sum()) >= 8 * 4
    for t, (x, y) in enumerate(zip(ref, got)):
        np.testing.assert_array_equal(x, y, err_msg=f"step {t}")
    np.testing.assert_array_equal(e0, e1)
    assert w0 == w1


def test_parkour_end_to_end_f64_bench_actions(parkour_model):
    """Bench conditions (BASELINE configs[1]): U(-lim, lim) actions over the full action space, the
    staged fp64 step of 8 envs x 25 steps against the oracle for as long as the oracle determines the
    trajectory. Two twins run beside the oracle — the free joint's position perturbed by 1e-12 after
    the reset, and the PGS residuals summed in reverse order (another fp64 rounding of the same
    solve). While the larger twin spread is <= 1e-6 the device must be within max(1e-6, 20 x spread)
    of the oracle (qpos, qvel relative to max(1, |x|)), the reward within 1e-3 and the flags exact."""
    from mujoco_gymnasium_environments_amd import cabi
    from mujoco_gymnasium_environments_amd.envs.parkour import ParkourVectorEnv, action_limits
    from mujoco_gymnasium_environments_amd.seeding import np_random
    m = parkour_model
    n, steps = 8, 25
    env = ParkourVectorEnv(n, precision="f64", autoreset=False)
    draws = np.stack([env.tables.reset_draws(np_random(300 + i)[0]) for i in range(n)])
    env.reset(draws=draws)
    packed = cabi.pack_model(m)
    free = [int(m.jnt_qposadr[j]) + k for j in range(m.njnt) if int(m.jnt_type[j]) == 0 for k in range(3)]
    runs = []
    for i in range(n):
        trio = [_OracleParkour(packed, env.tables, draws[i]) for _ in range(3)]
        trio[1].sim.qpos[free] += np.random.default_rng(i).normal(scale=1e-12, size=len(free))
        trio[2].sim.set_pgs_reverse(True)
        runs.append(trio)

    def err(q, v, o):
        x = np.concatenate([o.sim.qpos, o.sim.qvel])
        return float(np.max(np.abs(x - np.concatenate([q, v])) / np.maximum(1.0, np.abs(x))))

    rng = np.random.default_rng(7)
    lim = action_limits()
    live = set(range(n))
    horizon = np.zeros(n, dtype=int)
    worst = np.zeros(n)
    for k in range(steps):
        act = (rng.uniform(-1, 1, (n, 16)) * lim).astype(np.float32)
        obs, rew, term, trunc, _ = env.step(_t(act, torch.float32))
        torch.cuda.synchronize()
        rw, te, tr = rew.cpu().numpy(), term.cpu().numpy().astype(bool), trunc.cpu().numpy().astype(bool)
        qg, vg = env.batch.qpos.cpu().numpy(), env.batch.qvel.cpu().numpy()
        for i in sorted(live):
            out = [o.step(act[i]) for o in runs[i]]
            o = runs[i][0]
            spread = max(err(x.sim.qpos, x.sim.qvel, o) for x in runs[i][1:])
            if spread > 1e-6:
                live.discard(i)
                continue
            e = err(qg[i], vg[i], o)
            assert e <= max(1e-6, 20 * spread), (k, i, e, spread)
            _, r, t1, t2 = out[0]
            assert abs(rw[i] - r) < 1e-3, (i, k, rw[i], r)
            assert te[i] == t1 and tr[i] == t2, (i, k)
            horizon[i] += 1
            worst[i] = max(worst[i], e)
            if t1 or t2:
                live.discard(i)
    print(f"\nparkour U(+-lim): steps compared per env {horizon.tolist()}; "
          f"worst device error {[f'{w:.1e}' for w in worst]}")
    assert horizon.min() >= 2 and horizon.sum() >= 50, horizon


def test_parkour_stream_shards_equal_single_batch():
    """StreamShardedParkourEnv (3 shards on 3 HIP streams, ragged sizes) reproduces one
    ParkourVectorEnv over the same envs bit for bit at bench conditions (fp64, U(-lim, lim)
    actions, the heavy exploding-state slots and their same-step resets): the shards only
    partition the launches."""
    from mujoco_gymnasium_environments_amd.envs.parkour import (ParkourVectorEnv, StreamShardedParkourEnv,
                                                                action_limits)
    n = 190
    one = ParkourVectorEnv(n, precision="f64", seed=21)
    sh = StreamShardedParkourEnv(n, 3, precision="f64", seed=21)
    assert [b - a for a, b in sh.bounds] == [64, 63, 63]
    o1, _ = one.reset()
    o2, _ = sh.reset()
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    lim = torch.as_tensor(action_limits(), dtype=torch.float32, device="cuda:0")
    g = torch.Generator(device="cuda:0")
    g.manual_seed(13)
    for t in range(60):
        a = ((torch.rand(n, 16, device="cuda:0", generator=g) * 2 - 1) * lim).contiguous()
        s1 = one.step(a)
        s2 = sh.step(a)
        for x, y, name in zip(s1[:4], s2[:4], ("obs", "reward", "terminated", "truncated")):
            assert torch.equal(x, y), (t, name)
    torch.cuda.synchronize()
    assert torch.equal(one.episode, sh.episode) and torch.equal(one.final_obs, sh.final_obs)
    assert torch.equal(one.batch.qpos, torch.cat([s.batch.qpos for s in sh.shards]))
    assert torch.equal(one.checkpoints_reached(), sh.checkpoints_reached())
    assert torch.equal(one.info()["fall_count"], sh.info()["fall_count"])
    assert int(one.batch.warning.sum()) == sum(int(s.batch.warning.sum()) for s in sh.shards)
