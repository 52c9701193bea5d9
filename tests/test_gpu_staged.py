"""GPU: the staged soccer step (row builder -> lane-group PGS -> finisher, reset banks) against
the monolithic one-wave-per-env kernel and the CPU oracle.

Tolerances (fp64): staged vs monolithic steps differ only in the solver's summation order ->
obs atol 1e-7 over 30 moderate-action steps with identical flags; a reset installed from a bank
equals a fresh monolithic reset of the same (seed, env, episode) to atol 1e-8 in obs / qpos.
The bad-qacc fallback (checkAcc -> monolithic redo) is bit-identical to the monolithic kernel.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pair(n, prec="f64", seed=7, **kw):
    from mujoco_gymnasium_environments_amd.envs.soccer import SoccerVectorEnv
    a = SoccerVectorEnv(n, precision=prec, seed=seed, staged=True, **kw)
    b = SoccerVectorEnv(n, precision=prec, seed=seed, staged=False)
    return a, b


def test_staged_matches_monolithic_steps(soccer_model):
    staged, mono = _pair(6)
    o1, _ = staged.reset()
    o2, _ = mono.reset()
    torch.cuda.synchronize()
    np.testing.assert_allclose(o1.cpu().numpy(), o2.cpu().numpy(), atol=1e-9)
    rng = np.random.default_rng(3)
    for t in range(30):
        a = torch.from_numpy(rng.uniform(-20, 20, (6, soccer_model.nu)).astype(np.float32)).cuda()
        s1 = staged.step(a)
        s2 = mono.step(a)
        torch.cuda.synchronize()
        np.testing.assert_allclose(s1[0].cpu().numpy(), s2[0].cpu().numpy(), atol=1e-7, err_msg=f"obs step {t}")
        np.testing.assert_allclose(s1[1].cpu().numpy(), s2[1].cpu().numpy(), rtol=1e-7, atol=1e-5)
        assert torch.equal(s1[2], s2[2]) and torch.equal(s1[3], s2[3]), t
    np.testing.assert_allclose(staged.batch.qpos.cpu().numpy(), mono.batch.qpos.cpu().numpy(), atol=1e-7)


@pytest.mark.parametrize("banks", [1, 4])
def test_bank_reset_equals_monolithic_reset(soccer_model, banks):
    """Autoresets installed from banks (banks=1 also exercises the not-ready fallback) equal a
    monolithic Philox reset of the same episode index."""
    from mujoco_gymnasium_environments_amd.envs.soccer import SoccerVectorEnv
    n = 8
    env = SoccerVectorEnv(n, precision="f64", seed=21, staged=True, banks=banks)
    env.reset()
    rng = np.random.default_rng(9)
    last_obs = [None] * n
    last_qpos = [None] * n
    last_ep = [None] * n
    for t in range(150):
        a = torch.from_numpy(rng.uniform(-150, 150, (n, soccer_model.nu)).astype(np.float32)).cuda()
        obs, rew, term, trunc, _ = env.step(a)
        done = (term | trunc).cpu().numpy().astype(bool)
        for i in np.nonzero(done)[0]:
            last_obs[i] = obs[i].cpu().numpy().copy()
            last_qpos[i] = env.batch.qpos[i].cpu().numpy().copy()
            last_ep[i] = int(env.episode[i])
        assert torch.isfinite(obs).all()
    hit = [i for i in range(n) if last_obs[i] is not None]
    assert len(hit) >= n // 2, "too few terminations to exercise the banks"
    ref = SoccerVectorEnv(n, precision="f64", seed=21, staged=False)
    ep = torch.tensor([(last_ep[i] - 1) if last_ep[i] is not None else 0 for i in range(n)], dtype=torch.int32)
    ref.episode.copy_(ep.cuda())
    robs, _ = ref.reset()
    torch.cuda.synchronize()
    for i in hit:
        assert last_ep[i] >= 2
        np.testing.assert_allclose(last_obs[i], robs[i].cpu().numpy(), atol=1e-8, err_msg=f"env {i} ep {last_ep[i]}")
        np.testing.assert_allclose(last_qpos[i], ref.batch.qpos[i].cpu().numpy(), atol=1e-8)
    # later episodes than the prefilled ones were produced by staged settle steps
    assert max(last_ep[i] for i in hit) > banks + 1


def test_bad_qacc_redo_matches_monolithic(soccer_model):
    staged, mono = _pair(4)
    staged.reset()
    mono.reset()
    for e in (staged, mono):
        e.batch.qfrc_applied[1, 12] = 1e16  # qacc > 1e10 -> mj_checkAcc reset + second forward
    a = torch.zeros(4, soccer_model.nu, dtype=torch.float32, device="cuda:0")
    s1 = staged.step(a)
    s2 = mono.step(a)
    torch.cuda.synchronize()
    assert int(staged.batch.warning[1]) == int(mono.batch.warning[1]) >= 1
    assert torch.equal(s1[0][1], s2[0][1])
    assert torch.equal(staged.batch.qpos[1], mono.batch.qpos[1])
    np.testing.assert_allclose(s1[0].cpu().numpy(), s2[0].cpu().numpy(), atol=1e-7)


def test_staged_fp32_long_rollout_finite(soccer_model):
    """fp32 staged path at a bench-like load: 512 envs x 200 steps of U(-150,150) actions stay
    finite, every env keeps stepping, and the in-kernel rollout counters add up."""
    from mujoco_gymnasium_environments_amd.envs.soccer import SoccerVectorEnv
    n = 512
    env = SoccerVectorEnv(n, seed=1)
    env.reset()
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0)
    ep0 = int(env.episode.sum())
    for t in range(200):
        env.step(torch.rand(n, soccer_model.nu, device="cuda:0", generator=g) * 300 - 150)
    torch.cuda.synchronize()
    assert torch.isfinite(env.obs).all() and torch.isfinite(env.batch.qpos).all()
    ro = env.rollout.double().sum(0).cpu().numpy()
    assert ro[3] == n * 200
    assert ro[1] + ro[2] == int(env.episode.sum()) - ep0


def test_stream_sharded_equals_single_batch(soccer_model):
    """StreamShardedSoccerEnv (3 shards on 3 HIP streams, ragged sizes) reproduces one
    SoccerVectorEnv over the same envs bit for bit in fp32 at bench conditions (U(+-150)
    actions, same-step autoresets from the banks): every env's trajectory is keyed by its
    global index, and the shards only partition the launch."""
    from mujoco_gymnasium_environments_amd.envs.soccer import SoccerVectorEnv, StreamShardedSoccerEnv
    n = 200
    one = SoccerVectorEnv(n, precision="f32", seed=5, staged=True)
    sh = StreamShardedSoccerEnv(n, 3, precision="f32", seed=5, staged=True)
    assert [b - a for a, b in sh.bounds] == [67, 67, 66]
    o1, _ = one.reset()
    o2, _ = sh.reset()
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(11)
    resets = 0
    for t in range(120):
        a = (torch.rand(n, soccer_model.nu, device="cuda:0", generator=g) * 300.0 - 150.0).contiguous()
        s1 = one.step(a)
        s2 = sh.step(a)
        torch.cuda.synchronize()
        assert torch.equal(s1[0], s2[0]), f"obs step {t}"
        assert torch.equal(s1[1], s2[1]) and torch.equal(s1[2], s2[2]) and torch.equal(s1[3], s2[3]), t
        resets += int(s1[2].sum().item() + s1[3].sum().item())
    assert resets > 0  # the autoreset / bank path ran
    assert torch.equal(one.episode, sh.episode)
    assert torch.equal(one.info()["episode_stats"], sh.info()["episode_stats"])
    assert torch.equal(one.batch.qpos, torch.cat([s.batch.qpos for s in sh.shards]))
    # info() of the sharded batch behaves as the single batch's dict through every Mapping call
    i1, i2 = one.info(), sh.info()
    assert set(i2) == set(i1) and len(i2) == len(i1)
    assert torch.equal(i2.get("final_observation"), i1["final_observation"])
    assert i2.get("no_such_key") is None
    d2 = dict(i2.items())
    for k, v in i1.items():
        assert torch.equal(d2[k], v), k
    assert all(torch.equal(a, i1[k]) for k, a in zip(i2.keys(), i2.values()))
