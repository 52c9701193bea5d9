"""CPU: pin the humanoid_dancing env-logic oracle and reset draws to the reference's outputs.

Golden vectors (tests/golden/dancing_*.npz) come from the reference's own step() and reset()
(dancing_env.py:763-894) run on synthetic MjData-like state with physics stubbed out; see
tests/golden/make_fixtures.py. Bars: observation, reward (np.float64), flags, ctrl, rhythm and
move counters, combo / score / crowd, spotlight, stats and the fall_start_step attribute are
bit-exact.
"""
import numpy as np
import pytest

from mujoco_gymnasium_environments_amd.seeding import np_random
from oracle.dancing_logic import DancingLogic, DancingTables

G = "tests/golden/"
KEYS = ["current_step", "t_beat", "beat_count", "measure", "disco", "spotlight", "combo", "score", "move_idx",
        "move_start", "hist_len", "crowd", "applause", "stats", "fall_start", "fall_present", "prev_jvel"]


@pytest.fixture(scope="module")
def model(dancing_model):
    return dancing_model


@pytest.fixture(scope="module")
def golden():
    return dict(np.load(G + "dancing_envlogic.npz"))


@pytest.fixture(scope="module", params=["", "_f64"], ids=["float32_actions", "float64_actions"])
def golden_any(request):
    """The env-logic vectors with float32 actions, and the same states with float64 actions
    (make_fixtures.py main_f64: the reference keeps a float64 action float64 through np.clip)."""
    return dict(np.load(G + "dancing_envlogic" + request.param + ".npz"))


def state_from_golden(g, i, nu):
    s = {k: (g[k + "_in"][i].copy() if np.ndim(g[k + "_in"][i]) else g[k + "_in"][i].item()) for k in KEYS}
    s["hist"] = [int(x) for x in g["hist_in"][i] if x >= 0]
    n = int(g["ncon"][i])
    s.update(qpos=g["qpos"][i].copy(), qvel=g["qvel"][i].copy(), xpos=g["xpos"][i].copy(), xquat=g["xquat"][i].copy(),
             subtree_com=g["subtree_com"][i].copy(), con_geom=g["con_geom"][i][:n].astype(int), ctrl=np.zeros(nu),
             moves=g["moves"][i].copy(), durations=g["durations"][i].copy())
    return s


def test_golden_fixture_coverage(golden):
    n = golden["obs"].shape[0]
    assert golden["obs"].shape == (n, 94) and golden["action"].shape == (n, 29)
    for k in ("terminated", "truncated"):
        assert golden[k].any() and (~golden[k]).any(), k
    assert golden["reward_is_f64"].all()
    assert (golden["move_idx_out"] != golden["move_idx_in"]).any()
    assert (golden["fall_present_out"] != golden["fall_present_in"]).any()
    assert (golden["obs"][:, 78:88].sum(1) == 0).any(), "move index past the sequence end"


def test_dancing_logic_matches_reference(model, golden_any):
    golden = golden_any
    L = DancingLogic(DancingTables(model))
    n = golden["obs"].shape[0]
    for i in range(n):
        s = state_from_golden(golden, i, model.nu)
        a = L.pre(s, golden["action"][i])
        o, r, term, trunc = L.post(s, a)
        np.testing.assert_array_equal(s["ctrl"], golden["ctrl_out"][i], err_msg=f"ctrl case {i}")
        np.testing.assert_array_equal(o, golden["obs"][i], err_msg=f"obs case {i}")
        assert r == golden["reward"][i], (i, r, golden["reward"][i])
        assert term == bool(golden["terminated"][i]) and trunc == bool(golden["truncated"][i]), i
        for k in KEYS:
            np.testing.assert_array_equal(s[k], golden[k + "_out"][i], err_msg=f"{k} case {i}")
        h = golden["hist_out"][i]
        assert s["hist"] == [int(x) for x in h if x >= 0], i


def test_dancing_reset_draws(model):
    g = np.load(G + "dancing_reset.npz")
    t = DancingTables(model)
    L = DancingLogic(t)
    for seed, q, mv, du in zip(g["seeds"], g["qpos"], g["moves"], g["durations"]):
        rng, _ = np_random(int(seed))
        s = dict(qpos=np.zeros(model.nq), qvel=np.zeros(model.nv), ctrl=np.zeros(model.nu))
        L.apply_reset(s, t.reset_draws(rng))
        np.testing.assert_array_equal(s["qpos"], q)
        np.testing.assert_array_equal(s["moves"], mv)
        np.testing.assert_array_equal(s["durations"], du)
    # the initial pose lands on the first seven hinges (no root joint): abdomen_z = 1.8 rad
    assert model.id2name("joint", 2) == "abdomen_z" and g["qpos"][0][2] == 1.8
