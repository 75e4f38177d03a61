"""The oracle's opt-in task variant (NOT the reference env; include/ackphys.h ackphys_env_params):
action_repeat mj_steps per env step and nohit_clear (rangefinder -1 readings are no obstacle in the
collision test). Pinned against the oracle's own reference-semantics path: an R-repeat env step is
R single mj_steps with the same ctrl (state bit for bit), and the variant's collision reading is the
minimum over the non-negative rays of the same observation. The GPU kernels are held to this oracle
in tests/test_gpu_variant.py.
"""
import numpy as np
import pytest

from oracle.oracle import Oracle

NRAYS = 72


@pytest.fixture(scope="module")
def states(blob):
    o = Oracle(blob)
    st = np.zeros((32, 44))
    o.reset(st, seed=3)
    # spread the poses: a few reference steps with random actions
    rng = np.random.default_rng(3)
    for _ in range(20):
        o.step(st, rng.uniform(-1, 1, (32, 2)).astype(np.float32), flags=1, seed=3)
    return st


@pytest.mark.parametrize("repeat", [2, 5])
def test_action_repeat_is_repeated_mj_steps(blob, states, repeat):
    rng = np.random.default_rng(repeat)
    act = rng.uniform(-1, 1, (32, 2)).astype(np.float32)
    ref, o1 = states.copy(), Oracle(blob)
    rep, o2 = states.copy(), Oracle(blob)
    o2.set_env_params(action_repeat=repeat)
    for _ in range(repeat):
        obs1, rew1, term1, _, _, info1 = o1.step(ref, act, flags=1, seed=3)
    obs2, rew2, term2, _, _, info2 = o2.step(rep, act, flags=1, seed=3)
    np.testing.assert_array_equal(rep[:, :42], ref[:, :42])   # qpos, qvel, warm start, goal, ref
    np.testing.assert_array_equal(rep[:, 42], states[:, 42] + 1)   # one env step
    np.testing.assert_array_equal(ref[:, 42], states[:, 42] + repeat)
    # obs / reward / info come from the last mj_step's forward pass in both
    np.testing.assert_array_equal(obs2, obs1)
    np.testing.assert_array_equal(rew2, rew1)
    np.testing.assert_array_equal(info2, info1)


def test_action_repeat_truncates_on_env_steps(blob, states):
    o = Oracle(blob)
    o.set_env_params(max_episode_steps=3, action_repeat=4)
    st = states.copy()
    st[:, 42] = 0
    act = np.zeros((32, 2), np.float32)
    for k in range(3):
        _, _, _, trunc, _, _ = o.step(st, act, flags=1, seed=3)
        assert trunc.all() == (k == 2)


@pytest.mark.parametrize("flags", [0, 1])
def test_nohit_clear_collision_reading(blob, states, flags):
    act = np.random.default_rng(1).uniform(-1, 1, (32, 2)).astype(np.float32)
    base, var = Oracle(blob), Oracle(blob)
    var.set_env_params(nohit_clear=True)
    s0, s1 = states.copy(), states.copy()
    obs0, rew0, term0, _, _, info0 = base.step(s0, act, flags=flags, seed=3)
    obs1, rew1, term1, _, _, info1 = var.step(s1, act, flags=flags, seed=3)
    np.testing.assert_array_equal(s0, s1)        # dynamics untouched
    np.testing.assert_array_equal(obs0, obs1)    # so are the observations (the -1 readings stay)
    rays = obs0[:, :NRAYS]
    assert (rays < 0).any(axis=1).all()          # flat floor: the horizontal rays never hit
    np.testing.assert_allclose(info0[:, 0], rays.min(axis=1), atol=1e-6)
    assert info0[:, 1].all()                     # the reference: every -1 reading is a "collision"
    hit = np.where(rays >= 0, rays, np.inf).min(axis=1)
    want = np.where(np.isfinite(hit), hit, -1.0)
    np.testing.assert_allclose(info1[:, 0], want, atol=1e-6)
    np.testing.assert_array_equal(info1[:, 1] > 0, np.isfinite(hit) & (hit < 0.15))
    # the collision penalty is the only reward difference
    np.testing.assert_allclose(rew1 - rew0, 50.0 * (info0[:, 1] > 0) - 50.0 * (info1[:, 1] > 0), atol=1e-9)
    np.testing.assert_array_equal(term0, term1)
