"""Oracle vs golden vectors produced by the reference's own Python glue (tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest

from oracle.oracle import controller

G = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def glue():
    return np.load(os.path.join(G, "reference_glue.npz"))


def test_controller_matches_reference(glue):
    for a, ref in zip(glue["actions"], glue["ctrl"]):
        got = controller(a)
        nan = np.isnan(ref)
        assert np.array_equal(np.isnan(got), nan)
        np.testing.assert_allclose(got[~nan], ref[~nan], rtol=1e-12, atol=1e-15)


def test_lidar_alias_addresses(glue):
    assert list(glue["lidar_addrs"][:10]) == [76] * 10
    assert list(glue["lidar_addrs"][10:]) == list(range(15, 77))


def test_obs_reward_match_reference(glue, oracle):
    for k in range(len(glue["actions"])):
        obs, rew, term, info = oracle.observe_raw(glue["xpos"][k], glue["xquat"][k], glue["sensordata"][k],
                                                  glue["goal"], glue["ref"])
        np.testing.assert_array_equal(obs.astype(np.float32), glue["obs"][k])
        assert abs(rew - glue["reward"][k]) <= 1e-12 * max(1.0, abs(glue["reward"][k]))
        assert term == bool(glue["terminated"][k])
        assert info[0] == glue["min_lidar"][k]
        assert bool(info[1]) == bool(glue["collision"][k])
        assert abs(info[2] - glue["goal_distance"][k]) < 1e-12


def test_truncation_count(glue):
    # env.max_episode_steps was lowered to exercise truncation: steps >= limit are truncated
    lim = int(glue["max_episode_steps"])
    tr = glue["truncated"]
    assert not tr[: lim - 1].any() and tr[lim - 1:].all()


def test_checkpoint_pins():
    """SB3 checkpoints (maze runs) pin the obs layout: obs[0:10] == obs[71] (lidar name aliasing),
    obs[77] = |(dx,dy)|, obs[78] = wrap(atan2(dy,dx) - yaw)."""
    ck = np.load(os.path.join(G, "checkpoint_obs.npz"))
    for k in ck:
        o = ck[k].astype(np.float64)
        assert np.all(o[0:10] == o[71])
        assert abs(o[77] - np.hypot(o[75], o[76])) < 1e-6
        ang = np.arctan2(o[76], o[75]) - o[74]
        assert abs(np.arctan2(np.sin(ang), np.cos(ang)) - o[78]) < 1e-6
