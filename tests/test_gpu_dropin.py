"""The reference trainer's env surface, imported the way src/rl/train.py imports it, on the GPU.

train.py puts `<project>/src` on sys.path, does `from rl.envs import AckermannRobotEnv` (:34),
builds it with the CLI's kwargs (:279-283), runs its random baseline (`train_with_custom_algo`,
:189-227: reset / action_space.sample / step until done) or wraps it for SB3 (:70-76), and
evaluates with `rl.utils.evaluate_agent` (:313). The batched SB3 VecEnv adapter must give SB3
exactly what the torch VecEnv computes (NumPy copies of the same buffers) plus the DummyVecEnv /
Monitor info semantics.
"""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if os.path.join(REPO, "src") not in sys.path:
    sys.path.insert(0, os.path.join(REPO, "src"))

REF_INFO_KEYS = {"goal_distance", "collision", "min_lidar", "step", "linear_velocity", "angular_velocity"}


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_train_py_random_baseline_loop():
    from rl.envs import AckermannRobotEnv
    from rl.utils import evaluate_agent
    env = AckermannRobotEnv(render_mode=None, max_linear_velocity=1.0, goal_distance_threshold=0.5,
                            max_episode_steps=40)
    assert env.observation_space.shape == (79,) and env.action_space.shape == (2,)
    obs, info = env.reset(seed=7)
    assert obs.shape == (79,) and obs.dtype == np.float32
    assert set(info) == {"map_name", "goal_position", "start_position"} and info["map_name"] == "simple_floor"
    goal = list(info["goal_position"])
    _, info2 = env.reset(seed=7)
    assert info2["goal_position"] == goal  # reset(seed) is reproducible (np_random keys the Philox goal)
    env.action_space.seed(0)
    for episode in range(2):  # train_with_custom_algo's loop
        obs, info = env.reset()
        total, steps = 0.0, 0
        while True:
            obs, reward, terminated, truncated, info = env.step(env.action_space.sample())
            total += reward
            steps += 1
            assert obs.shape == (79,) and isinstance(reward, float)
            assert set(info) == REF_INFO_KEYS and info["step"] == steps
            assert obs[0] == obs[71] and (obs[:10] == obs[71]).all()  # the reference's lidar alias
            if terminated or truncated:
                break
        assert steps == 40 and truncated
    stats = evaluate_agent(env, lambda o: np.zeros(2, np.float32), num_episodes=2)
    assert stats["mean_length"] == 40 and stats["success_rate"] == 0.0
    env.close()


def test_sb3_vecenv_matches_torch_vecenv():
    from rl.envs import AckermannSB3VecEnv, AckermannVecEnv
    n, eplen = 96, 6
    kw = dict(seed=4, contacts=True, max_episode_steps=eplen)
    sb3 = AckermannSB3VecEnv(n, device="cuda:0", **kw)
    ref = AckermannVecEnv(n, device="cuda:0", **kw)
    o1 = sb3.reset()
    o2 = ref.reset()
    assert isinstance(o1, np.ndarray) and o1.shape == (n, 79) and o1.dtype == np.float32
    assert np.array_equal(o1, o2.cpu().numpy())
    rng = np.random.default_rng(0)
    seen_done = 0
    for k in range(2 * eplen + 1):
        a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        ob, rw, dn, inf = sb3.step(a)
        ob2, rw2, dn2, inf2 = ref.step(torch.from_numpy(a).cuda())
        assert ob.dtype == np.float32 and rw.dtype == np.float32 and dn.dtype == np.bool_
        assert np.array_equal(ob, ob2.cpu().numpy()) and np.array_equal(rw, rw2.cpu().numpy())
        assert np.array_equal(dn, dn2.cpu().numpy()) and isinstance(inf, list) and len(inf) == n
        for i in np.nonzero(dn)[0]:
            seen_done += 1
            d = inf[i]
            assert d["terminal_observation"].shape == (79,)
            assert d["TimeLimit.truncated"] is True  # eplen steps: truncation, not termination
            assert d["episode"]["l"] == eplen and set(d["episode"]) == {"r", "l", "t"} and d["episode"]["t"] >= 0
            assert np.array_equal(d["terminal_observation"], inf2[i]["terminal_observation"])
        for i in np.nonzero(~dn)[0][:3]:
            assert inf[i] == {}
    assert seen_done == 2 * n
    assert sb3.get_attr("max_episode_steps") == [eplen] * n
    assert sb3.get_attr("goal_distance_threshold", indices=[0, 5]) == [0.5, 0.5]
    assert len(sb3.get_attr("goal_position", indices=3)[0]) == 2
    Monitor = type("Monitor", (), {})
    assert sb3.env_is_wrapped(Monitor) == [True] * n
    assert sb3.env_is_wrapped(type("TimeLimit", (), {}), indices=[0]) == [False]
    # a batch-wide parameter set through set_attr reaches the kernels: episodes now last 3 steps
    sb3.set_attr("max_episode_steps", 3)
    sb3.reset()
    for k in range(3):
        _, _, dn, inf = sb3.step(np.zeros((n, 2), np.float32))
    assert dn.all() and inf[0]["episode"]["l"] == 3
    with pytest.raises(NotImplementedError):
        sb3.set_attr("max_episode_steps", 9, indices=[0])
    sb3.close()
