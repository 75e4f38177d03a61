"""The reference trainer's import surface, on the CPU (no GPU calls).

src/rl/train.py puts `<project>/src` on sys.path and does `from rl.envs import AckermannRobotEnv`
(:24-34), wraps the env in SB3's Monitor / DummyVecEnv (:70-76) and evaluates with
`rl.utils.evaluate_agent` (:313). These tests check that the same imports resolve to this repo's
classes, and that the classes derive from gymnasium.Env / SB3's VecEnv when those packages exist
(stand-in packages with those names are put on sys.path in a child interpreter: neither package
is installed in this image).
"""
import os
import subprocess
import sys
import textwrap

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(code: str, extra_path: str | None = None) -> subprocess.CompletedProcess:
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join(p for p in (extra_path, os.path.join(REPO, "src")) if p)
    return subprocess.run([sys.executable, "-c", textwrap.dedent(code)], capture_output=True, text=True, env=env,
                          timeout=180, cwd="/")


def test_reference_imports_resolve():
    r = _run("""
        from rl.envs import AckermannRobotEnv
        from rl.envs.simple_map_spawner import SimpleMapSpawner
        from rl.make_env import make_ackermann_env, list_available_mazes
        from rl.utils import evaluate_agent, compute_episode_stats
        import rl
        import mujoco_playground_amd.rl as mp
        assert AckermannRobotEnv is mp.AckermannRobotEnv
        assert rl.make_ackermann_env is mp.make_ackermann_env
        assert "PointMaze_UMaze-v3" in list_available_mazes()
        try:  # the reference's train.py guards this import (train.py:37-41)
            from rl.envs import AckermannGymnasiumMazeEnv  # noqa: F401
            raise SystemExit("maze env should be absent")
        except ImportError:
            pass
        s = compute_episode_stats([1.0, 3.0], [10, 20])
        assert s["mean_return"] == 2.0 and s["std_length"] == 5.0
        import numpy as np
        from rl.utils import create_action_mapping, normalize_observation
        class Box:
            low = np.array([-1.0, 0.0, 2.0]); high = np.array([1.0, 4.0, 2.0])
        assert np.allclose(normalize_observation(np.array([0.0, 1.0, 5.0]), Box()), [0.5, 0.25, 3.0])
        assert normalize_observation("x", object()) == "x"
        assert create_action_mapping(None, 0.5, 2.0)(np.array([1.0, -0.5])) == (0.5, -1.0)
        print("ok")
    """)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr


def test_gym_env_contract_with_standin_base():
    """Without gymnasium: the stand-in base seeds np_random in reset(seed=...), as gymnasium.Env does."""
    r = _run("""
        from rl.envs import AckermannRobotEnv, AckermannSB3VecEnv
        from mujoco_playground_amd.rl.gym_compat import Env, HAVE_GYMNASIUM, HAVE_SB3, VecEnv
        assert not HAVE_GYMNASIUM and not HAVE_SB3
        assert issubclass(AckermannRobotEnv, Env) and issubclass(AckermannSB3VecEnv, VecEnv)
        e = Env()
        e.reset(seed=3); a = e.np_random.integers(0, 1 << 30, 4)
        e.reset(seed=3); b = e.np_random.integers(0, 1 << 30, 4)
        e.reset();       c = e.np_random.integers(0, 1 << 30, 4)
        assert (a == b).all() and not (a == c).all() and e.unwrapped is e and e.np_random_seed == 3
        print("ok")
    """)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr


def test_real_bases_used_when_installed(tmp_path):
    """With (stand-in) gymnasium and stable_baselines3 packages importable, AckermannRobotEnv is a
    gymnasium.Env, its spaces are gymnasium Boxes, and AckermannSB3VecEnv is an SB3 VecEnv."""
    g = tmp_path / "gymnasium"
    g.mkdir()
    (g / "__init__.py").write_text(textwrap.dedent("""
        from . import spaces
        class Env:
            metadata = {}
            def reset(self, *, seed=None, options=None):
                self.seeded = seed
    """))
    (g / "spaces.py").write_text(textwrap.dedent("""
        class Box:
            def __init__(self, low, high, shape=None, dtype=None):
                self.low, self.high, self.shape, self.dtype = low, high, shape, dtype
    """))
    v = tmp_path / "stable_baselines3" / "common" / "vec_env"
    v.mkdir(parents=True)
    (tmp_path / "stable_baselines3" / "__init__.py").write_text("")
    (tmp_path / "stable_baselines3" / "common" / "__init__.py").write_text("")
    (v / "__init__.py").write_text(textwrap.dedent("""
        class VecEnv:
            def __init__(self, num_envs, observation_space, action_space):
                self.num_envs = num_envs
                self.observation_space, self.action_space = observation_space, action_space
    """))
    r = _run("""
        import gymnasium, stable_baselines3.common.vec_env as sv
        from rl.envs import AckermannRobotEnv, AckermannSB3VecEnv
        from mujoco_playground_amd.rl import spaces
        assert issubclass(AckermannRobotEnv, gymnasium.Env)
        assert issubclass(AckermannSB3VecEnv, sv.VecEnv)
        assert isinstance(spaces.observation_space(), gymnasium.spaces.Box)
        assert spaces.observation_space().shape == (79,) and spaces.action_space().shape == (2,)
        print("ok")
    """, extra_path=str(tmp_path))
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr
