"""Base classes of the drop-in surface: gymnasium.Env and stable-baselines3's VecEnv when they are
importable, else stand-ins with the same public attributes and methods.

The reference's env is `class AckermannRobotEnv(gym.Env)` (src/rl/envs/ackermann_env.py:33,73,145)
wrapped by SB3's `Monitor` and `DummyVecEnv` (src/rl/train.py:70-76). Neither gymnasium nor SB3 is
installed in this image, so on such a host the classes derive from the stand-ins below; where they
are installed, the real bases are used and `isinstance(env, gymnasium.Env)` /
`isinstance(venv, VecEnv)` hold, which is what SB3's Monitor / env checks require.
"""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - exercised only where gymnasium exists
    import gymnasium as _gym
    Env = _gym.Env
    HAVE_GYMNASIUM = True
except ImportError:
    HAVE_GYMNASIUM = False

    class Env:
        """gymnasium.Env (1.x) stand-in: metadata, render_mode, spec, np_random and the
        reset(seed=...) seeding contract (the reference calls super().reset(seed=seed), :145)."""
        metadata = {"render_modes": []}
        render_mode = None
        spec = None
        observation_space = None
        action_space = None
        _np_random = None
        _np_random_seed = None

        @property
        def np_random(self) -> np.random.Generator:
            if self._np_random is None:
                self._np_random = np.random.default_rng()
            return self._np_random

        @np_random.setter
        def np_random(self, value: np.random.Generator):
            self._np_random = value

        @property
        def np_random_seed(self):
            return self._np_random_seed

        def reset(self, *, seed=None, options=None):
            if seed is not None:
                self._np_random_seed = int(seed)
                self._np_random = np.random.default_rng(seed)
            return None

        def step(self, action):
            raise NotImplementedError

        def render(self):
            return None

        def close(self):
            pass

        @property
        def unwrapped(self):
            return self

        def get_wrapper_attr(self, name: str):
            return getattr(self, name)

        def has_wrapper_attr(self, name: str) -> bool:
            return hasattr(self, name)

        def set_wrapper_attr(self, name: str, value):
            setattr(self, name, value)

        def __enter__(self):
            return self

        def __exit__(self, *args):
            self.close()
            return False

        def __str__(self):
            return f"<{type(self).__name__} instance>"

try:  # pragma: no cover - exercised only where stable-baselines3 exists
    from stable_baselines3.common.vec_env import VecEnv
    HAVE_SB3 = True
except ImportError:
    HAVE_SB3 = False

    class VecEnv:
        """stable_baselines3.common.vec_env.VecEnv (2.x) stand-in: the constructor attributes and
        the concrete helpers; subclasses provide reset / step_async / step_wait / close /
        get_attr / set_attr / env_method / env_is_wrapped."""
        def __init__(self, num_envs: int, observation_space, action_space):
            self.num_envs = num_envs
            self.observation_space = observation_space
            self.action_space = action_space
            self.reset_infos = [{} for _ in range(num_envs)]
            self._seeds = [None for _ in range(num_envs)]
            self._options = [{} for _ in range(num_envs)]
            self.render_mode = None
            self.metadata = {"render_modes": []}

        def step(self, actions):
            self.step_async(actions)
            return self.step_wait()

        def get_images(self):
            raise NotImplementedError

        def render(self, mode=None):
            return None

        def seed(self, seed=None):
            if seed is None:
                seed = int(np.random.randint(0, 2**32, dtype=np.uint32))
            self._seeds = [seed + idx for idx in range(self.num_envs)]
            return self._seeds

        def set_options(self, options=None):
            if options is None:
                options = {}
            self._options = options if isinstance(options, list) else [options] * self.num_envs

        @property
        def unwrapped(self):
            return self

        def getattr_depth_check(self, name, already_found):
            return None

        def _get_indices(self, indices):
            if indices is None:
                return range(self.num_envs)
            if isinstance(indices, int):
                return [indices]
            return indices
