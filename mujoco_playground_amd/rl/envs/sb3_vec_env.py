"""AckermannSB3VecEnv: the batched env behind stable-baselines3's VecEnv interface, NumPy in and out.

The reference trains through `DummyVecEnv([make_env])` over `Monitor(AckermannRobotEnv(...))`
(src/rl/train.py:70-76). This class is the drop-in for that pair with N envs in one HIP launch:
it derives from SB3's `VecEnv` (a stand-in where SB3 is not installed, rl/gym_compat.py) and
gives SB3 what DummyVecEnv + Monitor give it:

  reset() -> obs float32 [N, 79]; step_async(actions [N, 2]); step_wait() -> (obs, rewards float32
  [N], dones bool [N], infos list of N dicts) with auto-reset, infos[i]["terminal_observation"],
  infos[i]["TimeLimit.truncated"] and Monitor's infos[i]["episode"] = {"r", "l", "t"};
  get_attr / set_attr / env_method / env_is_wrapped / seed / close.

NumPy arrays cross PCIe once per step (obs D2H, actions H2D). The torch-tensor path for on-device
learners is AckermannVecEnv (rl/envs/vec_env.py); rl/ppo.py steps the sim directly.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from ... import _lib
from ..gym_compat import VecEnv
from .vec_env import AckermannVecEnv

# per-env attributes of the reference env that are batch-wide constructor parameters here
_PARAMS = ("max_episode_steps", "goal_distance_threshold", "collision_threshold", "max_linear_velocity",
           "max_angular_velocity")


class _EnvView:
    """What `get_attr` / `env_method` see as env i (the reference env's attributes)."""

    def __init__(self, venv: "AckermannSB3VecEnv", i: int):
        self._v, self._i = venv, i

    def __getattr__(self, name):
        v = self._v.venv
        if name in _PARAMS or name in ("render_mode", "observation_space", "action_space", "metadata"):
            return getattr(v, name) if hasattr(v, name) else getattr(self._v, name)
        if name == "goal_position":
            return v.sim.state[37:39, self._i].cpu().numpy().astype(np.float64)
        if name == "step_count":
            return int(v.sim.state[42, self._i].view(torch.int32).item())
        if name == "np_random":
            return self._v._rngs[self._i]
        if name in ("render", "close"):
            return lambda *a, **k: None
        raise AttributeError(f"AckermannRobotEnv (batched) has no attribute {name!r}")


class AckermannSB3VecEnv(VecEnv):
    def __init__(self, num_envs: int = 4096, device="cuda:0", seed: int = 0, **env_kwargs):
        self.venv = AckermannVecEnv(num_envs, device=device, seed=seed, **env_kwargs)
        super().__init__(self.venv.num_envs, self.venv.observation_space, self.venv.action_space)
        self.render_mode = env_kwargs.get("render_mode")
        self.metadata = {"render_modes": ["human", "rgb_array"], "render_fps": 50}
        self._rngs = [np.random.default_rng(seed + i) for i in range(self.num_envs)]
        self._actions = None

    # -------- VecEnv abstract methods
    def reset(self) -> np.ndarray:
        if self._seeds[0] is not None:  # VecEnv.seed(s) applies at the next reset (SB3 2.x)
            self.venv.seed(int(self._seeds[0]))
            self._rngs = [np.random.default_rng(s) for s in self._seeds]
            self._seeds = [None] * self.num_envs
        obs = self.venv.reset()
        self.reset_infos = [{} for _ in range(self.num_envs)]
        return obs.cpu().numpy()

    def step_async(self, actions) -> None:
        a = np.asarray(actions, dtype=np.float32).reshape(self.num_envs, 2)
        self._actions = torch.from_numpy(a).to(self.venv.device, non_blocking=False)

    def step_wait(self):
        obs, rew, done, infos = self.venv.step(self._actions, infos=True)
        return obs.cpu().numpy(), rew.cpu().numpy().astype(np.float32), done.cpu().numpy().astype(bool), infos

    def close(self) -> None:
        self.venv.close()

    def get_attr(self, attr_name: str, indices=None) -> list:
        return [getattr(_EnvView(self, i), attr_name) for i in self._get_indices(indices)]

    def set_attr(self, attr_name: str, value, indices=None) -> None:
        idx = list(self._get_indices(indices))
        if attr_name not in _PARAMS:
            raise AttributeError(f"set_attr({attr_name!r}): only the env parameters {_PARAMS} can be set")
        if sorted(idx) != list(range(self.num_envs)):
            raise NotImplementedError(f"set_attr({attr_name!r}): env parameters are batch-wide (all indices)")
        setattr(self.venv, attr_name, value)
        s = self.venv.sim
        p = s.params
        setattr(p, attr_name, type(getattr(p, attr_name))(value))
        _lib.check(_lib.lib().ackphys_set_env_params(s._ctx, C.byref(p)), "ackphys_set_env_params")

    def env_method(self, method_name: str, *method_args, indices=None, **method_kwargs) -> list:
        return [getattr(_EnvView(self, i), method_name)(*method_args, **method_kwargs)
                for i in self._get_indices(indices)]

    def env_is_wrapped(self, wrapper_class, indices=None) -> list:
        # Monitor's statistics are built in (infos[i]["episode"]); no other wrapper is applied
        wrapped = getattr(wrapper_class, "__name__", "") == "Monitor"
        return [wrapped for _ in self._get_indices(indices)]

    def get_images(self):
        return [None for _ in range(self.num_envs)]
