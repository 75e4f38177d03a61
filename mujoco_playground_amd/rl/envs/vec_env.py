"""AckermannVecEnv: N Ackermann-robot environments stepped by one HIP launch.

SB3-VecEnv-shaped replacement for the reference's `DummyVecEnv([Monitor(AckermannRobotEnv)])`
(src/rl/train.py:70-76): reset() -> obs [N,79]; step(actions [N,2]) -> (obs, rewards, dones,
infos), with auto-reset of finished envs, `infos[i]["terminal_observation"]`,
`infos[i]["TimeLimit.truncated"]` and Monitor's `infos[i]["episode"] = {"r", "l"}`.
Tensors stay on the GPU; obs is a [N,79] view of the kernel's [79,N] SoA buffer.
"""
from __future__ import annotations

import time

import torch

from ...sim import BatchedAckermannSim
from .. import spaces


class AckermannVecEnv:
    def __init__(self, num_envs: int = 4096, device="cuda:0", seed: int = 0, contacts: bool = True,
                 env_offset: int = 0, max_episode_steps: int = 1000, goal_distance_threshold: float = 0.5,
                 collision_threshold: float = 0.15, max_linear_velocity: float = 1.0,
                 max_angular_velocity: float = 1.0, render_mode=None, variant: str = "auto",
                 scene: str = "flat", action_repeat: int = 1, nohit_clear: bool = False, goal_cells: int = 0):
        self.num_envs = int(num_envs)
        # the per-env constructor kwargs of the reference env (ackermann_env.py:51-60), batch-wide here
        self.max_episode_steps = max_episode_steps
        self.goal_distance_threshold = goal_distance_threshold
        self.collision_threshold = collision_threshold
        self.max_linear_velocity = max_linear_velocity
        self.max_angular_velocity = max_angular_velocity
        self.render_mode = render_mode
        self.observation_space = spaces.observation_space()
        self.action_space = spaces.action_space()
        self.sim = BatchedAckermannSim(num_envs, device, seed=seed, contacts=contacts, env_offset=env_offset,
                                       max_episode_steps=max_episode_steps,
                                       goal_distance_threshold=goal_distance_threshold,
                                       collision_threshold=collision_threshold,
                                       max_linear_velocity=max_linear_velocity,
                                       max_angular_velocity=max_angular_velocity, variant=variant,
                                       poststep_obs=(render_mode == "human"), scene=scene,
                                       action_repeat=action_repeat, nohit_clear=nohit_clear,
                                       goal_cells=goal_cells)
        self.device = self.sim.device
        self._actions = None
        self._ep_ret = torch.zeros(self.num_envs, device=self.device)
        self._ep_len = torch.zeros(self.num_envs, device=self.device)
        self._t_start = time.time()

    # -------- SB3 VecEnv API
    def reset(self) -> torch.Tensor:
        self.sim.reset()
        self.sim.episode.zero_()
        return self.sim.obs_soa.t()

    def step_async(self, actions):
        self._actions = torch.as_tensor(actions, dtype=torch.float32, device=self.device).reshape(self.num_envs, 2)

    def step_wait(self, infos: bool = True):
        ep_before = self.sim.episode[:2].clone() if infos else None
        obs, rew, term, trunc = self.sim.step(self._actions, autoreset=True)
        done = (term | trunc).bool()
        info_list = self._infos(done, term, trunc, rew, ep_before) if infos else None
        return obs.t(), rew, done, info_list

    def step(self, actions, infos: bool = True):
        self.step_async(actions)
        return self.step_wait(infos=infos)

    def step_tensors(self, actions: torch.Tensor):
        """Fast path: no per-env Python dicts. Returns (obs [N,79], reward, terminated, truncated)."""
        obs, rew, term, trunc = self.sim.step(actions, autoreset=True, want_info=False)
        return obs.t(), rew, term.bool(), trunc.bool()

    def _infos(self, done, term, trunc, rew, ep_before):
        info = self.sim.info
        n = self.num_envs
        idx = torch.nonzero(done).flatten().tolist()
        out = [dict() for _ in range(n)]
        if idx:
            tobs = self.sim.terminal_obs_soa.t()[idx].cpu().numpy()
            rets = (ep_before[0][idx] + rew[idx]).cpu().tolist()
            lens = (ep_before[1][idx] + 1).cpu().tolist()
            tr = trunc[idx].cpu().tolist()
            tm = term[idx].cpu().tolist()
            for j, i in enumerate(idx):
                out[i]["terminal_observation"] = tobs[j]
                out[i]["TimeLimit.truncated"] = bool(tr[j]) and not bool(tm[j])
                # Monitor's episode record: return, length, wall time since the env was made (train.py:70)
                out[i]["episode"] = {"r": round(rets[j], 6), "l": int(lens[j]),
                                     "t": round(time.time() - self._t_start, 6)}
        return out

    def env_info(self) -> dict:
        """Per-env reference info fields (ackermann_env.py:306-310) as device tensors."""
        return {"min_lidar": self.sim.info[0], "collision": self.sim.info[1] > 0,
                "goal_distance": self.sim.info[2], "bad_state": self.sim.info[3] > 0}

    def seed(self, seed: int):
        self.sim.seed = int(seed)

    def close(self):
        pass
