"""AckermannRobotEnv: the reference's single-env Gym surface on the batched HIP simulator.

Mirrors src/rl/envs/ackermann_env.py:33-325: a `gymnasium.Env` subclass (the stand-in base of
rl/gym_compat.py where gymnasium is not installed) with the same constructor kwargs, spaces,
reset()/step() return tuples and info keys, stepping N=1 env on the GPU. `Monitor(env)` and
`DummyVecEnv([lambda: env])` (train.py:70-76) wrap it as they wrap the reference's; batched
training uses AckermannVecEnv / AckermannSB3VecEnv. There is no CPU fallback: a missing HIP build
raises.
"""
from __future__ import annotations

import numpy as np
import torch

from ...sim import BatchedAckermannSim
from .. import spaces
from ..gym_compat import Env
from .simple_map_spawner import SimpleMapSpawner


class AckermannRobotEnv(Env):
    metadata = {"render_modes": ["human", "rgb_array"], "render_fps": 50}

    def __init__(self, map_spawner=None, max_episode_steps=1000, goal_distance_threshold=0.5,
                 collision_threshold=0.15, max_linear_velocity=1.0, max_angular_velocity=1.0, render_mode=None,
                 device="cuda:0", contacts: bool = True, scene: str | None = None, action_repeat: int = 1,
                 nohit_clear: bool = False, goal_cells: int = 0):
        super().__init__()
        # render_mode="human": the reference opens a passive MuJoCo viewer (out of scope here: no
        # window) and runs mj_forward after every mj_step (ackermann_env.py:202-207), so its
        # observations/rewards come from the post-step pose. That numerical effect is kept.
        self.max_episode_steps = max_episode_steps
        self.goal_distance_threshold = goal_distance_threshold
        self.collision_threshold = collision_threshold
        self.max_linear_velocity = max_linear_velocity
        self.max_angular_velocity = max_angular_velocity
        self.render_mode = render_mode
        # the spawner names the scene (ackermann_env.py:83-92); `scene` overrides it
        self.map_spawner = map_spawner if map_spawner is not None else SimpleMapSpawner(scene or "flat")
        scene = scene or getattr(self.map_spawner, "scene", "flat")
        self.observation_space = spaces.observation_space()
        self.action_space = spaces.action_space()
        self._sim = BatchedAckermannSim(1, device, seed=0, contacts=contacts, max_episode_steps=max_episode_steps,
                                        goal_distance_threshold=goal_distance_threshold,
                                        collision_threshold=collision_threshold,
                                        max_linear_velocity=max_linear_velocity,
                                        max_angular_velocity=max_angular_velocity,
                                        poststep_obs=(render_mode == "human"), scene=scene,
                                        action_repeat=action_repeat, nohit_clear=nohit_clear,
                                        goal_cells=goal_cells)
        # the reference's per-reset MuJoCo objects (:111-114): the batched sim owns the state
        self.model = None
        self.data = None
        self.controller = None
        self.odometry = None
        self.viewer = None
        self.step_count = 0
        self.goal_position = None
        self.robot_start_position = None

    def reset(self, seed=None, options=None):
        super().reset(seed=seed)  # seeds self.np_random (gymnasium contract, :145)
        # goals come from Philox(seed, env, episode) on the device, keyed by a draw of np_random
        # (the reference draws them from the unseeded global `random`, :167-172); a seeded reset
        # also restarts the episode counter, so reset(seed=s) gives the same goal every time
        if seed is not None:
            self._sim.state[43].zero_()
        self._sim.reset(seed=int(self.np_random.integers(0, 2**63 - 1)))
        self.step_count = 0
        st = self._sim.state[:, 0].cpu().numpy()
        self.goal_position = st[37:39].astype(np.float64)
        self.robot_start_position = np.zeros(2)   # odometry position at reset (odometry.py measures from it)
        obs = self._sim.obs_soa[:, 0].cpu().numpy().astype(np.float32)
        info = {"map_name": self.map_spawner.map_name if hasattr(self.map_spawner, "map_name") else "simple_floor",
                "goal_position": self.goal_position.tolist(),
                "start_position": self.robot_start_position.tolist()}
        return obs, info

    def step(self, action):
        a = np.clip(np.asarray(action, dtype=np.float32).reshape(2), -1.0, 1.0)
        act = torch.as_tensor(a, device=self._sim.device).reshape(1, 2)
        obs, rew, term, trunc = self._sim.step(act, autoreset=False)
        self.step_count += 1
        o = obs[:, 0].cpu().numpy().astype(np.float32)
        info_t = self._sim.info[:, 0].cpu().numpy()
        terminated = bool(term[0].item())
        truncated = bool(trunc[0].item())
        info = {"goal_distance": float(info_t[2]), "collision": bool(info_t[1] > 0), "min_lidar": float(info_t[0]),
                "step": self.step_count, "linear_velocity": float(a[0] * np.float32(self.max_linear_velocity)),
                "angular_velocity": float(a[1] * np.float32(self.max_angular_velocity))}
        return o, float(rew[0].item()), terminated, truncated, info

    def render(self):
        return None

    def close(self):
        self.viewer = None
