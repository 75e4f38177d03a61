"""RL environments (mirror of the reference's src/rl/envs/__init__.py). The Gymnasium-Robotics
maze env is out of scope, so AckermannGymnasiumMazeEnv is absent, as it is from
the reference's package when gymnasium-robotics is not installed."""
from .ackermann_env import AckermannRobotEnv
from .sb3_vec_env import AckermannSB3VecEnv
from .simple_map_spawner import SimpleMapSpawner
from .vec_env import AckermannVecEnv

__all__ = ["AckermannRobotEnv", "AckermannVecEnv", "AckermannSB3VecEnv", "SimpleMapSpawner"]
