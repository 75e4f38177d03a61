"""RL environments (mirror of the reference's src/rl/envs/__init__.py)."""
from .ackermann_env import AckermannRobotEnv
from .vec_env import AckermannVecEnv

__all__ = ["AckermannRobotEnv", "AckermannVecEnv"]
