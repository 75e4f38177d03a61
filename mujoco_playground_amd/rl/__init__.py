"""RL package (mirror of the reference's src/rl/__init__.py, with the missing make_env supplied)."""
from .envs import AckermannRobotEnv, AckermannSB3VecEnv, AckermannVecEnv
from .make_env import list_available_mazes, make_ackermann_env

__all__ = ["AckermannRobotEnv", "AckermannVecEnv", "AckermannSB3VecEnv", "make_ackermann_env",
           "list_available_mazes"]
