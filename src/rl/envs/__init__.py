"""`rl.envs` of the reference (src/rl/envs/__init__.py), served by mujoco_playground_amd.rl.envs."""
from mujoco_playground_amd.rl.envs import (AckermannRobotEnv, AckermannSB3VecEnv, AckermannVecEnv,  # noqa: F401
                                           SimpleMapSpawner)

__all__ = ["AckermannRobotEnv", "AckermannVecEnv", "AckermannSB3VecEnv", "SimpleMapSpawner"]
