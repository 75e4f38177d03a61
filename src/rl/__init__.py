"""The reference's `rl` package, served by the MI355X simulator (drop-in for src/rl/__init__.py).

The reference's trainer puts `<project>/src` on sys.path and imports `from rl.envs import
AckermannRobotEnv` (src/rl/train.py:24-34). With this repo's `src/` on sys.path the same import
resolves here: `rl`, `rl.envs`, `rl.envs.ackermann_env`, `rl.envs.simple_map_spawner` and
`rl.make_env` re-export `mujoco_playground_amd.rl` (the batched HIP simulator behind the
reference's Gym surface). The reference package imports a `make_env` module whose source it does
not ship (src/rl/__init__.py:3); it is supplied.
"""
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from mujoco_playground_amd.rl import (AckermannRobotEnv, AckermannSB3VecEnv, AckermannVecEnv,  # noqa: E402
                                      list_available_mazes, make_ackermann_env)

__all__ = ["AckermannRobotEnv", "AckermannVecEnv", "AckermannSB3VecEnv", "make_ackermann_env",
           "list_available_mazes"]
