"""make_env: factory with the API of the reference's orphan `src/rl/__pycache__/make_env.cpython-312.pyc`
(its source is missing, so `import rl` fails as shipped: src/rl/__init__.py:3). Strings in that
.pyc give the signature restated here:

    make_ackermann_env(env_type='maze', maze_id='PointMaze_UMaze-v3', render_mode=None,
                       max_linear_velocity=0.5, max_angular_velocity=1.0,
                       goal_distance_threshold=0.3, **kwargs)
    list_available_mazes()

The Gymnasium-Robotics maze env is out of scope (uninstallable runtime-generated
PointMaze XML); env_type='simple' builds AckermannRobotEnv (one env, gymnasium.Env surface),
env_type='vec' the batched AckermannVecEnv (torch tensors on the GPU) and env_type='sb3' the
batched AckermannSB3VecEnv (stable-baselines3 VecEnv, NumPy), with num_envs from kwargs.
"""
from __future__ import annotations

from .envs import AckermannRobotEnv, AckermannSB3VecEnv, AckermannVecEnv

_MAZES = ["PointMaze_UMaze-v3", "PointMaze_Open-v3", "PointMaze_Medium-v3", "PointMaze_Large-v3"]


def list_available_mazes():
    return list(_MAZES)


def make_ackermann_env(env_type="maze", maze_id="PointMaze_UMaze-v3", render_mode=None, max_linear_velocity=0.5,
                       max_angular_velocity=1.0, goal_distance_threshold=0.3, **kwargs):
    if env_type == "maze":
        raise NotImplementedError("env_type='maze' needs gymnasium-robotics PointMaze (not installable here); "
                                  "use env_type='simple', 'vec' or 'sb3'")
    common = dict(max_linear_velocity=max_linear_velocity, max_angular_velocity=max_angular_velocity,
                  goal_distance_threshold=goal_distance_threshold)
    if env_type == "simple":
        return AckermannRobotEnv(render_mode=render_mode, **common, **kwargs)
    if env_type == "vec":
        return AckermannVecEnv(render_mode=render_mode, **common, **kwargs)
    if env_type == "sb3":
        return AckermannSB3VecEnv(render_mode=render_mode, **common, **kwargs)
    raise ValueError(f"unknown env_type {env_type!r}")
