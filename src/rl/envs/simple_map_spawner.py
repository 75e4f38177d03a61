"""`rl.envs.simple_map_spawner` of the reference (src/rl/envs/simple_map_spawner.py:13); the
reference env falls back to it when `environments.map_spawner` is absent (ackermann_env.py:83-90)."""
from mujoco_playground_amd.rl.envs.simple_map_spawner import SimpleMapSpawner  # noqa: F401
