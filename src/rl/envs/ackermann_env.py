"""`rl.envs.ackermann_env` of the reference (src/rl/envs/ackermann_env.py:33)."""
from mujoco_playground_amd.rl.envs.ackermann_env import AckermannRobotEnv  # noqa: F401
