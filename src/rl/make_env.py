"""`rl.make_env` (the module src/rl/__init__.py:3 imports; the reference ships only its .pyc)."""
from mujoco_playground_amd.rl.make_env import list_available_mazes, make_ackermann_env  # noqa: F401
