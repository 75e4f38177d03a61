"""`rl.utils` of the reference (src/rl/utils.py): evaluate_agent / compute_episode_stats
(train.py:313), plus the batched evaluate_vec."""
from mujoco_playground_amd.rl.utils import compute_episode_stats, evaluate_agent, evaluate_vec  # noqa: F401
