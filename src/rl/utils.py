"""`rl.utils` of the reference (src/rl/utils.py): evaluate_agent / compute_episode_stats
(train.py:313), normalize_observation, create_action_mapping, plus the batched evaluate_vec."""
from mujoco_playground_amd.rl.utils import (compute_episode_stats, create_action_mapping,  # noqa: F401
                                            evaluate_agent, evaluate_vec, normalize_observation)
