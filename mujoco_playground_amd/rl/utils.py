"""Evaluation helpers with the reference's API (src/rl/utils.py:8-72): evaluate_agent /
compute_episode_stats, which train.py calls after training (`from rl.utils import evaluate_agent`,
train.py:313), normalize_observation and create_action_mapping, plus a batched evaluation over an
AckermannVecEnv (every env runs one episode in the same HIP launches).
"""
from __future__ import annotations

import numpy as np
import torch


def compute_episode_stats(returns, lengths) -> dict:
    """Mean / std / min / max of the episode returns and mean / std of the lengths (utils.py:8-17)."""
    r = np.asarray(returns, dtype=np.float64)
    n = np.asarray(lengths, dtype=np.float64)
    return {"mean_return": r.mean(), "std_return": r.std(), "min_return": r.min(), "max_return": r.max(),
            "mean_length": n.mean(), "std_length": n.std()}


def evaluate_agent(env, agent, num_episodes: int = 10) -> dict:
    """Run `num_episodes` episodes of a single Gym env with `agent.predict(obs, deterministic=True)`
    (or `agent(obs)` for a plain callable); success = the episode ended by termination (goal
    reached). Same statistics as utils.py:20-50."""
    act = ((lambda o: agent.predict(o, deterministic=True)[0]) if hasattr(agent, "predict") else agent)
    returns, lengths, success = [], [], []
    for _ in range(num_episodes):
        obs, _ = env.reset()
        ret, steps, done = 0.0, 0, False
        while not done:
            obs, reward, terminated, truncated, _ = env.step(act(obs))
            ret += reward
            steps += 1
            done = terminated or truncated
        returns.append(ret)
        lengths.append(steps)
        success.append(bool(terminated))
    out = compute_episode_stats(returns, lengths)
    out["success_rate"] = float(np.mean(success))
    return out


def evaluate_vec(venv, policy, max_steps: int | None = None) -> dict:
    """One episode per env of an AckermannVecEnv, all envs stepped together: `policy(obs [N,79])`
    returns actions [N,2] (torch, on the env's device). Each env's first episode is recorded (later
    auto-reset episodes are ignored); statistics as evaluate_agent over N episodes."""
    n = venv.num_envs
    obs = venv.reset()
    dev = venv.device
    ret = torch.zeros(n, dtype=torch.float64, device=dev)
    length = torch.zeros(n, dtype=torch.int64, device=dev)
    live = torch.ones(n, dtype=torch.bool, device=dev)
    success = torch.zeros(n, dtype=torch.bool, device=dev)
    limit = max_steps if max_steps is not None else int(venv.max_episode_steps)
    for _ in range(limit):
        obs, rew, term, trunc = venv.step_tensors(policy(obs))
        ret += torch.where(live, rew.double(), 0.0)
        length += live.long()
        success |= live & term
        live &= ~(term | trunc)
        if not bool(live.any()):
            break
    out = compute_episode_stats(ret.cpu().numpy(), length.cpu().numpy())
    out["success_rate"] = float(success.float().mean().item())
    return out


def normalize_observation(obs, obs_space):
    """(obs - low) / (high - low) per entry for a Box space (zero-width entries divide by 1); any
    other space returns obs unchanged (utils.py:53-63)."""
    if not (hasattr(obs_space, "low") and hasattr(obs_space, "high")):
        return obs
    low = np.asarray(obs_space.low)
    span = np.asarray(obs_space.high) - low
    span = np.where(span == 0, 1.0, span).astype(span.dtype)
    return (obs - low) / span


def create_action_mapping(action_space, max_linear: float = 1.0, max_angular: float = 1.0):
    """A function mapping a normalised action [2] to (linear_x, angular_z) = (a0 * max_linear,
    a1 * max_angular) (utils.py:66-72; action_space is unused there too)."""
    def map_action(action):
        return action[0] * max_linear, action[1] * max_angular
    return map_action
