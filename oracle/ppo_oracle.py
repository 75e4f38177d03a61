"""numpy float64 restatement of the PPO learner (TEST INFRASTRUCTURE ONLY).

Checker for libackppo.so (include/ackppo.h). Only tests/, __graft_entry__.smoke() and bench.py
may import it; the product never does.

What it restates: stable-baselines3 2.7.0 `PPO('MlpPolicy')` as the reference uses it
(src/rl/train.py:99-128 builds `PPO('MlpPolicy', vec_env, learning_rate=3e-4, n_steps=2048,
batch_size=64, n_epochs=10, gamma=0.99, gae_lambda=0.95, clip_range=0.2, ent_coef=...)`;
the checkpoints under rl_logs/ppo store vf_coef 0.5, max_grad_norm 0.5, normalize_advantage
True, clip_range_vf None, target_kl None, Adam eps 1e-5). SB3 (third-party, version 2.7.0 per
the checkpoints' system_info.txt) is NOT vendored in the reference nor installed here; its
published algorithm is restated from:
  * ActorCriticPolicy / MlpExtractor: separate pi and vf nets, Linear(79,64)-Tanh-Linear(64,64)-Tanh,
    action_net Linear(64,2), value_net Linear(64,1), log_std parameter (init 0), orthogonal
    init (gains sqrt(2) / 0.01 / 1, zero biases);
  * DiagGaussianDistribution: Normal(mean, exp(log_std)); log_prob and entropy summed over dims;
  * OnPolicyAlgorithm.collect_rollouts: actions clipped to the Box for env.step, stored raw;
    reward += gamma * V(terminal_observation) when done and TimeLimit.truncated;
  * RolloutBuffer.compute_returns_and_advantage: GAE(lambda), returns = advantages + values;
  * PPO.train: per-minibatch advantage normalisation (unbiased std, +1e-8), ratio =
    exp(logp - old_logp), clipped surrogate, MSE value loss, entropy loss = -mean(entropy),
    loss = pg + ent_coef * ent + vf_coef * vf, clip_grad_norm_(max_grad_norm), Adam.
torch semantics restated: clip_grad_norm_ coef = max_norm / (norm + 1e-6) clamped to 1;
Adam exp_avg.lerp_(g, 1-b1), exp_avg_sq = b2 v + (1-b2) g^2, p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps).
Anchors that pin it: the policy.pth tensors (shapes, key names, log_std values) via
tests/golden/ppo_policy.npz, and a torch-autograd cross-check of every gradient
(tests/test_ppo_oracle.py). Beyond those the SB3 semantics are "parity unpinned" (no SB3 run
can be made here).
"""
from __future__ import annotations

import numpy as np

NOBS, NACT, HID = 79, 2, 64
LOG_SQRT_2PI = 0.5 * np.log(2 * np.pi)

# flat layout: the SB3 state_dict tensors in parameters() order, each 4-float aligned
_SPEC = [("log_std", (2,)),
         ("mlp_extractor.policy_net.0.weight", (HID, NOBS)), ("mlp_extractor.policy_net.0.bias", (HID,)),
         ("mlp_extractor.policy_net.2.weight", (HID, HID)), ("mlp_extractor.policy_net.2.bias", (HID,)),
         ("mlp_extractor.value_net.0.weight", (HID, NOBS)), ("mlp_extractor.value_net.0.bias", (HID,)),
         ("mlp_extractor.value_net.2.weight", (HID, HID)), ("mlp_extractor.value_net.2.bias", (HID,)),
         ("action_net.weight", (NACT, HID)), ("action_net.bias", (NACT,)),
         ("value_net.weight", (1, HID)), ("value_net.bias", (1,))]


def _layout():
    out, off = {}, 0
    for name, shape in _SPEC:
        out[name] = (off, shape)
        off += -(-int(np.prod(shape)) // 4) * 4
    return out, off


LAYOUT, NPARAM = _layout()


def unpack(flat):
    return {k: np.asarray(flat[o:o + int(np.prod(s))], np.float64).reshape(s) for k, (o, s) in LAYOUT.items()}


def pack(sd, dtype=np.float32):
    flat = np.zeros(NPARAM, dtype)
    for k, (o, s) in LAYOUT.items():
        flat[o:o + int(np.prod(s))] = np.asarray(sd[k]).reshape(-1)
    return flat


# ------------------------------------------------------------------ Philox (noise stream)

def _mulhilo(a, b):
    p = np.uint64(a) * b.astype(np.uint64)
    return (p >> np.uint64(32)).astype(np.uint32), (p & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def philox4x32(ctr, key):
    """ctr: [4, n] uint32 arrays, key: (k0, k1). Philox4x32-10."""
    c = [np.asarray(x, np.uint32).copy() for x in ctr]
    k0, k1 = np.uint32(key[0]), np.uint32(key[1])
    for _ in range(10):
        hi0, lo0 = _mulhilo(0xD2511F53, c[0])
        hi1, lo1 = _mulhilo(0xCD9E8D57, c[2])
        c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
        k0 = np.uint32((int(k0) + 0x9E3779B9) & 0xFFFFFFFF)
        k1 = np.uint32((int(k1) + 0xBB67AE85) & 0xFFFFFFFF)
    return c


def gaussian_noise(seed, env_ids, step):
    """z [n, 2]: Box-Muller of Philox(key=seed, counter=(env, step, 2, 0)), f32 draws as the kernel."""
    env_ids = np.asarray(env_ids, np.uint32)
    n = env_ids.shape[0]
    c = philox4x32([env_ids, np.full(n, step, np.uint32), np.full(n, 2, np.uint32), np.zeros(n, np.uint32)],
                   (seed & 0xFFFFFFFF, seed >> 32))
    u1 = ((c[0] >> np.uint32(8)).astype(np.float64) + 1.0) / 16777216.0
    u2 = (c[1] >> np.uint32(8)).astype(np.float64) / 16777216.0
    r = np.sqrt(-2.0 * np.log(u1))
    return np.stack([r * np.cos(2 * np.pi * u2), r * np.sin(2 * np.pi * u2)], axis=1)


# ------------------------------------------------------------------ policy

def forward(flat, obs):
    """obs [B, 79] -> dict(mu [B,2], value [B], and the hidden activations)."""
    p = unpack(flat)
    x = np.asarray(obs, np.float64)
    a1 = np.tanh(x @ p["mlp_extractor.policy_net.0.weight"].T + p["mlp_extractor.policy_net.0.bias"])
    a2 = np.tanh(a1 @ p["mlp_extractor.policy_net.2.weight"].T + p["mlp_extractor.policy_net.2.bias"])
    c1 = np.tanh(x @ p["mlp_extractor.value_net.0.weight"].T + p["mlp_extractor.value_net.0.bias"])
    c2 = np.tanh(c1 @ p["mlp_extractor.value_net.2.weight"].T + p["mlp_extractor.value_net.2.bias"])
    mu = a2 @ p["action_net.weight"].T + p["action_net.bias"]
    v = (c2 @ p["value_net.weight"].T + p["value_net.bias"])[:, 0]
    return dict(x=x, a1=a1, a2=a2, c1=c1, c2=c2, mu=mu, value=v, log_std=p["log_std"])


def log_prob(mu, log_std, actions):
    sigma = np.exp(log_std)
    return np.sum(-((actions - mu) ** 2) / (2 * sigma ** 2) - np.log(sigma) - LOG_SQRT_2PI, axis=1)


def entropy(log_std):
    return float(np.sum(0.5 + LOG_SQRT_2PI + log_std))


def act(flat, obs, seed=0, step=0, env_offset=0, deterministic=False):
    """-> (action raw [B,2], env_action clipped, log_prob [B], value [B])."""
    f = forward(flat, obs)
    if deterministic:
        a = f["mu"].copy()
    else:
        z = gaussian_noise(seed, env_offset + np.arange(len(obs)), step)
        a = f["mu"] + np.exp(f["log_std"]) * z
    return a, np.clip(a, -1, 1), log_prob(f["mu"], f["log_std"], a), f["value"]


# ------------------------------------------------------------------ rollout bookkeeping

def bootstrap(flat, terminal_obs, reward, term, trunc, gamma):
    r = np.asarray(reward, np.float64).copy()
    m = np.asarray(trunc, bool) & ~np.asarray(term, bool)
    if m.any():
        r[m] += gamma * forward(flat, np.asarray(terminal_obs)[m])["value"]
    return r, (np.asarray(term, bool) | np.asarray(trunc, bool)).astype(np.float64)


def gae(rewards, values, episode_starts, last_values, last_dones, gamma, lam):
    T = rewards.shape[0]
    adv = np.zeros_like(rewards, dtype=np.float64)
    last = np.zeros(rewards.shape[1])
    for t in reversed(range(T)):
        if t == T - 1:
            nnt, nv = 1.0 - last_dones, last_values
        else:
            nnt, nv = 1.0 - episode_starts[t + 1], values[t + 1]
        delta = rewards[t] + gamma * nv * nnt - values[t]
        last = delta + gamma * lam * nnt * last
        adv[t] = last
    return adv, adv + values


# ------------------------------------------------------------------ PPO loss and its gradient

def loss_and_grad(flat, obs, actions, old_logp, advantages, returns, clip_range=0.2, ent_coef=0.0, vf_coef=0.5,
                  normalize=True):
    """One minibatch of PPO.train: returns (loss dict, flat gradient float64)."""
    f = forward(flat, obs)
    p = unpack(flat)
    B = obs.shape[0]
    adv = np.asarray(advantages, np.float64)
    if normalize and B > 1:
        adv = (adv - adv.mean()) / (adv.std(ddof=1) + 1e-8)
    sigma = np.exp(f["log_std"])
    lp = log_prob(f["mu"], f["log_std"], actions)
    ratio = np.exp(lp - old_logp)
    l1, l2 = adv * ratio, adv * np.clip(ratio, 1 - clip_range, 1 + clip_range)
    pg = -np.mean(np.minimum(l1, l2))
    vf = np.mean((returns - f["value"]) ** 2)
    ent = entropy(f["log_std"])
    loss = pg + ent_coef * (-ent) + vf_coef * vf
    # backward
    glogp = np.where(l1 <= l2, -adv * ratio / B, 0.0)
    dv = actions - f["mu"]
    gmu = glogp[:, None] * dv / sigma ** 2
    glog = np.sum(glogp[:, None] * (dv ** 2 / sigma ** 2 - 1.0), axis=0) - ent_coef
    gv = vf_coef * 2.0 * (f["value"] - returns) / B
    g = {}
    g["log_std"] = glog
    g["action_net.weight"] = gmu.T @ f["a2"]
    g["action_net.bias"] = gmu.sum(0)
    g["value_net.weight"] = (gv[:, None] * f["c2"]).sum(0)[None, :]
    g["value_net.bias"] = np.array([gv.sum()])
    for net, h1, h2, dout in (("policy_net", f["a1"], f["a2"], gmu @ p["action_net.weight"]),
                              ("value_net", f["c1"], f["c2"], gv[:, None] * p["value_net.weight"])):
        d2 = dout * (1 - h2 ** 2)
        g[f"mlp_extractor.{net}.2.weight"] = d2.T @ h1
        g[f"mlp_extractor.{net}.2.bias"] = d2.sum(0)
        d1 = (d2 @ p[f"mlp_extractor.{net}.2.weight"]) * (1 - h1 ** 2)
        g[f"mlp_extractor.{net}.0.weight"] = d1.T @ f["x"]
        g[f"mlp_extractor.{net}.0.bias"] = d1.sum(0)
    stats = dict(loss=loss, policy_gradient_loss=pg, value_loss=vf, entropy=ent,
                 clip_fraction=float(np.mean(np.abs(ratio - 1) > clip_range)),
                 approx_kl=float(np.mean((ratio - 1) - np.log(ratio))))
    return stats, pack(g, np.float64)


def clip_and_adam(flat, grad, m, v, step, lr=3e-4, beta1=0.9, beta2=0.999, eps=1e-5, max_grad_norm=0.5):
    """torch clip_grad_norm_ + Adam (returns new params, m, v, pre-clip norm)."""
    norm = float(np.sqrt(np.sum(np.asarray(grad, np.float64) ** 2)))
    g = grad * min(max_grad_norm / (norm + 1e-6), 1.0)
    m = m + (1 - beta1) * (g - m)
    v = beta2 * v + (1 - beta2) * g * g
    step_size = lr / (1 - beta1 ** step)
    denom = np.sqrt(v) / np.sqrt(1 - beta2 ** step) + eps
    return flat - step_size * m / denom, m, v, norm
