"""PPO learner, CPU side: the numpy oracle against torch autograd and the reference checkpoints,
the flat layout against include/ackppo.h, and libackppo.so's exports (no GPU calls)."""
import ctypes as C
import math
import os
import re

import numpy as np
import pytest
import torch

from oracle import ppo_oracle as po

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLD = os.path.join(HERE, "golden", "ppo_policy.npz")


def _random_params(seed=0, log_std=(-0.3, 0.2)):
    from mujoco_playground_amd.rl.ppo import init_params
    flat = init_params(seed).numpy().astype(np.float64)
    rng = np.random.default_rng(seed)
    # non-trivial heads (SB3's 0.01 action gain would make the actor gradient tiny)
    o, s = po.LAYOUT["action_net.weight"]
    flat[o:o + 128] = rng.normal(0, 0.3, 128)
    flat[po.LAYOUT["log_std"][0]:2] = log_std
    return flat


def test_layout_matches_header_and_host():
    from mujoco_playground_amd.rl import ppo
    hdr = open(os.path.join(REPO, "include", "ackppo.h")).read()
    offs = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define ACKPPO_OFF_(\w+) (\d+)", hdr)}
    names = ["LOG_STD", "PI_W1", "PI_B1", "PI_W2", "PI_B2", "VF_W1", "VF_B1", "VF_W2", "VF_B2", "ACT_W", "ACT_B",
             "VAL_W", "VAL_B"]
    assert [offs[n] for n in names] == [o for o, _ in po.LAYOUT.values()]
    assert int(re.search(r"#define ACKPPO_NPARAM (\d+)", hdr).group(1)) == po.NPARAM == ppo.NPARAM
    assert {k: (o, tuple(s)) for k, (o, s) in ppo.LAYOUT.items()} == {k: (o, tuple(s)) for k, (o, s) in
                                                                      po.LAYOUT.items()}


def test_libackppo_exports():
    from mujoco_playground_amd import _lib
    _lib.build()
    hdr = open(os.path.join(REPO, "include", "ackppo.h")).read()
    declared = set(re.findall(r"^(?:int|const char\*) (ackppo_\w+)\(", hdr, flags=re.M))
    assert declared == set(_lib.PPO_EXPORTS)
    L = C.CDLL(_lib.PPO_LIB_PATH)
    for name in declared:
        assert hasattr(L, name)


def test_checkpoint_policy_forward():
    """policy.pth of the reference's three checkpoints through the oracle's flat layout."""
    d = np.load(GOLD)
    for k in (10000, 20000, 30000):
        f = po.forward(d[f"params_{k}"].astype(np.float64), d[f"obs_{k}"][None])
        np.testing.assert_allclose(f["mu"][0], d[f"mu_{k}"], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(f["value"][0], d[f"value_{k}"][0], rtol=1e-6)
        ls = d[f"params_{k}"][:2]
        assert np.all(ls < 0.05) and np.all(ls > -0.2)   # the stored log_std (SURVEY §8c pin iv)
        step, lr, eps, b1, b2 = d[f"adam_{k}"]
        assert (lr, eps, b1, b2) == (3e-4, 1e-5, 0.9, 0.999)
        # Adam steps = completed rollouts x n_epochs (10) x n_steps/batch (2048/64): PPO.train's loop structure
        assert step == (k // 2048) * 10 * (2048 // 64)


def _torch_minibatch(flat, obs, actions, old_logp, adv, ret, clip, ent_coef, vf_coef):
    """Independent torch-autograd restatement of SB3 PPO.train's minibatch loss (float64)."""
    p = {k: torch.tensor(v, requires_grad=True) for k, v in po.unpack(flat).items()}
    x = torch.tensor(obs)
    pi = torch.tanh(torch.tanh(x @ p["mlp_extractor.policy_net.0.weight"].T + p["mlp_extractor.policy_net.0.bias"])
                    @ p["mlp_extractor.policy_net.2.weight"].T + p["mlp_extractor.policy_net.2.bias"])
    vf = torch.tanh(torch.tanh(x @ p["mlp_extractor.value_net.0.weight"].T + p["mlp_extractor.value_net.0.bias"])
                    @ p["mlp_extractor.value_net.2.weight"].T + p["mlp_extractor.value_net.2.bias"])
    mu = pi @ p["action_net.weight"].T + p["action_net.bias"]
    values = (vf @ p["value_net.weight"].T + p["value_net.bias"]).flatten()
    dist = torch.distributions.Normal(mu, torch.ones_like(mu) * p["log_std"].exp())
    logp = dist.log_prob(torch.tensor(actions)).sum(dim=1)
    ent = dist.entropy().sum(dim=1)
    a = torch.tensor(adv)
    a = (a - a.mean()) / (a.std() + 1e-8)
    ratio = torch.exp(logp - torch.tensor(old_logp))
    pg = -torch.min(a * ratio, a * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()
    vl = torch.nn.functional.mse_loss(torch.tensor(ret), values)
    loss = pg + ent_coef * (-torch.mean(ent)) + vf_coef * vl
    loss.backward()
    g = po.pack({k: v.grad.numpy() for k, v in p.items()}, np.float64)
    return float(loss.detach()), g


@pytest.mark.parametrize("ent_coef", [0.0, 0.01])
def test_oracle_gradient_matches_torch_autograd(ent_coef):
    rng = np.random.default_rng(3)
    flat = _random_params(1)
    B = 96
    obs = rng.normal(0, 1, (B, 79))
    f = po.forward(flat, obs)
    actions = f["mu"] + np.exp(f["log_std"]) * rng.normal(0, 1, (B, 2))
    # old policy slightly different so ratios straddle the clip range
    old_logp = po.log_prob(f["mu"], f["log_std"], actions) + rng.normal(0, 0.3, B)
    adv = rng.normal(0.5, 2.0, B)
    ret = f["value"] + rng.normal(0, 1, B)
    st, g = po.loss_and_grad(flat, obs, actions, old_logp, adv, ret, 0.2, ent_coef, 0.5)
    lt, gt = _torch_minibatch(flat, obs, actions, old_logp, adv, ret, 0.2, ent_coef, 0.5)
    assert abs(st["loss"] - lt) < 1e-12
    assert 0.05 < st["clip_fraction"] < 0.95
    np.testing.assert_allclose(g, gt, rtol=1e-9, atol=1e-12)


def test_oracle_adam_matches_torch():
    rng = np.random.default_rng(0)
    flat = _random_params(2)
    grads = [rng.normal(0, 1, po.NPARAM) * (np.arange(po.NPARAM) % 7 != 0) for _ in range(3)]
    params = torch.tensor(flat.copy(), requires_grad=True)
    opt = torch.optim.Adam([params], lr=3e-4, eps=1e-5)
    m = np.zeros(po.NPARAM)
    v = np.zeros(po.NPARAM)
    p = flat.copy()
    for t, g in enumerate(grads, 1):
        params.grad = torch.tensor(g.copy())
        norm_t = float(torch.nn.utils.clip_grad_norm_([params], 0.5))
        opt.step()
        p, m, v, norm = po.clip_and_adam(p, g, m, v, t)
        assert abs(norm - norm_t) < 1e-9 * norm
    np.testing.assert_allclose(p, params.detach().numpy(), rtol=1e-12, atol=1e-15)


def test_gae_matches_explicit_sum():
    """GAE restatement vs the closed form sum_l (gamma lambda)^l delta_{t+l} within an episode."""
    rng = np.random.default_rng(5)
    T, N, g, lam = 12, 3, 0.99, 0.95
    rew, val = rng.normal(size=(T, N)), rng.normal(size=(T, N))
    starts = np.zeros((T, N))
    starts[5, 1] = 1.0
    last_v, last_d = rng.normal(size=N), np.array([0.0, 0.0, 1.0])
    adv, ret = po.gae(rew, val, starts, last_v, last_d, g, lam)
    for e in range(N):
        nxt = np.append(val[1:, e], last_v[e])
        nnt = np.append(1 - starts[1:, e], 1 - last_d[e])
        delta = rew[:, e] + g * nxt * nnt - val[:, e]
        for t in range(T):
            acc, w = 0.0, 1.0
            for l in range(t, T):
                acc += w * delta[l]
                if nnt[l] == 0:
                    break
                w *= g * lam
            assert abs(adv[t, e] - acc) < 1e-12
    np.testing.assert_allclose(ret, adv + val)


def test_gaussian_noise_is_standard_normal():
    z = po.gaussian_noise(1234, np.arange(20000), 7)
    assert abs(z.mean()) < 0.03 and abs(z.std() - 1) < 0.03
    assert abs(np.corrcoef(z[:, 0], z[:, 1])[0, 1]) < 0.03


def test_init_params_sb3_gains():
    from mujoco_playground_amd.rl.ppo import init_params, state_dict_from_flat
    sd = state_dict_from_flat(init_params(0))
    w = sd["mlp_extractor.policy_net.2.weight"].double()
    np.testing.assert_allclose((w @ w.T).numpy(), 2.0 * np.eye(64), atol=1e-5)  # orthogonal, gain sqrt(2)
    a = sd["action_net.weight"].double()
    np.testing.assert_allclose((a @ a.T).numpy(), 1e-4 * np.eye(2), atol=1e-9)
    assert float(sd["log_std"].abs().sum()) == 0.0 and float(sd["value_net.bias"].abs().sum()) == 0.0
    assert math.isclose(float(sd["value_net.weight"].norm()), 1.0, rel_tol=1e-5)
