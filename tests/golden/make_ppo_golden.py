"""Golden vectors for the PPO learner from the reference's own checkpoints (build container only).

    python tests/golden/make_ppo_golden.py [--reference /root/reference]

Reads rl_logs/ppo/ppo_model_{10000,20000,30000}_steps.zip -> policy.pth and
policy.optimizer.pth with torch.load(weights_only=True, map_location="cpu") (nothing is
unpickled), and stores into tests/golden/ppo_policy.npz:
  params_<k>   the checkpoint policy in the flat ACKPPO_OFF_* layout (float32)
  adam_<k>     (step, lr, eps, beta1, beta2) of its Adam state (the SB3 hyper-parameters)
  obs_<k>      the checkpoint's own _last_obs (tests/golden/checkpoint_obs.npz)
  mu_<k>, value_<k>   the ActorCriticPolicy outputs on that observation, computed by an
               independent torch float64 evaluation of the SB3 module structure
               (Linear-Tanh-Linear-Tanh extractors, action_net, value_net).
The reference's sources are not copied: the fixture holds tensor data and outputs only.
"""
from __future__ import annotations

import argparse
import io
import os
import sys
import zipfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle.ppo_oracle import pack  # noqa: E402


def sb3_forward(sd, obs):
    t = {k: v.double() for k, v in sd.items()}
    x = torch.as_tensor(obs, dtype=torch.float64).reshape(1, -1)
    pi = torch.tanh(torch.tanh(x @ t["mlp_extractor.policy_net.0.weight"].T + t["mlp_extractor.policy_net.0.bias"])
                    @ t["mlp_extractor.policy_net.2.weight"].T + t["mlp_extractor.policy_net.2.bias"])
    vf = torch.tanh(torch.tanh(x @ t["mlp_extractor.value_net.0.weight"].T + t["mlp_extractor.value_net.0.bias"])
                    @ t["mlp_extractor.value_net.2.weight"].T + t["mlp_extractor.value_net.2.bias"])
    mu = pi @ t["action_net.weight"].T + t["action_net.bias"]
    v = vf @ t["value_net.weight"].T + t["value_net.bias"]
    return mu[0].numpy(), float(v[0, 0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    obs = np.load(os.path.join(HERE, "checkpoint_obs.npz"))
    out = {}
    for k in (10000, 20000, 30000):
        z = zipfile.ZipFile(os.path.join(a.reference, "rl_logs", "ppo", f"ppo_model_{k}_steps.zip"))
        sd = torch.load(io.BytesIO(z.read("policy.pth")), weights_only=True, map_location="cpu")
        opt = torch.load(io.BytesIO(z.read("policy.optimizer.pth")), weights_only=True, map_location="cpu")
        pg = opt["param_groups"][0]
        step = float(opt["state"][0]["step"])
        out[f"params_{k}"] = pack({n: v.numpy() for n, v in sd.items()}, np.float32)
        out[f"adam_{k}"] = np.array([step, pg["lr"], pg["eps"], pg["betas"][0], pg["betas"][1]])
        o = obs[f"obs_{k}"]
        mu, v = sb3_forward(sd, o)
        out[f"obs_{k}"] = o
        out[f"mu_{k}"] = mu
        out[f"value_{k}"] = np.array([v])
    np.savez(os.path.join(HERE, "ppo_policy.npz"), **out)
    print("wrote", os.path.join(HERE, "ppo_policy.npz"), sorted(out))


if __name__ == "__main__":
    main()
