"""GPU probe: where does a 2-step rollout differ from 2 single steps (flat scene, contacts on)?

Diagnostic for the split-quad kernels: golden controller actions (tests/golden/reference_glue.npz)
and random actions, rollout K=1 and K=2 against step calls; prints the envs and words that differ.

    python tools/probes/split_quad_probe.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from mujoco_playground_amd.sim import BatchedAckermannSim  # noqa: E402

DEV = "cuda:0"


def diff(tag, x, y):
    d = (x != y) & ~(torch.isnan(x) & torch.isnan(y))
    if not d.any():
        print(f"{tag}: equal", flush=True)
        return
    idx = d.nonzero()
    print(f"{tag}: {int(d.sum())} words differ, max |d| {float((x - y).abs().nan_to_num(0).max()):.3e}, "
          f"first {idx[:8].tolist()}", flush=True)


def run(acts, K, label, start=None):
    n = acts.shape[1]
    a = BatchedAckermannSim(n, DEV, seed=3, contacts=True)
    b = BatchedAckermannSim(n, DEV, seed=3, contacts=True)
    a.reset()
    b.reset()
    if start is not None:
        start(a)
        start(b)
    obs, rew, term, trunc = a.rollout(acts[:K].contiguous())
    for k in range(K):
        ob, rb, _, _ = b.step(acts[k])
        diff(f"{label} K={K} obs[{k}]", obs[k], ob)
        diff(f"{label} K={K} rew[{k}]", rew[k], rb)
    diff(f"{label} K={K} state", a.state, b.state)


def main():
    from test_gpu_golden_ctrl import GOLDEN, _start_state
    g = torch.tensor(GOLDEN["actions"], device=DEV)
    acts = torch.stack([torch.flip(g, [0]), g])
    for K in (1, 2):
        run(acts, K, "golden", _start_state)
    sim = BatchedAckermannSim(240, DEV, seed=3, contacts=True)
    r = sim.random_actions(2, seed=5)
    for K in (1, 2):
        run(r, K, "random")
    # same action twice: the controller hand-over cannot differ
    run(torch.stack([g, g]), 2, "golden-same", _start_state)


if __name__ == "__main__":
    main()
