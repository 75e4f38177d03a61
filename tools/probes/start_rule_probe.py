"""GPU probe: one step from the reset state through every kernel mapping, post-step obs on/off,
Newton start rule on/off; prints max |qpos| / |qvel| after the step (finite = ok)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mujoco_playground_amd.sim import BatchedAckermannSim  # noqa: E402

for variant in ("lane", "quad"):
    for post in (False, True):
        for mjws in (False, True):
            for contacts in (False, True):
                sim = BatchedAckermannSim(128, "cuda:0", seed=13, contacts=contacts, variant=variant,
                                          poststep_obs=post, mj_warmstart=mjws)
                sim.reset()
                acts = sim.random_actions(3, seed=13)
                out = []
                for k in range(3):
                    sim.step(acts[k])
                    torch.cuda.synchronize()
                    out.append(f"{sim.state[:13].abs().max().item():.3g}/{sim.state[13:25].abs().max().item():.3g}")
                print(f"{variant:5s} post={int(post)} mjws={int(mjws)} contacts={int(contacts)}: {' '.join(out)}",
                      flush=True)
