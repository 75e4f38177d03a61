"""Replay one saved env state (gpurun_out/hunt.npz from tools/parity_hunt.py) through each step
kernel variant and the oracle; prints the per-variant |dqpos| and primal cost."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from mujoco_playground_amd import _lib  # noqa: E402
from mujoco_playground_amd.sim import BatchedAckermannSim  # noqa: E402
from oracle.oracle import Oracle, controller  # noqa: E402
import parity_hunt as ph  # noqa: E402

h = np.load(sys.argv[1] if len(sys.argv) > 1 else os.path.join("tests", "golden", "quad_miss_state.npz"))
o = Oracle(_lib.load_blob())
before = h["before"]
ref = before[None].copy()
o.step(ref, h["action"][None], flags=3, seed=11)
d = o.diag(before, controller(h["action"]), flags=1)
print("oracle cost", ph.primal_cost(d, d["qacc"]))
for variant in ("lane", "quad"):
    for n in (1, 64):
        sim = BatchedAckermannSim(n, "cuda:0", seed=11, contacts=True, variant=variant)
        st = np.tile(before[:, None], (1, n)).astype(np.float32)
        st[42:44] = np.tile(before[42:44, None].astype(np.uint32), (1, n)).view(np.float32)
        sim.set_state(torch.tensor(st, device="cuda:0"))
        act = torch.tensor(np.tile(h["action"][None], (n, 1)), device="cuda:0")
        sim.step(act, autoreset=True)
        torch.cuda.synchronize()
        after = ph.f64(sim.state)
        dq = np.abs(after[:, :13] - ref[0, :13]).max(axis=1)
        print(variant, n, "max|dqpos|", dq.max(), "min", dq.min(), "cost", ph.primal_cost(d, after[0, 25:37]))
