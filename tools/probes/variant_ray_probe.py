"""Debug probe: dump the state of an obstacle-scene R=3 step that misses the oracle (test_gpu_variant)
with the GPU's R=1 chain from the same state."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
from conftest import f64_state  # noqa: E402
import test_gpu_obstacles as T  # noqa: E402
from test_gpu_variant import _boxes, _sim  # noqa: E402
from mujoco_playground_amd import _lib  # noqa: E402

K, E = int(sys.argv[1]), int(sys.argv[2])
sblob = _lib.load_blob("obstacles")
lo, hi = _boxes(sblob)
rng = np.random.default_rng(9)
n, steps = 256, 40
st = T.wall_states(n, lo, hi, rng)
kw = dict(action_repeat=3, nohit_clear=True)
sim = _sim(n, seed=9, scene="obstacles", **kw)
sim.set_state(T.to_device(st))
gen = torch.Generator(device="cpu").manual_seed(9)
acts = []
for _ in range(steps):
    x = torch.rand(n, 2, generator=gen) * 2 - 1
    x[:, 0] = 0.4 + 0.6 * torch.rand(n, generator=gen)
    acts.append(x.to("cuda:0"))
for k in range(K + 1):
    before = f64_state(sim.state)
    sim.step(acts[k], autoreset=True)
    torch.cuda.synchronize()
after = f64_state(sim.state)
chain = [before[E].copy()]
for nsim in (1, 256):   # a 1-env shadow and a full-width R=1 sim from the same states
    s1 = _sim(nsim, seed=9, scene="obstacles", nohit_clear=True)
    cur = before.copy()
    for j in range(3):
        s1.set_state(T.to_device(cur[:nsim] if nsim > 1 else cur[E:E + 1]))
        s1.step(acts[K][:nsim] if nsim > 1 else acts[K][E:E + 1], autoreset=False)
        torch.cuda.synchronize()
        nx = f64_state(s1.state)
        if nsim > 1:
            cur = np.concatenate([nx, cur[nsim:]])
            chain.append(nx[E].copy())
        else:
            cur = cur.copy()
            cur[E] = nx[0]
            chain.append(nx[0].copy())
np.savez("gpurun_out/variant_step_probe.npz", before=before[E], after=after[E], act=acts[K][E].cpu().numpy(),
         chain=np.array(chain))
print("saved")
