"""Debug probe: dump the state/obs of the first obstacle-scene R=3 ray mismatch (test_gpu_variant)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
from conftest import f64_state  # noqa: E402
import test_gpu_obstacles as T  # noqa: E402
from test_gpu_variant import _boxes, _oracle, _sim  # noqa: E402
from mujoco_playground_amd import _lib  # noqa: E402

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
o = _oracle(sblob, **kw)
for k in range(14):
    before = f64_state(sim.state)
    sim.step(acts[k], autoreset=True)
    torch.cuda.synchronize()
    after = f64_state(sim.state)
ref = before.copy()
a_np = acts[13].cpu().numpy()
oobs, *_ = o.step(ref, a_np, flags=3, seed=9)
# the GPU's own pose after 2 mj_steps: an R=2 sim from `before`
s2 = _sim(n, seed=9, scene="obstacles", action_repeat=2, nohit_clear=True)
s2.set_state(T.to_device(before))
s2.step(acts[13], autoreset=False)
torch.cuda.synchronize()
mid_gpu = f64_state(s2.state)
np.savez("gpurun_out/variant_ray_probe.npz", before=before, after=after, ref=ref, act=a_np,
         gobs=sim.obs_soa.cpu().numpy().T, oobs=oobs, mid_gpu=mid_gpu)
print("saved", np.abs(sim.obs_soa.cpu().numpy().T[5, 30] - oobs[5, 30]))
