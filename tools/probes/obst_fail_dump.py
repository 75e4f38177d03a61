"""Re-run the obstacle wall-contact scenario (tests/test_gpu_obstacles.py) and dump every env-step
whose GPU result misses the oracle tolerances (pre-step state, action, GPU after-state) to
gpurun_out/obst_fails.npz for CPU-side analysis."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_obstacles as T  # noqa: E402
from conftest import f64_state  # noqa: E402
from mujoco_playground_amd import _lib  # noqa: E402
from mujoco_playground_amd.model import blob as B  # noqa: E402

blob = _lib.load_blob("obstacles")
h = B.unpack_header(blob)
g = [i for i in range(h.ngeom) if h.geom_type[i] == 6]
c = np.array([list(h.geom_pos[i]) for i in g]); s = np.array([list(h.geom_size[i]) for i in g])
lo, hi = c - s, c + s
rng = np.random.default_rng(5)
n, steps = 512, 120
st = T.wall_states(n, lo, hi, rng)
sim = T.make_sim(n, seed=5)
sim.set_state(T.to_device(st))
gen = torch.Generator(device="cpu").manual_seed(5)
acts = []
for _ in range(steps):
    a = torch.rand(n, 2, generator=gen) * 2 - 1
    a[:, 0] = 0.4 + 0.6 * torch.rand(n, generator=gen)
    acts.append(a.to(T.DEV))
o = T.oracle(blob)
fails = []
alldv, alldq = [], []
for k in range(steps):
    before = f64_state(sim.state)
    sim.step(acts[k], autoreset=True)
    torch.cuda.synchronize()
    after = f64_state(sim.state)
    ref = before.copy()
    a_np = acts[k].cpu().numpy()
    o.step(ref, a_np, flags=3, seed=5)
    dq = np.abs(after[:, :13] - ref[:, :13]).max(axis=1)
    dv = np.abs(after[:, 13:25] - ref[:, 13:25]).max(axis=1)
    alldv.append(dv); alldq.append(dq)
    for e in np.nonzero((dq > T.TOL_QPOS) | (dv > T.TOL_QVEL))[0]:
        ex = T._excused(o, before[e], a_np[e], after[e], 3, 5)
        fails.append((k, e, dq[e], dv[e], ex, before[e], a_np[e], after[e], ref[e]))
        print(k, e, dq[e], dv[e], "excused" if ex else "NOT excused", flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
if fails:
    np.savez(os.path.join(ROOT, "gpurun_out", "obst_fails.npz"), k=[f[0] for f in fails], e=[f[1] for f in fails],
             excused=[f[4] for f in fails], before=np.array([f[5] for f in fails]),
             action=np.array([f[6] for f in fails]), after=np.array([f[7] for f in fails]),
             oracle=np.array([f[8] for f in fails]))
alldv, alldq = np.concatenate(alldv), np.concatenate(alldq)
print("dqvel quantiles 50/90/99/99.9/99.99/max", np.quantile(alldv, [0.5, 0.9, 0.99, 0.999, 0.9999, 1.0]))
print("dqpos quantiles 50/90/99/99.9/99.99/max", np.quantile(alldq, [0.5, 0.9, 0.99, 0.999, 0.9999, 1.0]))
print("fails", len(fails), "not excused", sum(1 for f in fails if not f[4]))
