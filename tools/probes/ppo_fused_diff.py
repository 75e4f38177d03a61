"""GPU probe: where the fused PPO rollout and the per-step path differ (first mismatches per buffer).
    python tools/probes/ppo_fused_diff.py [scene [physics library under csrc/build]]"""
import os
import sys

if len(sys.argv) > 2:  # another build of the physics library (before the first load)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from mujoco_playground_amd import _lib as _l
    _l.LIB_PATH = os.path.join(os.path.dirname(_l.LIB_PATH), sys.argv[2])

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_gpu_ppo_rollout import BUFFERS, _pair  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "flat"
n, T = 301, 23
a, b = _pair(n, scene, T, eplen=9, thr=2.4)
a.collect_rollouts()
b.collect_rollouts()
torch.cuda.synchronize()
for name in BUFFERS:
    x, y = getattr(a, name), getattr(b, name)
    d = (x != y)
    print(name, tuple(x.shape), "mismatches", int(d.sum()))
    if d.any():
        idx = torch.nonzero(d)[:8].tolist()
        for i in idx:
            print("   ", i, float(x[tuple(i)]), float(y[tuple(i)]))
        if name == "buf_obs":
            rows = torch.nonzero(d.any(1)).flatten()
            r0 = int(rows[0])
            print("    row", r0, "fused  ", [round(float(v), 4) for v in x[r0, list(range(10)) + list(range(70, 79))]])
            print("    row", r0, "perstep", [round(float(v), 4) for v in y[r0, list(range(10)) + list(range(70, 79))]])
            print("    steps", sorted(set((rows // n).tolist()))[:20], "cols", sorted(set(torch.nonzero(d)[:, 1].tolist())))
            st = (rows // n)
            env = rows % n
            print("    starts of those envs at those steps", [float(a.buf_start[s_, e_]) for s_, e_ in zip(st[:8].tolist(), env[:8].tolist())])
