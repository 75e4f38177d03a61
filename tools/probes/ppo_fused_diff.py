"""GPU probe: where the fused PPO rollout and the per-step path differ (first mismatches per buffer).
    python tools/probes/ppo_fused_diff.py [scene]"""
import os
import sys

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
            print("    steps", sorted(set((rows // n).tolist()))[:20], "cols", sorted(set(torch.nonzero(d)[:, 1].tolist())))
            st = (rows // n)
            env = rows % n
            print("    starts of those envs at those steps", [float(a.buf_start[s_, e_]) for s_, e_ in zip(st[:8].tolist(), env[:8].tolist())])
