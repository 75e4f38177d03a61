"""PPO.train() time per minibatch (the bench's update: 4096 envs x 32 steps, batch 8192, 10 epochs) for
several libackppo builds, each in its own child process (GPU box).

    python tools/probes/update_time.py LIBACKPPO.so [...] [--reps 3]

One line per build: median us per minibatch over the reps, all reps, and a checksum of the
parameters after the timed calls (builds that should agree bit for bit can be compared).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def child(lib, reps):
    sys.path.insert(0, REPO)
    import torch
    from mujoco_playground_amd import _lib
    _lib.PPO_LIB_PATH = os.path.abspath(lib)
    from mujoco_playground_amd.rl import AckermannVecEnv
    from mujoco_playground_amd.rl.ppo import PPO
    dev = torch.device("cuda:0")
    venv = AckermannVecEnv(4096, device=dev, seed=0, contacts=True)
    model = PPO("MlpPolicy", venv, n_steps=32, batch_size=8192, n_epochs=10, seed=0)
    model.collect_rollouts()
    nmb = 32 * 4096 // 8192 * 10
    model.train()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        model.train()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / nmb)
    print(json.dumps({"lib": lib, "us_per_minibatch": sorted(ts)[len(ts) // 2], "all": [round(t, 2) for t in ts],
                      "checksum": float(model.params.double().abs().sum())}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--child", default=None)
    a = ap.parse_args()
    if a.child:
        child(a.child, a.reps)
        return
    for lib in a.libs:
        r = subprocess.run([sys.executable, __file__, "--child", lib, "--reps", str(a.reps)], timeout=300)
        if r.returncode:
            print(f"{lib}: exit {r.returncode}", flush=True)
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
