"""Fused PPO rollout and open-loop contacts-on rollout time for several libackphys builds, each in its
own child process (GPU box): ms per collect_rollouts() (4096 envs x 32 steps) and us per open-loop
step (4096 envs, 200 steps in one launch), with checksums of the rollout buffers and the sim state
(builds that should agree bit for bit can be compared).

    python3 tools/probes/rollout_time.py LIBACKPHYS.so [...] [--reps 5] [--scene obstacles]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def child(lib, reps, scene):
    sys.path.insert(0, REPO)
    from mujoco_playground_amd import _lib
    _lib.LIB_PATH = os.path.abspath(lib)
    import torch
    from mujoco_playground_amd.rl import AckermannVecEnv
    from mujoco_playground_amd.rl.ppo import PPO
    from mujoco_playground_amd.sim import BatchedAckermannSim
    dev = torch.device("cuda:0")
    venv = AckermannVecEnv(4096, device=dev, seed=0, contacts=True, scene=scene)
    model = PPO("MlpPolicy", venv, n_steps=32, batch_size=8192, n_epochs=10, seed=0)
    for _ in range(2):
        model.collect_rollouts()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        model.collect_rollouts()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ck = float(model.buf_obs.double().abs().sum() + model.buf_act.double().abs().sum() + model.buf_rew.double().abs().sum())
    sim = BatchedAckermannSim(4096, dev, seed=0, contacts=True, scene=scene)
    sim.reset()
    acts = sim.random_actions(400, seed=0)
    sim.rollout(acts[:200], want_info=False, per_step_outputs=False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    sim.rollout(acts[200:400], want_info=False, per_step_outputs=False)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"lib": lib, "ppo_rollout_ms": sorted(ts)[len(ts) // 2], "all": [round(t, 4) for t in ts],
                      "open_loop_us_per_step": e0.elapsed_time(e1) * 1e3 / 200, "ppo_checksum": ck,
                      "sim_checksum": float(sim.state.double().abs().sum())}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--child", default=None)
    ap.add_argument("--scene", default="flat")
    a = ap.parse_args()
    if a.child:
        child(a.child, a.reps, a.scene)
        return
    for lib in a.libs:
        r = subprocess.run([sys.executable, __file__, "--child", lib, "--reps", str(a.reps), "--scene", a.scene], timeout=300)
        if r.returncode:
            print(f"{lib}: exit {r.returncode}", flush=True)
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
