"""Success-rate curve of the learnable variant (action_repeat 10, nohit_clear) for several builds and
seeds: is a change in the test_ppo_learns_the_variant_task number systematic or seed noise? (GPU box)

    python tools/probes/variant_learn.py PHYS.so:PPO.so ... [--seeds 0,1,2] [--iters 100,300]

Each build pair runs in a child process; one JSON line per (build, seed) with the deterministic-policy
success after each checkpoint of PPO iterations (4096 envs x 64 steps each).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def child(phys, ppo, seed, iters):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import torch
    from mujoco_playground_amd import _lib
    _lib.LIB_PATH, _lib.PPO_LIB_PATH = os.path.abspath(phys), os.path.abspath(ppo)
    from train_ppo import evaluate
    from mujoco_playground_amd.rl import make_ackermann_env
    from mujoco_playground_amd.rl.ppo import PPO
    kw = dict(action_repeat=10, nohit_clear=True)
    venv = make_ackermann_env(env_type="vec", num_envs=4096, device=torch.device("cuda:0"), seed=seed,
                              max_episode_steps=1000, **kw)
    model = PPO("MlpPolicy", venv, n_steps=64, batch_size=8192, n_epochs=10, seed=seed)
    done, curve = 0, {}
    for it in iters:
        model.learn(total_timesteps=(it - done) * 64 * 4096, reset_num_timesteps=False)
        done = it
        curve[it] = round(evaluate(model, horizon=1000, **kw)[0], 4)
    print(json.dumps({"phys": os.path.basename(phys), "ppo": os.path.basename(ppo), "seed": seed, "success": curve}),
          flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("builds", nargs="*")
    ap.add_argument("--seeds", default="0,1,2")
    ap.add_argument("--iters", default="100,300")
    ap.add_argument("--child", default=None)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    iters = [int(x) for x in a.iters.replace("+", ",").split(",")]
    if a.child:
        phys, ppo = a.child.split(":")
        child(phys, ppo, a.seed, iters)
        return
    for spec in a.builds:
        for s in a.seeds.replace("+", ",").split(","):
            r = subprocess.run([sys.executable, __file__, "--child", spec, "--seed", s, "--iters", a.iters.replace("+", ",")],
                               timeout=400)
            if r.returncode:
                print(f"{spec} seed {s}: exit {r.returncode}", flush=True)
                sys.exit(r.returncode)


if __name__ == "__main__":
    main()
