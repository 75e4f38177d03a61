"""Time PPO.train() (the bench's update: 4096 envs x 32 steps, batch 8192, 10 epochs) with the
gradient launches' weight image on and off, alternating, on one rollout buffer (GPU box).

    python tools/probes/ppo_update_ab.py [reps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mujoco_playground_amd.rl import AckermannVecEnv  # noqa: E402
from mujoco_playground_amd.rl.ppo import PPO  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda:0")
    venv = AckermannVecEnv(4096, device=dev, seed=0, contacts=True)
    model = PPO("MlpPolicy", venv, n_steps=32, batch_size=8192, n_epochs=10, seed=0)
    model.collect_rollouts()
    nmb = 32 * 4096 // 8192 * 10
    res = {True: [], False: []}
    for _ in range(reps):
        for img in (True, False):
            model.set_weight_image(img)
            model.train()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            model.train()
            e1.record()
            torch.cuda.synchronize()
            res[img].append(e0.elapsed_time(e1) * 1e3 / nmb)
    for img, v in res.items():
        print(f"weight_image={img}: us per minibatch {[round(x, 2) for x in v]}", flush=True)


if __name__ == "__main__":
    main()
