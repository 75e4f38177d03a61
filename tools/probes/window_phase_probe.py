"""GPU probe: is the short window's higher per-step cost the launch (first steps of any launch)
or the physics (steps right after reset)? Event-timed rollout windows of K = 20 and 200 steps
starting 50 and 550 steps after reset (contacts off, 4096 envs), best of 5 each.

    python tools/probes/window_phase_probe.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mujoco_playground_amd.sim import BatchedAckermannSim  # noqa: E402


def main():
    sim = BatchedAckermannSim(4096, "cuda:0", seed=0, contacts=False)
    acts = sim.random_actions(1000, seed=0)
    for start in (5, 50, 550):
        sim.reset()
        if start:
            sim.rollout(acts[:start], want_info=False, per_step_outputs=False)
        snap = sim.state.clone(), sim.episode.clone()
        for K in (20, 200):
            best = None
            for _ in range(5):
                sim.state.copy_(snap[0])
                sim.episode.copy_(snap[1])
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                sim.rollout(acts[start:start + K], want_info=False, per_step_outputs=False)
                e1.record()
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1) * 1e3 / K
                best = t if best is None or t < best else best
            print(json.dumps({"start_step": start, "K": K, "gpu_us_per_step": round(best, 3)}), flush=True)


if __name__ == "__main__":
    main()
