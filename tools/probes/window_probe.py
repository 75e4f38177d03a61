"""GPU probe: fixed cost of a short timed window (the driver's `--steps 20 --warmup 5`).

For K in 1, 2, 5, 10, 20, 50, 200 steps (contacts off, 4096 envs): host time of the Python call
alone, host time of the whole window (synchronize -> rollout -> synchronize) and the event-timed
GPU span, best of 5, so fixed and per-step costs separate by a fit.

    python tools/probes/window_probe.py
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mujoco_playground_amd.sim import BatchedAckermannSim  # noqa: E402


def main():
    sim = BatchedAckermannSim(4096, "cuda:0", seed=0, contacts=False)
    sim.reset()
    acts = sim.random_actions(400, seed=0)
    sim.rollout(acts[:50], want_info=False, per_step_outputs=False)
    snap = sim.state.clone(), sim.episode.clone()
    rows = []
    for K in (1, 2, 5, 10, 20, 50, 200):
        a = acts[50:50 + K]
        best = None
        for _ in range(5):
            sim.state.copy_(snap[0])
            sim.episode.copy_(snap[1])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record()
            tc0 = time.perf_counter()
            sim.rollout(a, want_info=False, per_step_outputs=False)
            tc1 = time.perf_counter()
            e1.record()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            r = ((t1 - t0) * 1e6, e0.elapsed_time(e1) * 1e3, (tc1 - tc0) * 1e6)
            best = r if best is None or r[0] < best[0] else best
        row = {"K": K, "window_host_us": round(best[0], 2), "gpu_event_us": round(best[1], 2),
               "python_call_us": round(best[2], 2)}
        rows.append(row)
        print(json.dumps(row), flush=True)
    # least-squares fit of the event span: fixed + K * per_step
    n = len(rows)
    sx = sum(r["K"] for r in rows)
    sy = sum(r["gpu_event_us"] for r in rows)
    sxx = sum(r["K"] ** 2 for r in rows)
    sxy = sum(r["K"] * r["gpu_event_us"] for r in rows)
    b = (n * sxy - sx * sy) / (n * sxx - sx * sx)
    print(json.dumps({"fit_gpu_fixed_us": round((sy - b * sx) / n, 2), "fit_gpu_per_step_us": round(b, 3)}))


if __name__ == "__main__":
    main()
