"""GPU probe: K steps as K launches (ackphys_step) vs one launch (ackphys_rollout), 4096 envs.

Prints host-clocked and event-timed microseconds per step for each workload and window length,
both paths from the same state (snapshot restored between them).

    python tools/probes/rollout_probe.py
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mujoco_playground_amd.sim import BatchedAckermannSim  # noqa: E402


def window(sim, acts, fused, per_step):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    if fused:
        sim.rollout(acts, want_info=False, per_step_outputs=per_step)
    else:
        for v in acts.unbind(0):
            sim.step(v, want_info=False)
    e1.record()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    k = acts.shape[0]
    return (t1 - t0) / k * 1e6, e0.elapsed_time(e1) / k * 1e3


def main():
    n = 4096
    out = []
    for name, kw, settle in (("contacts off", dict(contacts=False), 50),
                             ("contacts on", dict(contacts=True), 200),
                             ("obstacles", dict(contacts=True, scene="obstacles"), 200)):
        sim = BatchedAckermannSim(n, "cuda:0", seed=0, **kw)
        sim.reset()
        acts = sim.random_actions(settle + 1000, seed=0)
        for k in range(settle):
            sim.step(acts[k], want_info=False)
        snap = sim.state.clone(), sim.episode.clone()
        for K in (20, 100, 1000):
            a = acts[settle:settle + K].contiguous()
            row = {"workload": name, "K": K}
            for label, fused, per in (("steps", False, False), ("rollout", True, False), ("rollout_buf", True, True)):
                best = None
                for _ in range(3):
                    sim.state.copy_(snap[0])
                    sim.episode.copy_(snap[1])
                    r = window(sim, a, fused, per)
                    best = r if best is None or r[0] < best[0] else best
                row[label + "_host_us"], row[label + "_event_us"] = round(best[0], 3), round(best[1], 3)
            out.append(row)
            print(json.dumps(row), flush=True)
        del sim
    return out


if __name__ == "__main__":
    main()
