"""GPU probe: why a short bench run (--steps 20 --warmup 5) measures slower kernels than the
1000-step run. Times the contacts-off step kernel (HIP events, 20 steps) in four situations:
fresh process right after reset; after ~0.2 s of other GPU work (clocks up); the same sim far
from reset; a fresh sim from reset right after that busy period.

    python tools/probes/short_run_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mujoco_playground_amd.sim import BatchedAckermannSim  # noqa: E402


def timed(sim, acts, k0, k):
    """GPU time per step of steps k0 .. k0+k-1, replayed from a captured graph (no host gaps)"""
    views = acts[k0:k0 + k].unbind(0)
    snap = sim.state.clone(), sim.episode.clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for v in views:
            sim.step(v, want_info=False)
    sim.state.copy_(snap[0])
    sim.episode.copy_(snap[1])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / k * 1e3


def main():
    dev = torch.device("cuda:0")
    n = 4096
    sim = BatchedAckermannSim(n, dev, seed=0, contacts=False)
    sim.reset()
    acts = sim.random_actions(3000, seed=0)
    for i in range(5):
        sim.step(acts[i], want_info=False)
    print(f"fresh process, steps 5-25 from reset: {timed(sim, acts, 5, 20):.2f} us/step")
    print(f"same sim, steps 25-45: {timed(sim, acts, 25, 20):.2f} us/step")
    busy = BatchedAckermannSim(n, dev, seed=1, contacts=True)
    busy.reset()
    b = busy.random_actions(3000, seed=1)
    for i in range(3000):
        busy.step(b[i], want_info=False)
    torch.cuda.synchronize()
    print(f"same sim after ~0.2 s of contacts-on stepping, steps 45-65: {timed(sim, acts, 45, 20):.2f} us/step")
    for i in range(65, 1000):
        sim.step(acts[i], want_info=False)
    print(f"same sim, steps 1000-1020: {timed(sim, acts, 1000, 20):.2f} us/step")
    s2 = BatchedAckermannSim(n, dev, seed=2, contacts=False)
    s2.reset()
    a2 = s2.random_actions(100, seed=2)
    for i in range(5):
        s2.step(a2[i], want_info=False)
    print(f"fresh sim after that, steps 5-25 from reset: {timed(s2, a2, 5, 20):.2f} us/step")
    print(f"fresh sim, steps 25-45: {timed(s2, a2, 25, 20):.2f} us/step")


if __name__ == "__main__":
    main()
