"""GPU probe: host-clocked vs event-timed 20-step windows, the driver's bench shape
(`--steps 20 --warmup 5`), under different preludes: a fresh sim right after start-up, after the
~0.2 s clock warm-up on a throwaway sim, and back to back. Prints one JSON line per window.
With `spin` the HIP runtime is asked to spin-wait on synchronisation (hipDeviceScheduleSpin)
before anything touches the GPU. The last passes poll the end event (hipEventQuery) from the host
before the synchronise ("query": true) against the plain synchronise.

    python tools/probes/short_window_probe.py [spin]
"""
import ctypes
import gc
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from mujoco_playground_amd.sim import BatchedAckermannSim  # noqa: E402


def window(dev, tag, keep=None):
    sim = BatchedAckermannSim(4096, dev, seed=0, contacts=False)
    sim.reset()
    acts = sim.random_actions(25, seed=0)
    sim.rollout(acts[:5], want_info=False, per_step_outputs=False)
    timed = acts[5:]
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    launch = sim.rollout_launcher(timed) if FAST else None
    torch.cuda.synchronize(dev)
    if FAST:
        gc.disable()
    t0 = time.perf_counter()
    ev0.record()
    if FAST:
        launch()
    else:
        sim.rollout(timed, want_info=False, per_step_outputs=False)
    t_launch = time.perf_counter()
    ev1.record()
    if QUERY:  # poll the end event from the host before the synchronise
        while not ev1.query():
            pass
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    gc.enable()
    print(json.dumps({"prelude": tag, "fast": FAST, "query": QUERY, "host_us": round((t1 - t0) * 1e6, 1), "launch_call_us": round((t_launch - t0) * 1e6, 1),
                      "event_us": round(ev0.elapsed_time(ev1) * 1e3, 1)}), flush=True)
    if keep is not None:
        keep.append(sim)


FAST = False
QUERY = False


def main():
    global FAST, QUERY
    if len(sys.argv) > 1 and sys.argv[1] == "spin":
        hip = ctypes.CDLL("libamdhip64.so")
        print(json.dumps({"hipSetDeviceFlags(spin)": hip.hipSetDeviceFlags(ctypes.c_uint(1))}), flush=True)
    for FAST in (False, True):
        run()
    FAST = True
    for QUERY in (True, False, True):
        run()


def run():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    window(dev, "first")
    window(dev, "second")
    bench.clock_warm(dev, 4096)
    window(dev, "after clock_warm")
    window(dev, "again")
    keep = []
    for i in range(3):
        window(dev, f"kept sims {i}", keep)
    bench.clock_warm(dev, 4096)
    torch.cuda.synchronize(dev)
    time.sleep(0.05)
    window(dev, "after clock_warm + 50 ms idle")


if __name__ == "__main__":
    main()
