"""Event-timed contacts-on rollout launches for several step-library builds (GPU box).

    python tools/probes/quad_time.py LIB.so[:EPW] ... [--steps 1000] [--scene flat|obstacles]

Each build is loaded in a child process (one library per process), runs the bench's workload
(4096 envs, reset, 200 settle steps, then one ackphys_rollout launch of --steps steps, event-timed,
three times) and prints one line: library, envs per wave, us per step (median of 3), and the
state checksum (so builds that should agree bit for bit can be compared).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def child(lib, steps, scene, contacts, variant="auto"):
    sys.path.insert(0, REPO)
    import torch
    from mujoco_playground_amd import _lib
    _lib.LIB_PATH = os.path.abspath(lib)
    from mujoco_playground_amd.sim import BatchedAckermannSim
    dev = torch.device("cuda:0")
    sim = BatchedAckermannSim(4096, dev, seed=0, contacts=contacts, scene=scene, variant=variant)
    sim.reset()
    acts = sim.random_actions(200 + 3 * steps, seed=0)
    sim.rollout(acts[:200], want_info=False, per_step_outputs=False)
    torch.cuda.synchronize()
    ts = []
    for r in range(3):
        a = acts[200 + r * steps:200 + (r + 1) * steps]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        sim.rollout(a, want_info=False, per_step_outputs=False)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / steps)
    st = sim.state.double()
    print(json.dumps({"lib": os.path.basename(lib), "scene": scene, "epw": os.environ.get("ACKPHYS_QUAD_EPW", "8"),
                      "us_per_step": sorted(ts)[1], "all": ts, "checksum": float(st.abs().sum().item()),
                      "finite": bool(torch.isfinite(sim.state).all().item())}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--scene", default="flat", help="flat, obstacles or both")
    ap.add_argument("--contacts", type=int, default=1)
    ap.add_argument("--variant", default="auto")
    ap.add_argument("--child", default=None)
    a = ap.parse_args()
    if a.child:
        child(a.child, a.steps, a.scene, bool(a.contacts), a.variant)
        return
    rc = 0
    for spec in a.libs:
        lib, _, epw = spec.partition(":")
        env = dict(os.environ)
        if epw:
            env["ACKPHYS_QUAD_EPW"] = epw
        for scene in (("flat", "obstacles") if a.scene == "both" else (a.scene,)):
            r = subprocess.run([sys.executable, __file__, "--child", lib, "--steps", str(a.steps), "--scene", scene,
                                "--contacts", str(a.contacts), "--variant", a.variant], env=env, timeout=300)
            if r.returncode:
                print(f"{spec}: exit {r.returncode}", flush=True)
                sys.exit(r.returncode)
    sys.exit(rc)


if __name__ == "__main__":
    main()
