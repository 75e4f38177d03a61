"""Why did the obstacle wall-contact step change when the quad dynamics wave was compiled as a called
function (AK_DYN_NOINLINE)?

    python tools/probes/noinline_probe.py find  <libackphys.so>   -> gpurun_out/noinl_case.npz
    python tools/probes/noinline_probe.py step  <libackphys.so> <tag> -> gpurun_out/noinl_step_<tag>.npz

find: test_obstacle_wall_contacts' workload (512 robots at box walls, 120 steps, teacher-forced vs
the f64 oracle) on the given build; records every env-step beyond the tolerances that the oracle's
boundary excuse does not cover (state before, action, GPU state after), and the whole batch's state
before the first such step.
step: replays that recorded step on the given build -- the failing env alone (n = 1) and inside
its original batch (n = 512) -- and saves the states after, so the inline and noinline builds can be
compared value by value.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
OUT = os.path.join(ROOT, "gpurun_out")


def use_lib(path):
    from mujoco_playground_amd import _lib
    _lib.LIB_PATH = os.path.abspath(path)
    return _lib


def workload():
    import test_gpu_obstacles as TO
    from mujoco_playground_amd import _lib
    sblob = _lib.load_blob("obstacles")
    from mujoco_playground_amd.model import blob as B
    h = B.unpack_header(sblob)
    g = [i for i in range(h.ngeom) if h.geom_type[i] == 6]
    c = np.array([list(h.geom_pos[i]) for i in g])
    s = np.array([list(h.geom_size[i]) for i in g])
    lo, hi = c - s, c + s
    rng = np.random.default_rng(5)
    n, steps = 512, 120
    st = TO.wall_states(n, lo, hi, rng)
    gen = torch.Generator(device="cpu").manual_seed(5)
    acts = []
    for _ in range(steps):
        a = torch.rand(n, 2, generator=gen) * 2 - 1
        a[:, 0] = 0.4 + 0.6 * torch.rand(n, generator=gen)
        acts.append(a)
    return sblob, st, acts, TO


def find(path):
    use_lib(path)
    from conftest import f64_state
    from mujoco_playground_amd.sim import BatchedAckermannSim
    sblob, st, acts, TO = workload()
    sim = BatchedAckermannSim(len(st), "cuda:0", seed=5, scene="obstacles")
    sim.set_state(TO.to_device(st))
    o = TO.oracle(sblob)
    cases = []
    first_batch = None
    for k in range(len(acts)):
        before = f64_state(sim.state)
        a = acts[k].to("cuda:0")
        sim.step(a, autoreset=True)
        torch.cuda.synchronize()
        after = f64_state(sim.state)
        ref = before.copy()
        a_np = acts[k].numpy()
        o.step(ref, a_np, flags=3, seed=5)
        dq = np.abs(after[:, :13] - ref[:, :13]).max(axis=1)
        dv = np.abs(after[:, 13:25] - ref[:, 13:25]).max(axis=1)
        for e in np.nonzero((dq > TO.TOL_QPOS) | (dv > TO.TOL_QVEL))[0]:
            if TO._excused(o, before[e], a_np[e], after[e], 3, 5):
                continue
            print(f"step {k} env {e}: |dqpos| {dq[e]:.3e} |dqvel| {dv[e]:.3e}", flush=True)
            cases.append((k, e, before[e], a_np[e], after[e], ref[e]))
            if first_batch is None:
                first_batch = (k, before.copy(), a_np.copy())
    if not cases:
        print("no unexcused step: this build passes", flush=True)
        return
    k0, bb, ba = first_batch
    np.savez(os.path.join(OUT, "noinl_case.npz"), k=np.array([c[0] for c in cases]),
             e=np.array([c[1] for c in cases]), before=np.array([c[2] for c in cases]),
             action=np.array([c[3] for c in cases]), after=np.array([c[4] for c in cases]),
             oracle=np.array([c[5] for c in cases]), batch_k=k0, batch_before=bb, batch_action=ba)
    print(f"{len(cases)} unexcused env-steps; first at step {k0}", flush=True)


def step(path, tag):
    use_lib(path)
    import test_gpu_obstacles as TO
    from conftest import f64_state
    from mujoco_playground_amd.sim import BatchedAckermannSim
    d = np.load(os.path.join(OUT, "noinl_case.npz"))
    e0 = int(d["e"][0])
    res = {}
    # the failing env alone, and inside its original batch
    for name, st, act in (("alone", d["before"][:1], d["action"][:1]), ("batch", d["batch_before"], d["batch_action"])):
        sim = BatchedAckermannSim(len(st), "cuda:0", seed=5, scene="obstacles")
        sim.set_state(TO.to_device(st))
        sim.step(torch.tensor(act, device="cuda:0"), autoreset=True)
        torch.cuda.synchronize()
        res[name] = f64_state(sim.state)
    np.savez(os.path.join(OUT, f"noinl_step_{tag}.npz"), alone=res["alone"], batch=res["batch"], e0=e0)
    print(tag, "alone qvel", np.round(res["alone"][0, 13:25], 5), flush=True)
    print(tag, "batch qvel", np.round(res["batch"][e0, 13:25], 5), flush=True)
    print("oracle     qvel", np.round(d["oracle"][0, 13:25], 5), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "find":
        find(sys.argv[2])
    else:
        step(sys.argv[2], sys.argv[3])
