"""Find the first teacher-forced parity miss of a variant and explain it with the oracle.

    python tools/parity_hunt.py --variant quad --contacts 1 [--n 256 --steps 150 --seed 11]

At the first step whose |dqpos| exceeds 1e-5 it evaluates MuJoCo's primal cost (oracle diag:
M, qacc_smooth, efc rows, J) at the oracle's qacc and at the GPU's (the qacc_warmstart words of
the GPU's new state): a GPU cost above the oracle's means the GPU solve stopped early.
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mujoco_playground_amd import _lib  # noqa: E402
from mujoco_playground_amd.sim import BatchedAckermannSim  # noqa: E402
from oracle.oracle import Oracle, controller  # noqa: E402


def f64(st):
    s = st.cpu().numpy().T.copy()
    out = s.astype(np.float64)
    out[:, 42:44] = s[:, 42:44].view(np.uint32)
    return out


def _floss():
    from mujoco_playground_amd.model.blob import unpack_header
    m = unpack_header(_lib.load_blob())
    return np.array(m.dof_frictionloss[:12])


FLOSS = None


def primal_cost(d, a):
    global FLOSS
    if FLOSS is None:
        FLOSS = _floss()
    a0 = d["qacc_smooth"]
    c = 0.5 * (a - a0) @ d["qM"] @ (a - a0)
    for row, J in zip(d["efc"], d["efc_J"]):
        typ, pos, R, aref, force, diag = row
        x = J @ a - aref
        D = 1.0 / R
        if typ == 0:
            c += 0.5 * D * x * x
        elif typ == 1:  # frictionloss (Huber) on the dof the row's J selects; R*floss is the knee
            fl = FLOSS[int(np.argmax(np.abs(J)))]
            c += 0.5 * D * x * x if abs(x) < R * fl else fl * abs(x) - 0.5 * R * fl * fl
        elif x < 0:
            c += 0.5 * D * x * x
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="quad")
    ap.add_argument("--contacts", type=int, default=1)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--steps", type=int, default=150)
    ap.add_argument("--seed", type=int, default=11)
    a = ap.parse_args()
    sim = BatchedAckermannSim(a.n, "cuda:0", seed=a.seed, contacts=bool(a.contacts), variant=a.variant)
    sim.reset()
    acts = sim.random_actions(a.steps, seed=a.seed)
    o = Oracle(_lib.load_blob())
    flags = (1 if a.contacts else 0) | 2
    for k in range(a.steps):
        before = f64(sim.state)
        sim.step(acts[k], autoreset=True)
        torch.cuda.synchronize()
        after = f64(sim.state)
        ref = before.copy()
        o.step(ref, acts[k].cpu().numpy(), flags=flags, seed=a.seed)
        dq = np.abs(after[:, :13] - ref[:, :13]).max(axis=1)
        if dq.max() > 1e-5:
            e = int(np.argmax(dq))
            print(f"step {k}: env {e} |dqpos| {dq[e]:.3e}; {int((dq > 1e-5).sum())} envs over 1e-5")
            ctrl = controller(acts[k, e].cpu().numpy())
            d = o.diag(before[e], ctrl, flags=flags & 1)
            R = None
            q = before[e, 3:7] / np.linalg.norm(before[e, 3:7])
            w, x, y, z = q
            R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                          [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                          [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
            qacc_gpu = after[e, 25:37].copy()
            print("ncon", d["ncon"], "nefc", d["nefc"], "oracle niter", d["niter"])
            print("oracle qacc", np.round(d["qacc"], 4))
            print("gpu    qacc", np.round(qacc_gpu, 4))
            print("cost oracle", primal_cost(d, d["qacc"]), "cost gpu", primal_cost(d, qacc_gpu))
            print("efc types", d["efc"][:, 0].astype(int).tolist())
            print("efc pos", np.round(d["efc"][:, 1], 5).tolist())
            print("contacts (pos, dist, geom)", np.round(d["contacts"], 4).tolist())
            np.savez(os.path.join("gpurun_out", "hunt.npz"), before=before[e], after=after[e], ref=ref[e],
                     action=acts[k, e].cpu().numpy(), step=k, env=e)
            return
    print("no parity miss")


if __name__ == "__main__":
    main()
