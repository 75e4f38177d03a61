"""Per-phase cycle breakdown of ackphys_step_kernel from the stamped diagnostic build.

    tools/build_diag.sh && python tools/stamps.py [quad|obst]
    (STAMPS_ROLLOUT=K: step K - 1 of K-step ackphys_rollout launches for the lane kernels, a mid-rollout
    step whose state goes to the LDS mirror; the last step for the quad kernels, which store the state
    every step; STAMPS_JSON=path: merge the
    per-kernel summaries into that file, e.g. profiles/critical_path_latest.json)
Phases (stamp k -> k+1): 0 load/controller, 1 kinematics->dynamics entry, 2 M/bias/a0,
3 contacts, 4 rows+warmstart, 5 Newton, 6 force+Euler solve, 7 (return) -> 8 obs prep,
8 obs/reward write, 9 integrate+store.
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

NSTAMP = 24  # AK_NSTAMP of the diagnostic build
ROLL = int(os.environ.get("STAMPS_ROLLOUT", "1"))  # > 1: stamp one step of an ackphys_rollout launch of ROLL steps
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

# (from stamp, to stamp, name): the kernel's stamps in execution order
PHASES = [(0, 1, "load+controller"), (1, 2, "kin->dyn"), (2, 3, "M/bias/a0"), (3, 4, "contacts"),
          (4, 5, "rows+warm"), (5, 6, "newton"), (6, 7, "force+euler solve"), (7, 8, "integrate"),
          (8, 9, "barriers"), (9, 10, "state store"), (11, 12, "obs wave: rays")]


# contacts-off kernel: when each event happens, cycles after the dynamics wave's first stamp
TIMELINE = [(1, "dyn: state loaded"), (21, "prep: loads issued"), (22, "prep: controller done"),
            (23, "prep: rows done"), (20, "dyn: waits for prep words"), (13, "prep: ctrl+rows published"),
            (15, "dyn: prep words received"), (11, "obs: head done"), (16, "prep: Euler factor published"),
            (17, "dyn: waits for Euler factor"), (18, "dyn: Euler factor received"), (12, "obs: own rays done"),
            (14, "prep: rays published"), (19, "obs: prep rays received"), (7, "dyn: dynamics done"),
            (8, "dyn: integrated"), (9, "dyn: past barriers"), (10, "dyn: state stored")]


QUAD_PHASES = [(0, 1, "load+controller"), (1, 2, "kinematics"), (2, 3, "M/bias/a0"), (3, 4, "contacts"),
               (4, 5, "rows"), (5, 6, "newton"), (6, 10, "post-newton")]


def main():
    quad = len(sys.argv) > 1 and sys.argv[1] in ("quad", "obst")
    obst = len(sys.argv) > 1 and sys.argv[1] == "obst"
    # lane rollout: the stamped step is a mid-rollout one (no HBM state store; its span ends past the barriers)
    mid = ROLL > 1 and not quad
    phases = QUAD_PHASES if quad else ([ph for ph in PHASES if ph[2] != "state store"] if mid else PHASES)
    L = C.CDLL(os.path.join(REPO, "diag_libs", os.environ.get("DIAG_LIB", "libackphys_stamps.so")))
    P = C.c_void_p
    L.ackphys_create.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_int, C.POINTER(P)]
    L.ackphys_step.argtypes = [P] * 10 + [C.c_uint32, C.c_uint64, P]
    L.ackphys_reset.argtypes = [P, P, C.c_uint64, P, P, P]
    L.ackphys_random_actions.argtypes = [P, P, C.c_int, C.c_uint64, C.c_uint32, P]
    L.ackphys_diag_set_stamps.argtypes = [P]
    L.ackphys_rollout.argtypes = [P, C.c_int] + [P] * 9 + [C.c_uint32, C.c_uint64, C.c_int, P]
    sys.path.insert(0, REPO)
    from mujoco_playground_amd import _lib
    blob = _lib.load_blob("obstacles" if obst else "flat")
    n = 4096
    dev = torch.device("cuda:0")
    ctx = P()
    assert L.ackphys_create(blob, len(blob), n, 0, C.byref(ctx)) == 0
    L.ackphys_set_variant.argtypes = [P, C.c_int]
    assert L.ackphys_set_variant(ctx, 1 if quad else 0) == 0
    state = torch.zeros(44, n, device=dev)
    obs = torch.zeros(79, n, device=dev)
    rew = torch.zeros(n, device=dev)
    term = torch.zeros(n, dtype=torch.uint8, device=dev)
    trunc = torch.zeros(n, dtype=torch.uint8, device=dev)
    epw = 8 if quad else 64  # envs per workgroup of the stamped launch (quad_epw)
    nb = (n + epw - 1) // epw
    stamps = torch.zeros(NSTAMP * nb + nb * 64 + 5 * nb, dtype=torch.int64, device=dev)
    assert L.ackphys_diag_set_stamps(P(stamps.data_ptr())) == 0
    p = lambda t: P(t.data_ptr())
    stream = P(torch.cuda.current_stream().cuda_stream)
    acts = torch.zeros(300, n, 2, device=dev)
    L.ackphys_random_actions(ctx, p(acts), 300, 0, 0, stream)
    summary = {}
    # quad / obstacle kernels: contacts on only (the bench's contacts-off leg runs the lane kernel)
    for flags, label in ([(3, "contacts ON")] if quad else [(2, "contacts OFF"), (3, "contacts ON")]):
        state.zero_()
        L.ackphys_reset(ctx, None, 0, p(state), p(obs), stream)
        for k in range(200):
            L.ackphys_step(ctx, p(acts[k]), p(state), p(obs), p(rew), p(term), p(trunc), None, None, None, flags, 0,
                           stream)
        torch.cuda.synchronize()
        res, spans = [], []
        for k in range(200, 210):
            stamps.zero_()
            if ROLL > 1:  # the stamps left are those of step ROLL - 1 (lane) or of the last step (quad)
                L.ackphys_rollout(ctx, ROLL, p(acts[k]), p(state), p(obs), p(rew), p(term), p(trunc), None, None, None,
                                  flags, 0, 0, stream)
            else:
                L.ackphys_step(ctx, p(acts[k]), p(state), p(obs), p(rew), p(term), p(trunc), None, None, None, flags,
                               0, stream)
            torch.cuda.synchronize()
            allv = stamps.cpu().numpy()
            s = allv[: NSTAMP * nb].reshape(NSTAMP, nb)
            res.append(np.stack([s[b] - s[a] for a, b, _ in phases]))
            spans.append(np.sum(res[-1], axis=0) if quad else (s[9] - s[0] if mid else s[10] - s[0]))
            its = allv[NSTAMP * nb:NSTAMP * nb + 64 * nb]
            nt = allv[NSTAMP * nb + 64 * nb:].reshape(5, nb)
            if k == 200:
                print("  newton phases (median cycles/wave, summed over iterations): " + ", ".join(
                    f"{nm} {np.median(nt[i]):.0f}" for i, nm in enumerate(["grad+H", "chol+solve", "Jp+Mp", "LS", "update"]))
                    + f"; sum {np.median(nt.sum(0)):.0f} vs newton span {np.median(s[6] - s[5]):.0f}")
            its = its[: 64 * nb]
            if quad:
                its = its.reshape(nb, 64)[:, :epw].reshape(-1)
            if k == 200:
                ls = its >> 8
                its = its & 0xFF
                if quad:
                    lsw = ls.reshape(nb, -1).max(axis=1)
                    print(f"  line-search phi' evaluations per lane: mean {ls.mean():.2f} (per Newton iteration "
                          f"{ls.sum() / max((its // 8).sum(), 1):.2f}), hist {np.bincount(ls, minlength=4)[:20]}, "
                          f"wave-max hist {np.bincount(lsw, minlength=4)[:30]}")
                itn, why = its // 8, its % 8
                wmax = itn.reshape(nb, -1).max(axis=1)
                print(f"  iterations: lane mean {itn.mean():.2f}, lane hist {np.bincount(itn, minlength=13)}, "
                      f"wave-max hist {np.bincount(wmax, minlength=13)}, exit reasons (1 exact,2 grad,3 nodesc,4 maxit) "
                      f"{np.bincount(why, minlength=5)[1:]}")
            if not quad and k == 200 and flags == 2:
                print("  timeline (median cycles after the dynamics wave's first stamp): " + ", ".join(
                    f"{nm} {np.median(s[i] - s[0]):.0f}" for i, nm in TIMELINE if s[i].any()))
            if quad and k == 200:  # both waves' timeline from the dynamics wave's first stamp of the step
                tl = [(1, "dyn: loaded"), (4, "dyn: contacts done"), (5, "dyn: Newton starts"),
                      (6, "dyn: Newton done"), (9, "dyn: at barrier 1"), (13, "dyn: past barrier 1"),
                      (10, "dyn: stored"), (11, "obs: starts"), (14, "obs: slots published"), (12, "obs: at barrier 1"),
                      (2, "dyn: dynamics entry"), (3, "dyn: M/bias/a0 done")]
                print("  timeline (median cycles after dyn stamp 0): " + ", ".join(
                    f"{nm} {np.median(s[i] - s[0]):.0f}" for i, nm in tl if s[i].any()))
        d = np.median(np.concatenate(res, axis=1), axis=1)
        tot = np.median(np.concatenate(spans))
        print(f"== {label}: median cycles per wave, total {tot:.0f}")
        for (_, _, name), v in zip(phases, d):
            print(f"  {name:16s} {v:10.0f}  {100 * v / tot:5.1f}%")
        kern = (("obst8_kernel" if ROLL > 1 else "obst_kernel") if obst else
                ("quad_kernel" if quad else ("nc_kernel" if flags == 2 else "kernel")))
        label = f"{label}, {'obstacle scene' if obst else 'flat scene'}, {'quad' if quad else 'lane'} mapping"
        summary[label] = {"kernel": ("ackphys_rollout_" if ROLL > 1 else "ackphys_step_") + kern,
                          "dyn_wave_cycles_per_step_median": float(tot),
                          "dyn_wave_cycles_per_step_max": float(np.max(np.concatenate(spans))),
                          "phases_median": {name: float(v) for (_, _, name), v in zip(phases, d)},
                          "measured": "diag build (s_memtime stamps, ~+11 % cycles), 4096 envs, steps 200-209 after "
                                      "reset, " + ((f"step {ROLL - 1} of {ROLL}-step rollout launches (mid-rollout: "
                                                    "the state into the LDS mirror)" if mid else
                                                    f"last step of {ROLL}-step rollout launches") if ROLL > 1
                                                   else "single-step launches")}
    if os.environ.get("STAMPS_JSON"):  # merged into the file's other entries (one file for every kernel)
        import json
        old = {}
        if os.path.exists(os.environ["STAMPS_JSON"]):
            with open(os.environ["STAMPS_JSON"]) as f:
                old = json.load(f)
        old.update(summary)
        with open(os.environ["STAMPS_JSON"], "w") as f:
            json.dump(old, f, indent=1)


if __name__ == "__main__":
    main()
