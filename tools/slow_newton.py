"""Collect env steps whose Newton solve needs many iterations (stamped diagnostic build, lane
kernel) -> gpurun_out/slow_cases.npz (pre-step state, action, iterations, exit reason).

    tools/build_diag.sh && python tools/slow_newton.py [--contacts 0] [--steps 300] [--min-it 8]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--contacts", type=int, default=0)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--min-it", type=int, default=8)
    a = ap.parse_args()
    L = C.CDLL(os.path.join(REPO, "diag_libs", "libackphys_stamps.so"))
    P = C.c_void_p
    L.ackphys_create.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_int, C.POINTER(P)]
    L.ackphys_step.argtypes = [P] * 10 + [C.c_uint32, C.c_uint64, P]
    L.ackphys_reset.argtypes = [P, P, C.c_uint64, P, P, P]
    L.ackphys_random_actions.argtypes = [P, P, C.c_int, C.c_uint64, C.c_uint32, P]
    L.ackphys_diag_set_stamps.argtypes = [P]
    L.ackphys_set_variant.argtypes = [P, C.c_int]
    blob = open(os.path.join(REPO, "mujoco_playground_amd", "model", "assets", "ackermann_robot_v2.apm"), "rb").read()
    n, dev = 4096, torch.device("cuda:0")
    ctx = P()
    assert L.ackphys_create(blob, len(blob), n, 0, C.byref(ctx)) == 0
    assert L.ackphys_set_variant(ctx, 0) == 0
    state = torch.zeros(44, n, device=dev)
    obs = torch.zeros(79, n, device=dev)
    rew = torch.zeros(n, device=dev)
    term = torch.zeros(n, dtype=torch.uint8, device=dev)
    trunc = torch.zeros(n, dtype=torch.uint8, device=dev)
    nb = n // 64
    stamps = torch.zeros(16 * nb + nb * 64 + 5 * nb, dtype=torch.int64, device=dev)
    assert L.ackphys_diag_set_stamps(P(stamps.data_ptr())) == 0
    p = lambda t: P(t.data_ptr())
    s = P(torch.cuda.current_stream().cuda_stream)
    acts = torch.zeros(a.steps, n, 2, device=dev)
    L.ackphys_random_actions(ctx, p(acts), a.steps, 0, 0, s)
    L.ackphys_reset(ctx, None, 0, p(state), p(obs), s)
    flags = (1 if a.contacts else 0) | 2
    cases, hist = [], np.zeros(13, np.int64)
    for k in range(a.steps):
        before = state.clone()
        L.ackphys_step(ctx, p(acts[k]), p(state), p(obs), p(rew), p(term), p(trunc), None, None, None, flags, 0, s)
        torch.cuda.synchronize()
        its = stamps.cpu().numpy()[16 * nb:16 * nb + 64 * nb]
        itn, why = its // 8, its % 8
        hist += np.bincount(itn, minlength=13)[:13]
        for e in np.nonzero(itn >= a.min_it)[0][:4]:
            st = before[:, e].cpu().numpy()
            cases.append((st, acts[k, e].cpu().numpy(), int(itn[e]), int(why[e]), k, int(e)))
    print("iteration histogram over all env-steps:", hist.tolist())
    print(f"{len(cases)} slow cases (>= {a.min_it} iterations); first: ",
          [(c[2], c[3], c[4], c[5]) for c in cases[:10]])
    if cases:
        np.savez(os.path.join(REPO, "gpurun_out", "slow_cases.npz"),
                 state=np.stack([c[0] for c in cases]), action=np.stack([c[1] for c in cases]),
                 it=np.array([c[2] for c in cases]), why=np.array([c[3] for c in cases]),
                 step=np.array([c[4] for c in cases]), env=np.array([c[5] for c in cases]))


if __name__ == "__main__":
    main()
