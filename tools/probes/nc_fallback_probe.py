"""GPU probe (diag build): how many contacts-off lanes leave the predicted piece for the Newton
fallback, on the random states of tests/test_gpu_parity.py::test_contacts_off_random_states.

    tools/build_diag.sh && python tools/probes/nc_fallback_probe.py
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

NSTAMP = 24  # AK_NSTAMP of the diagnostic build
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    L = C.CDLL(os.path.join(REPO, "mujoco_playground_amd", "csrc", "build", "libackphys_stamps.so"))
    P = C.c_void_p
    L.ackphys_create.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_int, C.POINTER(P)]
    L.ackphys_step.argtypes = [P] * 10 + [C.c_uint32, C.c_uint64, P]
    L.ackphys_reset.argtypes = [P, P, C.c_uint64, P, P, P]
    L.ackphys_random_actions.argtypes = [P, P, C.c_int, C.c_uint64, C.c_uint32, P]
    L.ackphys_diag_set_stamps.argtypes = [P]
    L.ackphys_set_variant.argtypes = [P, C.c_int]
    blob = open(os.path.join(REPO, "mujoco_playground_amd", "model", "assets", "ackermann_robot_v2.apm"), "rb").read()
    n = 512
    dev = torch.device("cuda:0")
    ctx = P()
    assert L.ackphys_create(blob, len(blob), n, 0, C.byref(ctx)) == 0
    assert L.ackphys_set_variant(ctx, 0) == 0
    p = lambda t: P(t.data_ptr())
    stream = P(torch.cuda.current_stream().cuda_stream)
    nb = (n + 63) // 64
    stamps = torch.zeros(NSTAMP * nb + nb * 64 + 5 * nb, dtype=torch.int64, device=dev)
    assert L.ackphys_diag_set_stamps(p(stamps)) == 0
    obs = torch.zeros(79, n, device=dev)
    rew = torch.zeros(n, device=dev)
    term = torch.zeros(n, dtype=torch.uint8, device=dev)
    trunc = torch.zeros(n, dtype=torch.uint8, device=dev)
    acts = torch.zeros(4, n, 2, device=dev)
    # the benchmark workload's first steps from reset (the driver's short runs time steps 5..25)
    n4 = 4096
    ctx4 = P()
    assert L.ackphys_create(blob, len(blob), n4, 0, C.byref(ctx4)) == 0
    assert L.ackphys_set_variant(ctx4, 0) == 0
    nb4 = (n4 + 63) // 64
    st4 = torch.zeros(NSTAMP * nb4 + nb4 * 64 + 5 * nb4, dtype=torch.int64, device=dev)
    state4, obs4 = torch.zeros(44, n4, device=dev), torch.zeros(79, n4, device=dev)
    rew4, term4, trunc4 = (torch.zeros(n4, device=dev), torch.zeros(n4, dtype=torch.uint8, device=dev),
                           torch.zeros(n4, dtype=torch.uint8, device=dev))
    acts4 = torch.zeros(40, n4, 2, device=dev)
    L.ackphys_random_actions(ctx4, p(acts4), 40, 0, 0, stream)
    L.ackphys_reset(ctx4, None, 0, p(state4), p(obs4), stream)
    assert L.ackphys_diag_set_stamps(p(st4)) == 0
    for k in range(40):
        st4.zero_()
        L.ackphys_step(ctx4, p(acts4[k]), p(state4), p(obs4), p(rew4), p(term4), p(trunc4), None, None, None, 2, 0,
                       stream)
        torch.cuda.synchronize()
        it = (st4.cpu().numpy()[NSTAMP * nb4: NSTAMP * nb4 + 64 * nb4] & 0xFF) // 8
        w = it.reshape(-1, 64).max(1)
        print(f"bench step {k}: lane hist {np.bincount(it, minlength=4)[:6]} wave-max hist {np.bincount(w, minlength=4)[:6]}")
    assert L.ackphys_diag_set_stamps(p(stamps)) == 0
    for seed in (31, 32, 33):
        rng = np.random.default_rng(seed)
        st = np.zeros((n, 44))
        q = rng.normal(size=(n, 4))
        q /= np.linalg.norm(q, axis=1, keepdims=True)
        st[:, 0:3] = rng.uniform(-2, 2, (n, 3))
        st[:, 3:7] = q
        st[:, 7:13] = rng.uniform(-3, 3, (n, 6))
        st[:, [9, 11]] = rng.uniform(-0.8, 0.8, (n, 2))
        st[:, 13:19] = rng.normal(0, 2, (n, 6))
        st[:, 19:25] = rng.normal(0, 20, (n, 6))
        st[:, [21, 23]] = rng.normal(0, 3, (n, 2))
        st[:, 25:37] = rng.normal(0, 50, (n, 12))
        state = torch.tensor(st.T.astype(np.float32), device=dev)
        L.ackphys_random_actions(ctx, p(acts), 4, seed, 0, stream)
        for k in range(4):
            stamps.zero_()
            L.ackphys_step(ctx, p(acts[k]), p(state), p(obs), p(rew), p(term), p(trunc), None, None, None, 2, seed,
                           stream)
            torch.cuda.synchronize()
            it = (stamps.cpu().numpy()[NSTAMP * nb: NSTAMP * nb + 64 * nb] & 0xFF) // 8
            print(f"seed {seed} step {k}: Newton iterations after the predicted piece, lane hist "
                  f"{np.bincount(it, minlength=4)[:8]}")


if __name__ == "__main__":
    main()
