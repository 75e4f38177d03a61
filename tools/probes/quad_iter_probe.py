"""Debug probe (stamped diagnostic build): Newton iterations / line-search evaluations of the quad
obstacle kernel for the states saved by variant_ray_probe.py (gpurun_out/variant_step_probe.npz).

    bash tools/build_diag.sh && python tools/probes/quad_iter_probe.py
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, REPO)
from mujoco_playground_amd import _lib  # noqa: E402

L = C.CDLL(os.path.join(REPO, "mujoco_playground_amd", "csrc", "build", "libackphys_stamps.so"))
P = C.c_void_p
L.ackphys_create.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_int, C.POINTER(P)]
L.ackphys_step.argtypes = [P] * 10 + [C.c_uint32, C.c_uint64, P]
L.ackphys_diag_set_stamps.argtypes = [P]
L.ackphys_set_variant.argtypes = [P, C.c_int]
d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "variant_step_probe.npz"))
chain, act = d["chain"], d["act"]
blob = _lib.load_blob("obstacles")
n, dev = 1, torch.device("cuda:0")
ctx = P()
assert L.ackphys_create(blob, len(blob), n, 0, C.byref(ctx)) == 0
assert L.ackphys_set_variant(ctx, 1) == 0
nb = 1
stamps = torch.zeros(24 * nb + nb * 64 + 5 * nb, dtype=torch.int64, device=dev)
assert L.ackphys_diag_set_stamps(P(stamps.data_ptr())) == 0
p = lambda t: P(t.data_ptr())
s = P(torch.cuda.current_stream().cuda_stream)
obs = torch.zeros(79, n, device=dev)
rew = torch.zeros(n, device=dev)
term = torch.zeros(n, dtype=torch.uint8, device=dev)
trunc = torch.zeros(n, dtype=torch.uint8, device=dev)
a = torch.tensor(act.reshape(1, 2), device=dev)
for j in range(3):
    st = chain[j].astype(np.float32)
    st[42:44] = chain[j][42:44].astype(np.uint32).view(np.float32)
    state = torch.tensor(st.reshape(44, 1), device=dev)
    stamps.zero_()
    assert L.ackphys_step(ctx, p(a), p(state), p(obs), p(rew), p(term), p(trunc), None, None, None, 1, 9, s) == 0
    torch.cuda.synchronize()
    rec = int(stamps.cpu().numpy()[24 * nb])
    nx = state.cpu().numpy()[:, 0].astype(np.float64)
    print(f"substep {j}: it_done {(rec & 255) // 8} flag {rec & 7} ls_evals {rec >> 8} "
          f"|qvel - chain| {np.abs(nx[13:25] - chain[j + 1][13:25]).max():.3g}")
