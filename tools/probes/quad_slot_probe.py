"""Debug probe (stamped diagnostic build): the quad obstacle kernel's contact slots of env 0 (chassis
point, D, start rows, mu, tran, Jacobian rows) and qacc for the state saved by variant_ray_probe.py
(substep 1 of tools/probes/data/variant_step_probe.npz) -> gpurun_out/quad_slot_probe.npz.

    bash tools/build_diag.sh && python tools/probes/quad_slot_probe.py [substep]
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, REPO)
from mujoco_playground_amd import _lib  # noqa: E402

j = int(sys.argv[1]) if len(sys.argv) > 1 else 1
L = C.CDLL(os.path.join(REPO, "mujoco_playground_amd", "csrc", "build", "libackphys_stamps.so"))
P = C.c_void_p
L.ackphys_create.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_int, C.POINTER(P)]
L.ackphys_step.argtypes = [P] * 10 + [C.c_uint32, C.c_uint64, P]
L.ackphys_diag_set_stamps.argtypes = [P]
L.ackphys_diag_set_dump.argtypes = [P]
L.ackphys_set_variant.argtypes = [P, C.c_int]
d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "variant_step_probe.npz"))
chain, act = d["chain"], d["act"]
blob = _lib.load_blob("obstacles")
dev = torch.device("cuda:0")
ctx = P()
assert L.ackphys_create(blob, len(blob), 1, 0, C.byref(ctx)) == 0
assert L.ackphys_set_variant(ctx, 1) == 0
stamps = torch.zeros(24 + 64 + 5, dtype=torch.int64, device=dev)
dump = torch.zeros(4 * 12 * 40 + 24, dtype=torch.float32, device=dev)
assert L.ackphys_diag_set_stamps(P(stamps.data_ptr())) == 0
assert L.ackphys_diag_set_dump(P(dump.data_ptr())) == 0
p = lambda t: P(t.data_ptr())
s = P(torch.cuda.current_stream().cuda_stream)
obs = torch.zeros(79, 1, device=dev)
rew = torch.zeros(1, device=dev)
term = torch.zeros(1, dtype=torch.uint8, device=dev)
trunc = torch.zeros(1, dtype=torch.uint8, device=dev)
a = torch.tensor(act.reshape(1, 2), device=dev)
st = chain[j].astype(np.float32)
st[42:44] = chain[j][42:44].astype(np.uint32).view(np.float32)
state = torch.tensor(st.reshape(44, 1), device=dev)
assert L.ackphys_step(ctx, p(a), p(state), p(obs), p(rew), p(term), p(trunc), None, None, None, 1, 9, s) == 0
torch.cuda.synchronize()
out = dump.cpu().numpy()
np.savez(os.path.join(REPO, "gpurun_out", "quad_slot_probe.npz"), slots=out[:4 * 12 * 40].reshape(4, 12, 40),
         a0=out[1920:1932], qacc=out[1932:1944], state=state.cpu().numpy()[:, 0])
print("slots on per lane:", (out[:1920].reshape(4, 12, 40)[:, :, 0] > 0).sum(axis=1))
