"""Replay saved slow-Newton cases (tests/golden/slow_newton_cases.npz) one env at a time
through the printf trace build (tools/build_trace.sh)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
args = sys.argv[1:]
flags = 2
if args and args[0] == "--contacts":
    flags, args = 3, args[1:]
d = np.load(os.path.join(REPO, "tests", "golden",
                         "slow_newton_cases_contacts.npz" if flags & 1 else "slow_newton_cases.npz"))
idxs = [int(x) for x in args] or list(np.argsort(-d["it"])[:3])
L = C.CDLL(os.path.join(REPO, "mujoco_playground_amd", "csrc", "build", "libackphys_trace.so"))
P = C.c_void_p
L.ackphys_create.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_int, C.POINTER(P)]
L.ackphys_step.argtypes = [P] * 10 + [C.c_uint32, C.c_uint64, P]
L.ackphys_set_variant.argtypes = [P, C.c_int]
blob = open(os.path.join(REPO, "mujoco_playground_amd", "model", "assets", "ackermann_robot_v2.apm"), "rb").read()
dev = torch.device("cuda:0")
ctx = P()
assert L.ackphys_create(blob, len(blob), 1, 0, C.byref(ctx)) == 0
assert L.ackphys_set_variant(ctx, 0) == 0
p = lambda t: P(t.data_ptr())
for i in idxs:
    print(f"== case {i}: gpu iterations {d['it'][i]} why {d['why'][i]}", flush=True)
    st = torch.tensor(d["state"][i][:, None].copy(), device=dev)
    act = torch.tensor(d["action"][i][None].copy(), device=dev)
    obs, rew = torch.zeros(79, 1, device=dev), torch.zeros(1, device=dev)
    term, trunc = torch.zeros(1, dtype=torch.uint8, device=dev), torch.zeros(1, dtype=torch.uint8, device=dev)
    L.ackphys_step(ctx, p(act), p(st), p(obs), p(rew), p(term), p(trunc), None, None, None, flags, 0,
                   P(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
