"""Dump the quad dynamics of one env (contact slots, qacc_smooth, final qacc; diagnostic AK_STAMPS
build) for the first failing case of noinline_probe.py, from a given build:

    python tools/probes/noinline_dump.py <libackphys_stamps*.so> <tag>   -> gpurun_out/noinl_dump_<tag>.npz

Build the two diagnostic libraries first (host only):
    bash tools/build_diag.sh                                   (inline dynamics wave)
    DIAG_OUT=libackphys_stamps_noinl.so bash tools/build_diag.sh -DAK_DYN_NOINLINE
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, REPO)
from mujoco_playground_amd import _lib  # noqa: E402

path, tag = sys.argv[1], sys.argv[2]
L = C.CDLL(path)
P = C.c_void_p
L.ackphys_create.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_int, C.POINTER(P)]
L.ackphys_step.argtypes = [P] * 10 + [C.c_uint32, C.c_uint64, P]
L.ackphys_diag_set_stamps.argtypes = [P]
L.ackphys_diag_set_dump.argtypes = [P]
L.ackphys_set_variant.argtypes = [P, C.c_int]
d = np.load(os.path.join(REPO, "tools", "probes", "data", "noinl_case.npz"))  # noinline_probe.py find (first case)
before, act = d["before"][0], d["action"][0]
blob = _lib.load_blob("obstacles")
dev = torch.device("cuda:0")
ctx = P()
assert L.ackphys_create(blob, len(blob), 1, 0, C.byref(ctx)) == 0
assert L.ackphys_set_variant(ctx, 1) == 0
stamps = torch.zeros(4096, dtype=torch.int64, device=dev)
dump = torch.zeros(4 * 12 * 40 + 24, dtype=torch.float32, device=dev)
assert L.ackphys_diag_set_stamps(P(stamps.data_ptr())) == 0
assert L.ackphys_diag_set_dump(P(dump.data_ptr())) == 0
p = lambda t: P(t.data_ptr())  # noqa: E731
s = P(torch.cuda.current_stream().cuda_stream)
obs = torch.zeros(79, 1, device=dev)
rew = torch.zeros(1, device=dev)
term = torch.zeros(1, dtype=torch.uint8, device=dev)
trunc = torch.zeros(1, dtype=torch.uint8, device=dev)
a = torch.tensor(act.reshape(1, 2).astype(np.float32), device=dev)
st = before.astype(np.float32)
st[42:44] = before[42:44].astype(np.uint32).view(np.float32)
state = torch.tensor(st.reshape(44, 1), device=dev)
assert L.ackphys_step(ctx, p(a), p(state), p(obs), p(rew), p(term), p(trunc), None, None, None, 1 | 2, 5, s) == 0
torch.cuda.synchronize()
out = dump.cpu().numpy()
slots = out[:4 * 12 * 40].reshape(4, 12, 40)
np.savez(os.path.join(REPO, "gpurun_out", f"noinl_dump_{tag}.npz"), slots=slots, a0=out[1920:1932],
         qacc=out[1932:1944], state=state.cpu().numpy()[:, 0])
print(tag, "slots on per lane:", (slots[:, :, 0] > 0).sum(axis=1), flush=True)
print(tag, "qacc_smooth", np.round(out[1920:1932], 4), flush=True)
print(tag, "qacc       ", np.round(out[1932:1944], 4), flush=True)
for q in range(4):
    for t in range(12):
        if slots[q, t, 0] > 0:
            print(tag, f"lane {q} slot {t}: P {np.round(slots[q, t, 1:4], 5)} D {slots[q, t, 4]:.4g} x {np.round(slots[q, t, 5:9], 4)} "
                  f"mu {slots[q, t, 9]:.3g} tran {slots[q, t, 10]:.4g} | at D: dist {slots[q, t, 35]:.6g} imp {slots[q, t, 36]:.6g} "
                  f"tran {slots[q, t, 37]:.6g} mu {slots[q, t, 38]:.6g} R {slots[q, t, 39]:.6g}", flush=True)
