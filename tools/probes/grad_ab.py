"""A/B the gradient partial rows of two libackppo builds on identical inputs (GPU box).

    python tools/probes/grad_ab.py LIB_A.so LIB_B.so

Prints, per parameter block of the flat layout (rl/ppo.py LAYOUT), the max |difference| of the
partial rows the two builds' ackppo_grad writes, so a staging / operand change that should keep
the bits can be checked block by block.
"""
import ctypes as C
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from mujoco_playground_amd.rl.ppo import LAYOUT, NPARAM  # noqa: E402

dev = torch.device("cuda:0")


def grads(path, B=8192):
    L = C.CDLL(path)
    p, i32, f32 = C.c_void_p, C.c_int, C.c_float
    L.ackppo_grad.argtypes = [p] * 7 + [i32, p, f32, f32, f32, p, p, p]
    L.ackppo_grad_blocks.argtypes = [i32]
    g = torch.Generator(device="cpu").manual_seed(0)
    S = 131072
    params = (torch.randn(NPARAM, generator=g) * 0.1).to(dev)
    obs = torch.randn(S, 79, generator=g).to(dev)
    act = torch.randn(S, 2, generator=g).to(dev)
    lp, adv, ret = (torch.randn(S, generator=g).to(dev) for _ in range(3))
    idx = torch.randperm(S, generator=g).to(torch.int32).to(dev)
    stats = torch.tensor([0.0, 1.0], device=dev)
    nblk = L.ackppo_grad_blocks(B)
    gp, lpart = torch.zeros(nblk, NPARAM, device=dev), torch.zeros(nblk, 8, device=dev)
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert L.ackppo_grad(P(params), P(obs), P(act), P(lp), P(adv), P(ret), P(idx), B, P(stats), 0.2, 0.0, 0.5,
                         P(gp), P(lpart), s) == 0
    torch.cuda.synchronize()
    return gp.cpu().numpy(), lpart.cpu().numpy()


a, la = grads(sys.argv[1])
b, lb = grads(sys.argv[2])
for k, (o, shp) in LAYOUT.items():
    n = int(np.prod(shp))
    d = np.abs(a[:, o:o + n] - b[:, o:o + n]).max()
    print(f"{k:40s} max|diff| {d:.3e}  max|a| {np.abs(a[:, o:o + n]).max():.3e}")
print("loss rows max|diff|", np.abs(la - lb).max())
print("bit-identical:", bool((a == b).all() and (la == lb).all()))
