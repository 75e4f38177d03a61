"""Time the PPO kernels of one or more libackppo builds (event-timed, B=8192 minibatch, 4096 envs).
    python tools/ppo_kbench.py path/to/libackppo.so [...]"""
import ctypes as C
import sys

import numpy as np
import torch

NP = 18764
dev = torch.device("cuda:0")


def P(t):
    return C.c_void_p(t.data_ptr())


def run(path):
    L = C.CDLL(path)
    p32, i32, f32, u32, u64, i64 = C.c_void_p, C.c_int, C.c_float, C.c_uint32, C.c_uint64, C.c_int64
    L.ackppo_act.argtypes = [p32, p32, i32, i64, u64, u32, i32, p32, p32, p32, p32, p32, p32]
    L.ackppo_grad.argtypes = [p32] * 7 + [i32, p32, f32, f32, f32, p32, p32, p32]
    L.ackppo_reduce.argtypes = [p32, p32, i32, f32, p32, p32, p32]
    L.ackppo_adam.argtypes = [p32, p32, p32, p32, f32, f32, f32, f32, f32, f32, f32, p32, p32]
    g = torch.Generator(device="cpu").manual_seed(0)
    params = (torch.randn(NP, generator=g) * 0.1).to(dev)
    S, B, N = 131072, 8192, 4096
    obs = torch.randn(S, 79, device=dev)
    act = torch.randn(S, 2, device=dev)
    lp = torch.randn(S, device=dev)
    adv = torch.randn(S, device=dev)
    ret = torch.randn(S, device=dev)
    idx = torch.randperm(S, device=dev).to(torch.int32)
    stats = torch.tensor([0.0, 1.0], device=dev)
    L.ackppo_grad_blocks.argtypes = [i32]
    nblk = L.ackppo_grad_blocks(B)
    gp, lpart = torch.zeros(nblk, NP, device=dev), torch.zeros(nblk, 8, device=dev)
    grad, loss = torch.zeros(NP, device=dev), torch.zeros(8, device=dev)
    m, v, nrm = torch.zeros(NP, device=dev), torch.zeros(NP, device=dev), torch.zeros(1, device=dev)
    obs_soa = torch.randn(79, N, device=dev)
    ea, a2, l2, v2 = (torch.zeros(N, 2, device=dev), torch.zeros(N, 2, device=dev), torch.zeros(N, device=dev),
                      torch.zeros(N, device=dev))
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = {}
    for name, fn in [
        ("grad", lambda: L.ackppo_grad(P(params), P(obs), P(act), P(lp), P(adv), P(ret), P(idx), B, P(stats), 0.2, 0.0,
                                       0.5, P(gp), P(lpart), s)),
        ("reduce", lambda: L.ackppo_reduce(P(gp), P(lpart), nblk, 0.0, P(grad), P(loss), s)),
        ("adam", lambda: L.ackppo_adam(P(params), P(grad), P(m), P(v), 1.0, 0.5, 0.9, 0.999, 1e-5, 3e-4, 0.03,
                                       P(nrm), s)),
        ("act", lambda: L.ackppo_act(P(params), P(obs_soa), N, 0, 1, 2, 0, None, P(a2), P(ea), P(l2), P(v2), s)),
    ]:
        for _ in range(3):
            assert fn() == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) / 20 * 1000, 1)
    import hashlib
    print(path, res, "grad checksum", float(grad.abs().sum()), "grad sha1",
          hashlib.sha1(grad.cpu().numpy().tobytes()).hexdigest()[:12], flush=True)


if __name__ == "__main__" and (len(sys.argv) < 2 or sys.argv[1] != "--stamps"):
    for p in sys.argv[1:]:
        run(p)


def stamps(path, batches=(8192, 4096)):
    """Per-phase cycles of ackppo_grad from the PP_STAMPS build (median over workgroups), and the
    launch's timeline from the 100 MHz clock (stamps 13 / 14: workgroup start / end): span, start
    skew, median workgroup duration; for each minibatch size."""
    L = C.CDLL(path)
    p32, i32, f32 = C.c_void_p, C.c_int, C.c_float
    L.ackppo_grad.argtypes = [p32] * 7 + [i32, p32, f32, f32, f32, p32, p32, p32]
    L.ackppo_diag_set_stamps.argtypes = [p32]
    S = 131072
    params = (torch.randn(NP) * 0.1).to(dev)
    obs, act = torch.randn(S, 79, device=dev), torch.randn(S, 2, device=dev)
    lp, adv, ret = torch.randn(S, device=dev), torch.randn(S, device=dev), torch.randn(S, device=dev)
    idx = torch.randperm(S, device=dev).to(torch.int32)
    stats = torch.tensor([0.0, 1.0], device=dev)
    L.ackppo_grad_blocks.argtypes = [C.c_int]
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for B in batches:
        nblk = L.ackppo_grad_blocks(B)
        gp, lpart = torch.zeros(nblk, NP, device=dev), torch.zeros(nblk, 8, device=dev)
        st = torch.zeros(16 * 2 * nblk, dtype=torch.int64, device=dev)  # grad1: two workgroups per row
        L.ackppo_diag_set_stamps(P(st))
        call = lambda: L.ackppo_grad(P(params), P(obs), P(act), P(lp), P(adv), P(ret), P(idx), B, P(stats), 0.2,  # noqa: E731
                                     0.0, 0.5, P(gp), P(lpart), s)
        for _ in range(3):
            call()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            call()
        e1.record()
        torch.cuda.synchronize()
        a = st.cpu().numpy().reshape(16, -1)
        a = a[:, : int((a[0] != 0).sum())]
        used = [k for k in range(13) if a[k].any()]
        ph = {f"{used[i]}->{used[i + 1]}": int(np.median(a[used[i + 1]] - a[used[i]])) for i in range(len(used) - 1)}
        t0, t1 = a[13], a[14]
        print(f"batch {B}: {a.shape[1]} workgroups, event-timed {e0.elapsed_time(e1) / 10 * 1e3:.1f} us; "
              f"phases (median cycles per workgroup) {ph} total {int(np.median(a[used[-1]] - a[used[0]]))}; "
              f"timeline (100 MHz): span {(t1.max() - t0.min()) / 100:.2f} us, start skew {(t0.max() - t0.min()) / 100:.2f} us, "
              f"median workgroup {np.median(t1 - t0) / 100:.2f} us, max {(t1 - t0).max() / 100:.2f} us", flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "--stamps":
    stamps(sys.argv[2])
