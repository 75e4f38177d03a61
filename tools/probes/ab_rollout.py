"""A/B timing of ackphys_rollout between two builds of libackphys.so (same C-ABI subset):
contacts on, 4096 envs, K steps per launch, interleaved repetitions.

    python tools/probes/ab_rollout.py libA.so libB.so [K] [reps]
"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from mujoco_playground_amd import _lib  # noqa: E402


def setup(path, n, K, flags, scene):
    L = C.CDLL(os.path.abspath(path))
    P = C.c_void_p
    L.ackphys_create.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_int, C.POINTER(P)]
    L.ackphys_reset.argtypes = [P, P, C.c_uint64, P, P, P]
    L.ackphys_random_actions.argtypes = [P, P, C.c_int, C.c_uint64, C.c_uint32, P]
    L.ackphys_rollout.argtypes = [P, C.c_int] + [P] * 9 + [C.c_uint32, C.c_uint64, C.c_int, P]
    blob = _lib.load_blob(scene)
    ctx = P()
    assert L.ackphys_create(blob, len(blob), n, 0, C.byref(ctx)) == 0
    dev = torch.device("cuda:0")
    b = dict(state=torch.zeros(44, n, device=dev), obs=torch.zeros(K, 79, n, device=dev),
             rew=torch.zeros(K, n, device=dev), term=torch.zeros(K, n, dtype=torch.uint8, device=dev),
             trunc=torch.zeros(K, n, dtype=torch.uint8, device=dev), acts=torch.zeros(K, n, 2, device=dev))
    p = lambda t: P(t.data_ptr())
    s = P(torch.cuda.current_stream().cuda_stream)
    L.ackphys_random_actions(ctx, p(b["acts"]), K, 0, 0, s)
    L.ackphys_reset(ctx, None, 0, p(b["state"]), p(b["obs"][0]), s)

    def run():
        rc = L.ackphys_rollout(ctx, K, p(b["acts"]), p(b["state"]), p(b["obs"]), p(b["rew"]), p(b["term"]),
                               p(b["trunc"]), None, None, None, flags, 0, 0, s)
        assert rc == 0
    for _ in range(3):
        run()
    return run


def main():
    a, bpath = sys.argv[1], sys.argv[2]
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 6
    for scene, flags in (("flat", 3), ("obstacles", 3), ("flat", 2)):
        runs = {"A": setup(a, 4096, K, flags, scene), "B": setup(bpath, 4096, K, flags, scene)}
        res = {"A": [], "B": []}
        for _ in range(reps):
            for k, run in runs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run()
                e1.record()
                torch.cuda.synchronize()
                res[k].append(e0.elapsed_time(e1) * 1000 / K)
        print(scene, "flags", flags, {k: [round(x, 2) for x in sorted(v)] for k, v in res.items()}, flush=True)


if __name__ == "__main__":
    main()
