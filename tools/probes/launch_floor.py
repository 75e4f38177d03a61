"""Launch-floor probe (GPU box): per-launch time of empty / load-store / load-chain-store kernels of
the contacts-off kernel's grid (4096 envs, 64 workgroups of 192 threads), timed like bench.py
(HIP events around 1000 back-to-back launches on one stream).

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o mujoco_playground_amd/csrc/build/libprobe_floor.so \\
        tools/probes/launch_floor.hip && python tools/probes/launch_floor.py
"""
import ctypes as C
import os

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    L = C.CDLL(os.path.join(REPO, "mujoco_playground_amd", "csrc", "build", "libprobe_floor.so"))
    L.probe_launch.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    n = 4096
    s = torch.zeros(37, n, device="cuda")
    st = torch.cuda.current_stream()
    for which, name in enumerate(["empty", "load+store 37 words", "+1000 FMAs, 1 chain", "+1000 FMAs, 2 chains",
                                      "+1000 FMAs, 4 chains", "+2000 FMAs, 1 chain"]):
        L.probe_launch(which, C.c_void_p(s.data_ptr()), n, 50, C.c_void_p(st.cuda_stream))
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        L.probe_launch(which, C.c_void_p(s.data_ptr()), n, 1000, C.c_void_p(st.cuda_stream))
        b.record()
        torch.cuda.synchronize()
        print(f"{name:24s} {a.elapsed_time(b):.3f} us per launch")


if __name__ == "__main__":
    main()
