"""Algorithmic FLOPs per env-step, counted in the CPU oracle (host tool, no GPU).

The oracle's FLOP-counting build (`make -C oracle flops`: ackphys_oracle.c compiled as C++ with
oracle/flops/fd.hpp, a double that counts + - * / sqrt per OR_STAGE) runs the benchmark workload
through `ackphys_step_cpu` -- reset, uniform random actions, auto-reset -- and the per-stage counts
divided by the env-steps are written to profiles/oracle_flops.json, which bench.py reads to report
the effective FP32 rate (oracle FLOPs per env-step x env-steps/s) against the vector peak. These
are the reference algorithm's operations (MuJoCo's mj_step restated in f64: dense 12x12
factorisations, every ray against every geom with its bounding tests, the Newton solver with its
line searches), not what the GPU kernels execute.

    python tools/count_flops.py [--envs 256] [--steps 200]
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mujoco_playground_amd import _lib  # noqa: E402  (model blobs only)

STAGES = ["glue", "controller", "kinematics", "mass matrix", "collision", "sensors (rays)", "velocity/bias/actuation",
          "qacc_smooth", "constraint rows", "Newton solver", "Euler", "obs/reward", "reset"]
CONFIGS = [  # (name, scene, flags, untimed steps from reset: bench.py's warm-up / landing settle)
    ("configs[1] contacts off", "flat", 2, 50),
    ("configs[2] contacts on", "flat", 3, 200),
    ("configs[4] obstacle scene, contacts on", "obstacles", 3, 200),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "oracle_flops.json"))
    a = ap.parse_args()
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "flops"], check=True, capture_output=True)
    L = C.CDLL(os.path.join(REPO, "oracle", "build", "libackphys_oracle_flops.so"))
    P, i32, u32, u64 = C.c_void_p, C.c_int, C.c_uint32, C.c_uint64
    L.or_create.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(P)]
    L.ackphys_reset_cpu.argtypes = [P, i32, P, u64, P, P]
    L.ackphys_step_cpu.argtypes = [P, i32] + [P] * 9 + [u32, u64, i32]
    ULL = C.c_ulonglong * 16
    L.or_flops_read.argtypes = [ULL, ULL, i32]
    n = a.envs
    ptr = lambda x: x.ctypes.data_as(P)
    res = {"note": __doc__.split("\n\n")[1].replace("\n", " "), "envs": n, "configs": {}}
    for name, scene, flags, warm in CONFIGS:
        blob = _lib.load_blob(scene)
        ctx = P()
        assert L.or_create(blob, len(blob), C.byref(ctx)) == 0
        st = np.zeros((44, n), np.float32)
        obs, rew = np.zeros((79, n), np.float32), np.zeros(n, np.float32)
        term, trunc = np.zeros(n, np.uint8), np.zeros(n, np.uint8)
        tobs, info, ep = np.zeros((79, n), np.float32), np.zeros((4, n), np.float32), np.zeros((4, n), np.float32)
        assert L.ackphys_reset_cpu(ctx, n, None, 7, ptr(st), ptr(obs)) == 0
        rng = np.random.default_rng(0)
        for k in range(warm + a.steps):
            if k == warm:
                L.or_flops_reset()
            act = np.ascontiguousarray(rng.uniform(-1, 1, (n, 2)).astype(np.float32))
            assert L.ackphys_step_cpu(ctx, n, ptr(act), ptr(st), ptr(obs), ptr(rew), ptr(term), ptr(trunc), ptr(tobs),
                                      ptr(info), ptr(ep), flags, 7, 1) == 0
        fl, tr = ULL(), ULL()
        L.or_flops_read(fl, tr, 16)
        es = n * a.steps
        counts = {STAGES[i]: fl[i] / es for i in range(len(STAGES)) if fl[i]}
        total = sum(fl) / es
        res["configs"][name] = {"scene": scene, "flags": flags, "untimed_steps": warm, "counted_steps": a.steps,
                                "flops_per_env_step": total, "transcendentals_per_env_step": sum(tr) / es,
                                "per_stage": counts}
        print(f"{name}: {total:.0f} FLOPs/env-step (+{sum(tr) / es:.0f} transcendental calls); " +
              ", ".join(f"{k} {v:.0f}" for k, v in counts.items()))
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
