"""Per-step time and shader clock of the open-loop contacts-on rollout and the fused PPO rollout
(GPU box; the stamped diagnostic build, tools/build_diag.sh): LOOP_CLOCK records s_memtime and
s_memrealtime (100 MHz) at the loop top of the first and the last step of each workgroup, so
cycles per step, microseconds per step and the clock the workgroup ran at come from one launch.

    python3 tools/probes/step_clock.py
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
NSTAMP = 24
ROW = NSTAMP + 69  # LOOP_CLOCK's rows: clock / realtime at step 0, clock / realtime at the last step


def report(name, stamps, nb, steps):
    s = stamps.cpu().numpy()
    rows = s[ROW * nb:(ROW + 4) * nb].reshape(4, nb).astype(np.int64)
    ok = (rows > 0).all(axis=0)
    c = (rows[2] - rows[0])[ok] / (steps - 1)
    r = (rows[3] - rows[1])[ok] / (steps - 1) / 100.0
    ghz = c / (r * 1e3)
    print(f"{name}: {ok.sum()} workgroups, {steps} steps; per step (median / p10 / p90): cycles "
          f"{np.median(c):.0f} / {np.percentile(c, 10):.0f} / {np.percentile(c, 90):.0f}, us {np.median(r):.2f} / "
          f"{np.percentile(r, 10):.2f} / {np.percentile(r, 90):.2f}, clock GHz {np.median(ghz):.3f}", flush=True)


def main():
    from mujoco_playground_amd import _lib
    _lib.LIB_PATH = os.path.join(ROOT, "diag_libs", "libackphys_stamps.so")
    import torch
    from mujoco_playground_amd.rl import AckermannVecEnv
    from mujoco_playground_amd.rl.ppo import PPO
    from mujoco_playground_amd.sim import BatchedAckermannSim
    L = _lib.lib()
    L.ackphys_diag_set_stamps.argtypes = [C.c_void_p]
    dev = torch.device("cuda:0")
    n = 4096
    nb = (n + 7) // 8
    stamps = torch.zeros((ROW + 4) * nb, dtype=torch.int64, device=dev)
    assert L.ackphys_diag_set_stamps(C.c_void_p(stamps.data_ptr())) == 0
    sim = BatchedAckermannSim(n, dev, seed=0, contacts=True)
    sim.reset()
    acts = sim.random_actions(300, seed=0)
    sim.rollout(acts[:200], want_info=False, per_step_outputs=False)
    for _ in range(2):
        stamps.zero_()
        sim.rollout(acts[200:300], want_info=False, per_step_outputs=False)
        torch.cuda.synchronize()
        report("open-loop contacts-on rollout", stamps, nb, 100)
    venv = AckermannVecEnv(n, device=dev, seed=0, contacts=True)
    model = PPO("MlpPolicy", venv, n_steps=32, batch_size=8192, n_epochs=10, seed=0)
    for i in range(4):
        stamps.zero_()
        model.collect_rollouts()
        torch.cuda.synchronize()
        if i >= 2:
            report("fused PPO rollout", stamps, nb, 32)


if __name__ == "__main__":
    main()
