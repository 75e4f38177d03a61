"""Where a fused PPO rollout step's time goes (stamped diagnostic build, tools/build_diag.sh): per
workgroup, the cycles of the dynamics wave (state loaded -> barrier 1) against the observation
wave's observation, TimeLimit bootstrap and policy (all before barrier 1), for step T - 2 of an
n_steps rollout (the last step runs the critic alone). 4096 envs, 16 per workgroup: the stamps are
those of dynamics wave 0 and observation wave 2 (the actor's; the diagnostic build flushes no others).

    python tools/probes/ppo_rollout_stamps.py [flat|obstacles]
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
NSTAMP = 24


def main(scene):
    from mujoco_playground_amd import _lib
    _lib.LIB_PATH = os.path.join(ROOT, "diag_libs", "libackphys_stamps.so")  # tools/build_diag.sh; before the first load
    import torch
    from mujoco_playground_amd.rl import AckermannVecEnv
    from mujoco_playground_amd.rl.ppo import PPO
    L = _lib.lib()
    L.ackphys_diag_set_stamps.argtypes = [C.c_void_p]
    dev = torch.device("cuda:0")
    n = 4096
    venv = AckermannVecEnv(n, device=dev, seed=0, contacts=True, scene=scene)
    model = PPO("MlpPolicy", venv, n_steps=32, batch_size=8192, n_epochs=10, seed=0)
    nb = (n + 15) // 16
    stamps = torch.zeros(NSTAMP * nb + nb * 64 + 5 * nb, dtype=torch.int64, device=dev)
    assert L.ackphys_diag_set_stamps(C.c_void_p(stamps.data_ptr())) == 0
    for _ in range(3):  # past the first episodes' start-up
        model.collect_rollouts()
    rows = []
    for _ in range(5):
        stamps.zero_()
        model.collect_rollouts()
        torch.cuda.synchronize()
        s = stamps.cpu().numpy()[: NSTAMP * nb].reshape(NSTAMP, nb).astype(np.int64)
        ok = (s[0] > 0) & (s[9] > 0) & (s[11] > 0) & (s[15] > 0) & (s[14] > 0)
        ok &= (s[16] > 0) & (s[17] > 0) & (s[18] > 0) & (s[19] > 0)
        # slot 13 is written by both waves (the observation wave's "bootstrap done", then the dynamics
        # wave's "past barrier 1", which lands last): the bootstrap and policy spans are taken from
        # stamps 12 and 14 together, and slot 13 is read as the dynamics wave's
        rows.append(np.stack([s[9] - s[0], s[12] - s[11], s[14] - s[12], s[15] - s[14], s[13] - s[9],
                              s[11] - s[0], s[15] - s[11], s[17] - s[16], s[18] - s[17], s[19] - s[18],
                              s[14] - s[19], s[1] - s[0]])[:, ok])
    r = np.concatenate(rows, axis=1)
    names = ["dyn: loaded -> barrier 1", "obs: observation", "obs: bootstrap + policy", "obs: waits at barrier 1",
             "dyn: at barrier 1 -> past it", "obs entry - dyn entry", "obs: entry -> past barrier 1",
             "policy: layer 2", "policy: heads", "policy: rollout rows", "policy: sample + controller",
             "dyn: loaded -> controller"]
    print(f"== {scene} scene, PPO rollout step T-2, {r.shape[1]} workgroup samples; cycles (median / p90)")
    for nm, v in zip(names, r):
        print(f"  {nm:30s} {np.median(v):9.0f} {np.percentile(v, 90):9.0f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "flat")
