"""Per-phase cycles of the weight-image gradient launch (ackppo_grad1i_kernel) as PPO.train() runs it:
the PP_STAMPS build of libackppo (diag_libs/libackppo_stamps.so, see tools/ppo_kbench.py --stamps for
the plain ackppo_grad launch) keeps the stamps of the LAST gradient launch of a train() call (GPU box).

    python tools/probes/grad1i_stamps.py diag_libs/libackppo_stamps.so
"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    import torch
    from mujoco_playground_amd import _lib
    _lib.PPO_LIB_PATH = os.path.abspath(sys.argv[1])
    from mujoco_playground_amd.rl import AckermannVecEnv
    from mujoco_playground_amd.rl.ppo import PPO
    dev = torch.device("cuda:0")
    venv = AckermannVecEnv(4096, device=dev, seed=0, contacts=True)
    model = PPO("MlpPolicy", venv, n_steps=32, batch_size=8192, n_epochs=10, seed=0)
    model.collect_rollouts()
    L = _lib.ppo_lib()
    L.ackppo_diag_set_stamps.argtypes = [C.c_void_p]
    nblk = L.ackppo_grad_blocks(8192)
    st = torch.zeros(16 * 2 * nblk, dtype=torch.int64, device=dev)
    assert L.ackppo_diag_set_stamps(C.c_void_p(st.data_ptr())) == 0
    for _ in range(2):
        model.train()
    torch.cuda.synchronize()
    a = st.cpu().numpy().reshape(16, -1)
    used = [k for k in range(13) if a[k].any()]
    ph = {f"{used[i]}->{used[i + 1]}": int(np.median(a[used[i + 1]] - a[used[i]])) for i in range(len(used) - 1)}
    end = int(np.median(a[15] - a[8])) if a[15].any() else None
    t0, t1 = a[13], a[14]
    print(f"grad1i (train's last launch): {a.shape[1]} workgroups; phases (median cycles) {ph}; 8->15 (exchange + "
          f"stores) {end}; total {int(np.median(a[15] - a[0]))}; timeline (100 MHz): span {(t1.max() - t0.min()) / 100:.2f} us, "
          f"start skew {(t0.max() - t0.min()) / 100:.2f} us, median workgroup {np.median(t1 - t0) / 100:.2f} us", flush=True)


if __name__ == "__main__":
    main()
