"""Is the data-parallel update host-bound? (GPU box) For the single-rank sequence and the one-rank
data-parallel sequences (libackppo's communicator "rccl", torch's "torch"), on bench.py's configs[3]
shape: the host time of the ackppo_train call alone (enqueue of every launch and collective of a
train(), no wait) against the GPU time of the same call (events), per minibatch.

    python3 tools/probes/dp_host_probe.py
"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist

    from mujoco_playground_amd import _lib
    from mujoco_playground_amd.rl import AckermannVecEnv
    from mujoco_playground_amd.rl.ppo import PPO
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1)  # as shard.init: lazy comm
    venv = AckermannVecEnv(4096, device=dev, seed=0, contacts=True)
    model = PPO("MlpPolicy", venv, n_steps=32, batch_size=8192, n_epochs=10, seed=0, ent_coef=0.0)
    model.collect_rollouts()
    nmb = 16 * 10
    stream = torch.cuda.current_stream(dev)
    for kind in (None, "rccl", "torch", None):
        model.set_collective(kind)
        model.train()
        torch.cuda.synchronize(dev)
        d = model._desc
        host, gpu = [], []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(dev)
            e0.record(stream)
            t0 = time.perf_counter()
            _lib.ppo_check(model.L.ackppo_train(C.byref(d), model._stream()), "ackppo_train")
            t1 = time.perf_counter()
            e1.record(stream)
            torch.cuda.synchronize(dev)
            host.append((t1 - t0) * 1e6 / nmb)
            gpu.append(e0.elapsed_time(e1) * 1e3 / nmb)
        host.sort()
        gpu.sort()
        print(f"collective {kind}: host enqueue {host[2]:.2f} us per minibatch, GPU {gpu[2]:.2f} us per minibatch "
              f"(min {gpu[0]:.2f})", flush=True)
    model.set_collective(None)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
