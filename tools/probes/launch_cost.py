"""Host cost of one ackphys_rollout launch call (GPU box): N back-to-back calls of the bench's
pre-bound launcher (K = 20 steps each, no synchronisation between them), the host time per call,
against a torch elementwise launch on the same stream.

    python3 tools/probes/launch_cost.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from mujoco_playground_amd.sim import BatchedAckermannSim
    dev = torch.device("cuda:0")
    sim = BatchedAckermannSim(4096, dev, seed=0, contacts=False)
    sim.reset()
    acts = sim.random_actions(20, seed=0)
    launch = sim.rollout_launcher(acts)
    x = torch.zeros(16, device=dev)
    for _ in range(50):
        launch()
    torch.cuda.synchronize()
    for rep in range(3):
        n = 200
        t0 = time.perf_counter()
        for _ in range(n):
            launch()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        for _ in range(n):
            x.add_(1.0)
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        # one launch after an idle GPU, as in the bench window
        time.sleep(0.01)
        t4 = time.perf_counter()
        launch()
        t5 = time.perf_counter()
        torch.cuda.synchronize()
        t6 = time.perf_counter()
        print(f"rollout launch {1e6 * (t1 - t0) / n:.2f} us/call (queued), torch add_ {1e6 * (t3 - t2) / n:.2f} us/call; "
              f"single launch after idle {1e6 * (t5 - t4):.2f} us, its sync {1e6 * (t6 - t5):.2f} us", flush=True)


if __name__ == "__main__":
    main()
