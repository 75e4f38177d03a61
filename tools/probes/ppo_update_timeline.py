"""Where a PPO update's time goes: one rollout (4096 envs x 32 steps), then PPO.train() timed with
and without the all-epochs shuffle buffers and the weight image (event-timed, 3 calls each). Under
`rocprofv3 --kernel-trace` (tools/gpu_steps.sh prof) the kernel trace then gives each kernel's duration
and the idle gaps between consecutive kernels (tools/probes/ppo_update_timeline.py --trace DIR).

    python tools/probes/ppo_update_timeline.py              (timing)
    python tools/probes/ppo_update_timeline.py --only 1,0    (one configuration: epoch_buffers, weight_image)
    python tools/probes/ppo_update_timeline.py --trace DIR  (summarise a rocprofv3 kernel trace)
"""
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def timing(configs=((True, False), (True, True), (False, False), (True, False), (True, True), (False, False))):
    import torch
    from mujoco_playground_amd.rl import AckermannVecEnv
    from mujoco_playground_amd.rl.ppo import PPO
    dev = torch.device("cuda:0")
    venv = AckermannVecEnv(4096, device=dev, seed=0, contacts=True)
    model = PPO("MlpPolicy", venv, n_steps=32, batch_size=8192, n_epochs=10, seed=0)
    model.collect_rollouts()
    nmb = 32 * 4096 // 8192 * 10
    for epochs, img in configs:
        model.set_epoch_buffers(epochs)
        model.set_weight_image(img)
        model.train()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(3):
            model.train()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 3
        print(f"epoch_buffers={epochs} weight_image={img}: train() {ms:.3f} ms = {ms * 1e3 / nmb:.2f} us per minibatch",
              flush=True)


def trace(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    rows.sort()
    # the last train() calls only: from the last "ackppo_perm" run of 10 epochs
    stats, gaps = {}, {}
    for i, (s, e, k) in enumerate(rows):
        stats.setdefault(k, []).append(e - s)
        if i:
            prev = rows[i - 1][2]
            gaps.setdefault(f"{prev} -> {k}", []).append(s - rows[i - 1][1])
    print("kernel: count, mean duration us")
    for k, v in sorted(stats.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {k}: {len(v)}, {sum(v) / len(v) / 1e3:.2f}")
    print("gap (previous end -> next start): count, median us")
    for k, v in sorted(gaps.items(), key=lambda kv: -len(kv[1]))[:12]:
        v = sorted(v)
        print(f"  {k}: {len(v)}, {v[len(v) // 2] / 1e3:.2f}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--trace":
        trace(sys.argv[2])
    elif len(sys.argv) > 2 and sys.argv[1] == "--only":  # one configuration (kernel traces): EPOCHS,IMAGE
        timing((tuple(bool(int(v)) for v in sys.argv[2].split(",")),))
    else:
        timing()
