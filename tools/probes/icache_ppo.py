"""Instruction-cache misses of the open-loop quad rollout kernel against the fused PPO rollout kernel
(GPU box, repo root): in the PPO kernel the observation wave runs the policy while the dynamics wave
runs Newton, so both waves' hot code competes for the instruction cache.

    python3 tools/probes/icache_ppo.py            (profiles itself with rocprofv3 --pmc, one pass)
    python3 tools/probes/icache_ppo.py --work     (the workload alone)
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
COUNTERS = ["SQC_ICACHE_REQ", "SQC_ICACHE_HITS", "SQC_ICACHE_MISSES", "SQC_ICACHE_MISSES_DUPLICATE", "SQ_WAVES",
            "SQ_BUSY_CYCLES"]
KERNELS = ["ackphys_rollout_quad_kernel", "ackphys_ppo_rollout_quad_kernel"]


def work():
    sys.path.insert(0, ROOT)
    import torch
    from mujoco_playground_amd.rl import AckermannVecEnv
    from mujoco_playground_amd.rl.ppo import PPO
    from mujoco_playground_amd.sim import BatchedAckermannSim
    dev = torch.device("cuda:0")
    sim = BatchedAckermannSim(4096, dev, seed=0, contacts=True)
    sim.reset()
    acts = sim.random_actions(264, seed=0)
    sim.rollout(acts[:200], want_info=False, per_step_outputs=False)
    for k in range(2):
        sim.rollout(acts[200 + 32 * k:232 + 32 * k], want_info=False, per_step_outputs=False)
    venv = AckermannVecEnv(4096, device=dev, seed=0, contacts=True)
    model = PPO("MlpPolicy", venv, n_steps=32, batch_size=8192, n_epochs=10, seed=0)
    for _ in range(3):
        model.collect_rollouts()
    torch.cuda.synchronize()


def main():
    if "--work" in sys.argv:
        work()
        return
    out = os.path.join(ROOT, "gpurun_out", "icache_ppo")
    os.makedirs(out, exist_ok=True)
    cmd = ["timeout", "-k", "10", "180", "rocprofv3", "--pmc", *COUNTERS, "--output-format", "csv", "-d", out, "-o",
           "pmc", "--", sys.executable, os.path.abspath(__file__), "--work"]
    subprocess.run(cmd, check=True, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), stdout=subprocess.DEVNULL)
    res = {}
    for kern in KERNELS:
        vals = {c: [] for c in COUNTERS}
        for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if row.get("Kernel_Name", "").startswith(kern) and row.get("Counter_Name") in vals:
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
        res[kern] = {c: (sorted(v)[len(v) // 2] if v else None) for c, v in vals.items()}
        r = res[kern]
        if r["SQC_ICACHE_REQ"]:
            r["miss_rate"] = r["SQC_ICACHE_MISSES"] / r["SQC_ICACHE_REQ"]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
