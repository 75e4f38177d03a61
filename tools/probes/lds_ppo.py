"""LDS bank conflicts and waits of the PPO update launches (GPU box): one rocprofv3 --pmc pass over
tools/ppo_train_workload.py (PPO.train() as the product runs it: ackppo_grad1i_kernel per 8192-sample
minibatch, 3 x 160 launches), per-kernel means.

    python3 tools/probes/lds_ppo.py

conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (the share of LDS-array cycles that are
conflict cycles); lds_wait_per_wave = SQ_WAIT_INST_LDS / SQ_WAVES (cycles a wave waited to issue an
LDS instruction).
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
KERNELS = ("ackppo_grad1i_kernel", "ackppo_reduce_norm", "ackppo_adam_blocked_kernel")
COUNTERS = ["SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_LDS", "SQ_WAIT_INST_LDS", "SQ_WAVES",
            "SQ_WAVE_CYCLES"]


def main():
    out = os.path.join(ROOT, "gpurun_out", "lds_ppo")
    os.makedirs(out, exist_ok=True)
    cmd = ["timeout", "-s", "KILL", "180", "rocprofv3", "--pmc", *COUNTERS, "--output-format", "csv", "-d", out, "-o",
           "p", "--", sys.executable, os.path.join(ROOT, "tools", "ppo_train_workload.py")]
    subprocess.run(cmd, check=True, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), stdout=subprocess.DEVNULL)
    per = {}
    for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "")
            name = next((n for n in KERNELS if k.startswith(n)), None)
            if name is None:
                continue
            d = per.setdefault(name, {}).setdefault(int(row.get("Dispatch_Id", 0)), {})
            d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    res = {}
    for k, ds in per.items():
        m = {c: sum(d.get(c, 0.0) for d in ds.values()) / len(ds) for c in COUNTERS}
        m["dispatches"] = len(ds)
        if m["SQ_LDS_IDX_ACTIVE"]:
            m["conflict_frac"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]
        if m["SQ_WAVES"]:
            m["lds_wait_per_wave"] = m["SQ_WAIT_INST_LDS"] / m["SQ_WAVES"]
            m["lds_insts_per_wave"] = m["SQ_INSTS_LDS"] / m["SQ_WAVES"]
            m["wave_cycles_per_wave"] = m["SQ_WAVE_CYCLES"] / m["SQ_WAVES"]
        res[k] = m
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "lds_ppo_latest.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
