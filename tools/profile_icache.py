"""rocprofv3 PMC pass: instruction-cache behaviour of the step kernels (GPU box, repo root).

    python3 tools/profile_icache.py
Counters SQC_ICACHE_REQ / HITS / MISSES / MISSES_DUPLICATE, SQ_WAVES, SQ_WAVE_CYCLES, SQ_BUSY_CYCLES
(kernel trace only, one pass per workload), median dispatch of the bench's step kernel.
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {0: "ackphys_step_nc_kernel", 1: "ackphys_step_quad_kernel"}
COUNTERS = ["SQC_ICACHE_REQ", "SQC_ICACHE_HITS", "SQC_ICACHE_MISSES", "SQC_ICACHE_MISSES_DUPLICATE", "SQ_WAVES",
            "SQ_WAVE_CYCLES"]


def main():
    res = {}
    for contacts, kern in KERNELS.items():
        out = os.path.join(ROOT, "gpurun_out", f"icache_c{contacts}")
        os.makedirs(out, exist_ok=True)
        cmd = ["timeout", "-k", "10", "120", "rocprofv3", "--pmc", *COUNTERS, "--output-format", "csv", "-d", out,
               "-o", "pmc", "--", sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu", "--no-secondary",
               "--no-ppo", "--no-obstacles", "--steps", "60", "--warmup", "5", "--contacts", str(contacts)]
        subprocess.run(cmd, check=True, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), stdout=subprocess.DEVNULL)
        vals = {c: [] for c in COUNTERS}
        for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if row.get("Kernel_Name", "").startswith(kern) and row.get("Counter_Name") in vals:
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
        res[kern] = {c: (sorted(v)[len(v) // 2] if v else None) for c, v in vals.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
