"""rocprofv3 PMC passes for the step kernel -> profiles/pmc_latest.json (run on the GPU box).

Separate passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950), kernel-trace
only, no sys/runtime trace. Correction per MI355X_MICROARCH.md §HBM: FETCH_SIZE tallies 128-B
requests at 64 B for lane-contiguous streaming reads -> doubled; WRITE_SIZE taken as reported
(dword-per-lane stores: uncalibrated, noted).
    python3 tools/profile_pmc.py [--contacts 0]
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_pass(counter, out, contacts):
    os.makedirs(out, exist_ok=True)
    cmd = ["timeout", "-k", "10", "300", "rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", out, "-o",
           "pmc", "--", sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu", "--no-secondary", "--steps", "60",
           "--warmup", "5", "--contacts", str(contacts)]
    env = dict(os.environ, TMPDIR="/tmp")
    subprocess.run(cmd, check=True, cwd="/tmp", env=env, stdout=subprocess.DEVNULL)
    vals = []
    for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Kernel_Name", "").startswith("ackphys_step_kernel") and row.get("Counter_Name") == counter:
                vals.append(float(row["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--contacts", type=int, default=0)
    a = ap.parse_args()
    out = os.path.join(ROOT, "gpurun_out", "pmc")
    fetch = run_pass("FETCH_SIZE", out + "_fetch", a.contacts)
    write = run_pass("WRITE_SIZE", out + "_write", a.contacts)
    # steady state: drop the warmup dispatches
    f = sorted(fetch)[len(fetch) // 2] if fetch else None
    w = sorted(write)[len(write) // 2] if write else None
    res = {"ackphys_step_kernel": {
        "contacts": bool(a.contacts), "dispatches": [len(fetch), len(write)],
        "FETCH_SIZE_kB_median": f, "WRITE_SIZE_kB_median": w,
        "hbm_bytes_per_launch": (2 * f * 1024 + w * 1024) if (f is not None and w is not None) else None,
        "correction": "FETCH_SIZE x2 (gfx950 tallies 128-B read requests at 64 B), WRITE_SIZE as reported",
        "algorithmic_bytes_per_launch": 690 * 4096}}
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "pmc_latest.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
