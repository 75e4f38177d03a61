"""Per-dispatch durations of the rollout kernels from a rocprofv3 kernel trace.

A rollout launch runs K steps, so the --stats average mixes launches of different K (warm-up,
settle and timed windows). This lists every rollout dispatch in order with its duration, so the
timed launch's duration / K can be checked against bench.py's event-timed kernel_ms.

    python3 tools/dispatch_summary.py <rocprofv3 output dir>
"""
import csv
import glob
import os
import sys


def main(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if "rollout" in name:
                rows.append((int(r["Start_Timestamp"]), name.split("(")[0], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows.sort()
    print("kernel,duration_ns")
    for _, name, dur in rows:
        print(f"{name},{dur}")


if __name__ == "__main__":
    main(sys.argv[1])
