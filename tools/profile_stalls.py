"""SQ stall breakdown (one rocprofv3 --pmc pass, 8 SQ counters) of the step kernels.

    python3 tools/profile_stalls.py [tag]      (GPU box, repo root) -> gpurun_out/stalls_<tag>.json
SQ_WAVE_CYCLES = SQ_WAIT_ANY (parked on s_waitcnt) + SQ_WAIT_INST_ANY (issue stall: dependency,
pipe, instruction fetch) + SQ_ACTIVE_INST_ANY (issuing); all in quad-cycles (MI355X_MICROARCH.md).
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SQ = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
      "SQ_INSTS_VALU", "SQ_INSTS_SALU"]
RUNS = [("lane_off", "ackphys_rollout_nc_kernel", ["--contacts", "0", "--variant", "lane"]),
        ("quad_on", "ackphys_rollout_quad_kernel", ["--contacts", "1", "--variant", "quad"])]
if len(sys.argv) > 2:  # e.g. quad_on only
    RUNS = [r for r in RUNS if r[0] in sys.argv[2:]]


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "run"
    res = {}
    for name, kern, extra in RUNS:
        out = os.path.join(ROOT, "gpurun_out", f"stalls_{tag}_{name}")
        os.makedirs(out, exist_ok=True)
        cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc", *SQ, "--output-format", "csv", "-d", out, "-o",
               "pmc", "--", sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu", "--no-secondary", "--no-ppo",
               "--no-obstacles", "--no-per-step", "--no-buffer-leg", "--steps", "200", "--warmup", "5", *extra]
        subprocess.run(cmd, check=True, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), stdout=subprocess.DEVNULL)
        vals = {c: [] for c in SQ}
        for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if row.get("Kernel_Name", "").startswith(kern) and row.get("Counter_Name") in vals:
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
        med = {c: (sorted(v)[len(v) // 2] if v else None) for c, v in vals.items()}
        w = med["SQ_WAVES"] or 1.0
        per = {c: med[c] / w for c in SQ if med[c] is not None}
        res[name] = {"kernel": kern, "median_per_launch": med, "per_wave": per,
                     "per_wave_cycles": {c: 4 * per[c] for c in ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                                  "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"] if c in per}}
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", f"stalls_{tag}.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
