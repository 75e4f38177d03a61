"""MFMA utilisation of the PPO kernels (north_star: "MFMA util where used") -> gpurun_out/mfma_latest.json.

Runs tools/ppo_train_workload.py -- PPO.train() as the product runs it (ackppo_train with the weight
image: ackppo_grad1i_kernel per 8192-sample minibatch, then the reduction and Adam launches; the
rollout's policy runs inside ackphys_ppo_rollout_quad_kernel) -- under rocprofv3, one pass per
counter group, kernel-trace only (the round-5 figures were of ackppo_grad1_kernel,
which tools/ppo_kbench.py launches and PPO.train does not):
  pass 1  SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_F32, SQ_INSTS_VALU_MFMA_F32, GRBM_GUI_ACTIVE
  pass 2  the derived MfmaUtil (ROCm's formula: sum MFMA busy cycles / (max GRBM_GUI_ACTIVE x SIMDs))
  pass 3  --kernel-trace --stats (durations)
Per kernel (mean over its dispatches): util = MFMA busy cycles / (GRBM_GUI_ACTIVE / 8 XCDs x 1024
SIMDs); MFMA FLOP/s = MOPS_F32 x 512 / duration, against the 157.3 TFLOP/s f32 MFMA peak.
    python3 tools/profile_mfma.py
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("ackppo_grad1i_kernel", "ackppo_reduce_norm128_kernel", "ackppo_adam_blocked_kernel",
           "ackppo_perm_stats_kernel")
SIMDS, XCDS, F32_MFMA_PEAK_TFLOPS = 1024, 8, 157.3


def rocprof(args, out):
    os.makedirs(out, exist_ok=True)
    cmd = ["timeout", "-s", "KILL", "180", "rocprofv3", *args, "--output-format", "csv", "-d", out, "-o", "p", "--",
           sys.executable, os.path.join(ROOT, "tools", "ppo_train_workload.py")]
    subprocess.run(cmd, check=True, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), stdout=subprocess.DEVNULL)


def counters(out):
    per = {}  # kernel -> dispatch -> counter -> value
    for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "")
            name = next((n for n in KERNELS if k.startswith(n)), None)
            if name is None:
                continue
            d = per.setdefault(name, {}).setdefault(int(row.get("Dispatch_Id", 0)), {})
            c = row["Counter_Name"]
            d[c] = d.get(c, 0.0) + float(row["Counter_Value"])
    return per


def durations(out):
    res = {}
    for f in glob.glob(os.path.join(out, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "")
            name = next((n for n in KERNELS if k.startswith(n)), None)
            if name is not None:
                res.setdefault(name, []).append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    return res


def main():
    base = os.path.join(ROOT, "gpurun_out", "mfma")
    rocprof(["--pmc", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU_MFMA_MOPS_F32", "SQ_INSTS_VALU_MFMA_F32",
             "GRBM_GUI_ACTIVE"], base + "_raw")
    raw = counters(base + "_raw")
    derived = {}
    try:
        rocprof(["--pmc", "MfmaUtil"], base + "_derived")
        derived = counters(base + "_derived")
    except subprocess.CalledProcessError:
        pass
    rocprof(["--kernel-trace", "--stats"], base + "_trace")
    dur = durations(base + "_trace")
    res = {}
    for k in KERNELS:
        ds = list(raw.get(k, {}).values())
        if not ds or k not in dur:
            continue
        mean = lambda c: sum(d.get(c, 0.0) for d in ds) / len(ds)  # noqa: E731
        busy, mops, n, gui = (mean("SQ_VALU_MFMA_BUSY_CYCLES"), mean("SQ_INSTS_VALU_MFMA_MOPS_F32"),
                              mean("SQ_INSTS_VALU_MFMA_F32"), mean("GRBM_GUI_ACTIVE"))
        ns = sorted(dur[k])[len(dur[k]) // 2]
        dv = list(derived.get(k, {}).values())
        res[k] = {"dispatches": len(ds), "median_duration_ns": ns, "mfma_f32_instructions": n,
                  "mfma_busy_cycles": busy, "grbm_gui_active": gui,
                  "mfma_util": busy / (gui / XCDS * SIMDS) if gui else None,
                  "mfma_util_rocprof_derived_pct": (sum(d.get("MfmaUtil", 0.0) for d in dv) / len(dv)) if dv else None,
                  "mfma_tflops": mops * 512 / (ns * 1e-9) / 1e12, "f32_mfma_peak_tflops": F32_MFMA_PEAK_TFLOPS,
                  "workload": "tools/ppo_train_workload.py: 3 PPO.train() calls (ackppo_train, weight image), "
                              "4096 envs x 32 steps, batch 8192 (256 two-tile one-net workgroups per minibatch), "
                              "10 epochs = 160 minibatches per call"}
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "mfma_latest.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
