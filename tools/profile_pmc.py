"""rocprofv3 PMC passes for the step kernels -> gpurun_out/pmc_latest.json (run on the GPU box).

For each workload (contacts off -> ackphys_rollout_nc_kernel, contacts on -> ackphys_rollout_quad_kernel,
the obstacle scene -> ackphys_rollout_obst8_kernel: the kernels bench.py's AUTO mapping runs; one
launch = the K timed steps) and each K in KS, three
separate passes, kernel-trace only, no sys/runtime trace:
  FETCH_SIZE, WRITE_SIZE (HBM bytes; they do not fit one TCC pass on gfx950),
  SQ_INSTS_VALU + SQ_INSTS_SALU + SQ_WAVES (instruction mix, one SQ pass).
Correction per MI355X_MICROARCH.md §HBM: FETCH_SIZE tallies 128-B requests at 64 B for
lane-contiguous streaming reads -> doubled; WRITE_SIZE taken as reported. The counters of the
timed launch (the kernel's last dispatch) are divided by its K steps: bytes and instructions per
step. Entries are keyed "<kernel>@K<k>"; bench.py reports the entry whose K equals its --steps (or
the nearest K, saying so), since a launch's first-step loads and last-step stores are spread over
its K steps.
    python3 tools/profile_pmc.py [K,K,...] [--buffers]   (default 20,1000: the driver's and bench's defaults)
--buffers: the flat-scene launches with per-step output slices (bench.py --buffers: a [K][79][N]
rollout buffer), keyed "<kernel>@K<k>+buf" with per_step_outputs true.
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = [a for a in sys.argv[1:] if not a.startswith("--")]
BUFFERS = "--buffers" in sys.argv[1:]
# (contacts, scene) -> kernel
KERNELS = {(0, "flat"): "ackphys_rollout_nc_kernel", (1, "flat"): "ackphys_rollout_quad_kernel"}
if not BUFFERS:
    KERNELS[(1, "obstacles")] = "ackphys_rollout_obst8_kernel"
KS = [int(k) for k in (ARGS[0] if ARGS else "20,1000").split(",")]


def run_pass(counters, out, contacts, scene, k):
    os.makedirs(out, exist_ok=True)
    cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d", out, "-o",
           "pmc", "--", sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu", "--no-secondary", "--no-ppo",
           "--no-obstacles", "--no-per-step", "--no-buffer-leg", "--steps", str(k), "--warmup", "5", "--contacts",
           str(contacts), "--scene", scene] + (["--buffers"] if BUFFERS else [])
    env = dict(os.environ, TMPDIR="/tmp")
    subprocess.run(cmd, check=True, cwd="/tmp", env=env, stdout=subprocess.DEVNULL)
    vals = {c: {} for c in counters}  # counter -> dispatch id -> value (summed over the rows of a dispatch)
    for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Kernel_Name", "").startswith(KERNELS[(contacts, scene)]) and row.get("Counter_Name") in vals:
                d = int(row.get("Dispatch_Id", 0))
                v = vals[row["Counter_Name"]]
                v[d] = v.get(d, 0.0) + float(row["Counter_Value"])
    return {c: (v[max(v)] if v else None) for c, v in vals.items()}  # the timed launch = the last dispatch


def main():
    res = {}
    for k in KS:
        for (contacts, scene), kern in KERNELS.items():
            out = os.path.join(ROOT, "gpurun_out", f"pmc_c{contacts}_{scene}_k{k}{'_buf' if BUFFERS else ''}")
            f = run_pass(["FETCH_SIZE"], out + "_fetch", contacts, scene, k)["FETCH_SIZE"]
            w = run_pass(["WRITE_SIZE"], out + "_write", contacts, scene, k)["WRITE_SIZE"]
            sq = run_pass(["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVES"], out + "_sq", contacts, scene, k)
            ok = f is not None and w is not None
            key = f"{kern}@K{k}" + ("+buf" if BUFFERS else "")
            res[key] = {
                "kernel": kern, "scene": scene, "contacts": bool(contacts), "launch_steps": k, "per_step_outputs": BUFFERS, "FETCH_SIZE_kB": f, "WRITE_SIZE_kB": w,
                "hbm_bytes_per_launch": (2 * f * 1024 + w * 1024) if ok else None,
                "hbm_bytes_per_step": (2 * f * 1024 + w * 1024) / k if ok else None,
                "correction": "FETCH_SIZE x2 (gfx950 tallies 128-B read requests at 64 B), WRITE_SIZE as reported",
                "algorithmic_bytes_per_step": 690 * 4096,
                "SQ_INSTS_VALU": sq["SQ_INSTS_VALU"], "SQ_INSTS_SALU": sq["SQ_INSTS_SALU"], "SQ_WAVES": sq["SQ_WAVES"],
                "valu_insts_per_wave_step": (sq["SQ_INSTS_VALU"] / sq["SQ_WAVES"] / k) if sq["SQ_WAVES"] else None,
            }
            print(json.dumps({key: res[key]}), flush=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "pmc_latest" + ("_buf" if BUFFERS else "") + ".json"), "w"),
              indent=1)


if __name__ == "__main__":
    main()
