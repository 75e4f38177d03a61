"""Static instruction mix of the step kernels (host tool, no GPU).

    python3 tools/isa_mix.py [extra hipcc flags...]
Compiles csrc/ackphys_step.hip to gfx950 assembly and counts, per kernel, scratch (spill) loads and
stores, s_waitcnt, vector-memory, scalar-memory, LDS, AGPR moves, VALU and SALU instructions.
"""
import os
import subprocess
import sys
import tempfile
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "mujoco_playground_amd", "csrc", "ackphys_step.hip")
KERNELS = ["ackphys_step_kernel", "ackphys_step_nc_kernel", "ackphys_step_serial_kernel", "ackphys_step_quad_serial_kernel", "ackphys_step_quad_kernel", "ackphys_step_obst_kernel"]


def category(op: str) -> str:
    for pre, name in (("scratch_load", "scratch_load"), ("scratch_store", "scratch_store"),
                      ("s_waitcnt", "s_waitcnt"), ("global_load", "vmem_load"), ("buffer_load", "vmem_load"),
                      ("global_store", "vmem_store"), ("buffer_store", "vmem_store"), ("s_load", "s_load"),
                      ("s_buffer_load", "s_load"), ("ds_", "lds"), ("v_accvgpr", "agpr_mov"),
                      ("v_readlane", "lane_rw"), ("v_writelane", "lane_rw"), ("v_", "valu"), ("s_", "salu")):
        if op.startswith(pre):
            return name
    return "other"


def main():
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-fast-math",
                        "--cuda-device-only", "-S", *sys.argv[1:], SRC, "-o", out], check=True,
                       stderr=subprocess.DEVNULL)
        s = open(out).read()
    for k in KERNELS:
        i = s.find("\n" + k + ":")
        if i < 0:
            continue
        j = s.index(".Lfunc_end", i)
        ops = [ln.split()[0] for ln in s[i:j].split("\n") if ln.startswith("\t") and ln.strip()
               and not ln.strip().startswith((".", ";"))]
        c = Counter(category(o) for o in ops)
        print(f"{k}: {len(ops)} static instructions", dict(sorted(c.items(), key=lambda t: -t[1])))


if __name__ == "__main__":
    main()
