"""No product kernel may use private (scratch) memory -- checked on the built code objects (CPU only).

Round 4 met two wrong-data cases that both came through private-memory lowering (a
flat load of a private slot returned the neighbouring slot; a select table placed in scratch read
back zeros), and the fixes were source idioms only. This test makes the invariant automatic: it
extracts the gfx950 code object from each library the product loads (libackphys.so,
libackppo.so: the `.hip_fatbin` section, unbundled with clang-offload-bundler), reads every
kernel's AMDGPU metadata (llvm-readelf --notes) and fails if any kernel has a dynamic stack, or an
instruction that can reach private memory in its disassembly: on gfx950 (architected flat scratch,
no private-segment buffer) that is a `scratch_*` instruction or a `flat_*` one (a flat address can
point into the private aperture -- the round-4 bug). A private segment the code never touches is
reported, not failed: the backend reserves an emergency register-scavenging slot in kernels with
heavy SGPR spilling to VGPR lanes (the flat per-step quad kernel in round 6: 68 bytes, no scratch or
flat instruction), and the instruction check is the invariant that matters.

Register spills that stay in registers are reported, not failed: with a zero private segment a
`.vgpr_spill_count` is VGPRs parked in AGPRs (v_accvgpr_write/read) and an `.sgpr_spill_count` is
SGPRs parked in VGPR lanes (v_writelane/readlane) -- neither touches memory. The committed counts
below fail the test if they grow, so a change that pushes a kernel towards memory spills is seen.
"""
from __future__ import annotations

import os
import re
import subprocess

import pytest

from mujoco_playground_amd import _lib

LLVM = "/opt/rocm/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def _tool(name):
    p = os.path.join(LLVM, name)
    if not os.path.exists(p):
        pytest.skip(f"{p} not present")
    return p


def _code_object(lib_path: str, tmp_path) -> str:
    fat = str(tmp_path / (os.path.basename(lib_path) + ".fatbin"))
    co = str(tmp_path / (os.path.basename(lib_path) + ".gfx950.o"))
    subprocess.run([_tool("llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", lib_path], check=True,
                   capture_output=True)
    subprocess.run([_tool("clang-offload-bundler"), "--unbundle", "--type=o", f"--targets={TARGET}",
                    f"--input={fat}", f"--output={co}"], check=True, capture_output=True)
    return co


def kernel_metadata(co: str) -> dict:
    """{kernel name: {field: int}} from the code object's AMDGPU metadata note."""
    import yaml
    notes = subprocess.run([_tool("llvm-readelf"), "--notes", co], check=True, capture_output=True,
                           text=True).stdout
    i = notes.index("---")
    j = notes.index("\n...", i)
    doc = yaml.safe_load(notes[i:j])
    out = {}
    for k in doc["amdhsa.kernels"]:
        out[k[".name"]] = {f.lstrip("."): v for f, v in k.items() if f != ".args"}
    return out


def scratch_instructions(co: str) -> dict:
    """{kernel: number of instructions that can reach private memory: scratch_* and flat_*}."""
    dis = subprocess.run([_tool("llvm-objdump"), "-d", "--mcpu=gfx950", co], check=True, capture_output=True,
                         text=True).stdout
    out, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\w+)>:", line)
        if m:
            cur = m.group(1)
            out.setdefault(cur, 0)
            continue
        if cur and re.match(r"\s+(scratch|flat)_", line):
            out[cur] += 1
    return out


@pytest.fixture(scope="module")
def libs(tmp_path_factory):
    _lib.build()
    tmp = tmp_path_factory.mktemp("codeobj")
    res = {}
    for path in (_lib.LIB_PATH, _lib.PPO_LIB_PATH):
        co = _code_object(path, tmp)
        res[os.path.basename(path)] = (kernel_metadata(co), scratch_instructions(co))
    return res


def test_every_loaded_kernel_found(libs):
    """The kernels the C-ABI launches are all in the code objects read here."""
    md_phys, _ = libs["libackphys.so"]
    md_ppo, _ = libs["libackppo.so"]
    for k in ("ackphys_rollout_quad_kernel", "ackphys_rollout_nc_kernel", "ackphys_rollout_obst8_kernel",
              "ackphys_step_quad_kernel", "ackphys_step_nc_kernel", "ackphys_step_obst_kernel",
              "ackphys_ppo_rollout_quad_kernel", "ackphys_ppo_rollout_obst8_kernel", "ackphys_reset_kernel",
              "ackphys_step_quad_serial_kernel", "ackphys_step_obst_serial_kernel"):
        assert k in md_phys, k
    for k in ("ackppo_grad1_kernel", "ackppo_act_kernel", "ackppo_gae_kernel"):
        assert k in md_ppo, k
    assert len(md_phys) >= 20 and len(md_ppo) >= 10


@pytest.mark.parametrize("lib", ["libackphys.so", "libackppo.so"])
def test_no_private_memory(libs, lib):
    md, scr = libs[lib]
    bad = {k: (v.get("private_segment_fixed_size"), v.get("uses_dynamic_stack"), scr.get(k, 0))
           for k, v in md.items() if v.get("uses_dynamic_stack") or scr.get(k, 0)}
    assert not bad, f"kernels that can reach private memory (private segment B, dynamic stack, scratch/flat instructions): {bad}"
    untouched = {k: v.get("private_segment_fixed_size") for k, v in md.items() if v.get("private_segment_fixed_size", 0)}
    if untouched:
        print(f"{lib}: private segments no instruction touches (scavenging slots): {untouched}")


# register-resident spills of the hot kernels at this commit (VGPR -> AGPR, SGPR -> VGPR lane):
# a bound, not a target -- growth means the allocator is closer to spilling into memory
SPILL_BOUND = {"ackphys_rollout_quad_kernel": (16, 260), "ackphys_rollout_obst8_kernel": (32, 300),
               "ackphys_rollout_nc_kernel": (8, 200), "ackphys_ppo_rollout_quad_kernel": (16, 300),
               "ackphys_ppo_rollout_obst8_kernel": (32, 340), "ackppo_grad1_kernel": (0, 16),
               "ackppo_act_kernel": (0, 16)}


def test_register_spills_bounded(libs):
    md = {**libs["libackphys.so"][0], **libs["libackppo.so"][0]}
    over = {k: (md[k].get("vgpr_spill_count"), md[k].get("sgpr_spill_count"), b)
            for k, b in SPILL_BOUND.items()
            if md[k].get("vgpr_spill_count", 0) > b[0] or md[k].get("sgpr_spill_count", 0) > b[1]}
    assert not over, f"register spills above the committed bound (vgpr, sgpr, bound): {over}"
