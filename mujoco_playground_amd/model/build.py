"""Compile the reference MJCF into the in-tree model assets (offline, host-only).

    python -m mujoco_playground_amd.model.build [--reference /root/reference]

Writes
  mujoco_playground_amd/model/assets/ackermann_robot_v2.apm   (blob for ackphys_create)
  mujoco_playground_amd/csrc/ackphys_model_gen.h              (constexpr kernel constants)
Both are committed: the GPU box has no /root/reference, so it only consumes them.
"""
from __future__ import annotations

import argparse
import os

from . import blob as blobmod
from .codegen import generate
from .compiler import compile_mjcf, default_model_path

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BLOB_PATH = os.path.join(PKG, "model", "assets", "ackermann_robot_v2.apm")
HEADER_PATH = os.path.join(PKG, "csrc", "ackphys_model_gen.h")


def build(reference_root: str = "/root/reference", check_only: bool = False) -> bool:
    """Recompile; returns True if the committed assets were already up to date."""
    m = compile_mjcf(default_model_path(reference_root))
    b = blobmod.pack(m)
    hdr = generate(m, blobmod.fnv1a64(b))
    same = (os.path.exists(BLOB_PATH) and open(BLOB_PATH, "rb").read() == b
            and os.path.exists(HEADER_PATH) and open(HEADER_PATH).read() == hdr)
    if not same and not check_only:
        os.makedirs(os.path.dirname(BLOB_PATH), exist_ok=True)
        with open(BLOB_PATH, "wb") as f:
            f.write(b)
        with open(HEADER_PATH, "w") as f:
            f.write(hdr)
    return same


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    ok = build(a.reference, a.check)
    print("up to date" if ok else ("STALE" if a.check else "written"))
