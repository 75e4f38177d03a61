"""Compile the reference MJCF into the in-tree model assets (offline, host-only).

    python -m mujoco_playground_amd.model.build [--reference /root/reference]

Writes
  mujoco_playground_amd/model/assets/ackermann_robot_v2.apm   (blob for ackphys_create)
  mujoco_playground_amd/csrc/ackphys_model_gen.h              (constexpr kernel constants)
  mujoco_playground_amd/model/assets/ackermann_obstacles.apm  (obstacle scene blob)
  mujoco_playground_amd/csrc/ackphys_scene_gen.h              (its static-world constants)
Both are committed: the GPU box has no /root/reference, so it only consumes them.
"""
from __future__ import annotations

import argparse
import os

from . import blob as blobmod
from .codegen import generate, generate_scene
from .compiler import compile_mjcf, compile_scene, default_model_path, obstacle_scene_path

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BLOB_PATH = os.path.join(PKG, "model", "assets", "ackermann_robot_v2.apm")
HEADER_PATH = os.path.join(PKG, "csrc", "ackphys_model_gen.h")
SCENE_BLOB_PATH = os.path.join(PKG, "model", "assets", "ackermann_obstacles.apm")
SCENE_HEADER_PATH = os.path.join(PKG, "csrc", "ackphys_scene_gen.h")


def build(reference_root: str = "/root/reference", check_only: bool = False) -> bool:
    """Recompile; returns True if the committed assets were already up to date."""
    m = compile_mjcf(default_model_path(reference_root))
    b = blobmod.pack(m)
    hdr = generate(m, blobmod.fnv1a64(b))
    ms = compile_scene(obstacle_scene_path(reference_root), default_model_path(reference_root))
    bs = blobmod.pack(ms)
    hs = generate_scene(ms, blobmod.fnv1a64(bs), m)
    outs = [(BLOB_PATH, b), (HEADER_PATH, hdr.encode()), (SCENE_BLOB_PATH, bs), (SCENE_HEADER_PATH, hs.encode())]
    same = all(os.path.exists(p) and open(p, "rb").read() == data for p, data in outs)
    if not same and not check_only:
        for p, data in outs:
            os.makedirs(os.path.dirname(p), exist_ok=True)
            with open(p, "wb") as f:
                f.write(data)
    return same


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    ok = build(a.reference, a.check)
    print("up to date" if ok else ("STALE" if a.check else "written"))
