#!/bin/bash
# Timing ablations of the step kernels (host side): copy csrc/ + include/ to a scratch tree, apply one
# sed edit per variant, build csrc/build/variants/<name>.so. The ablated builds compute WRONG physics
# on purpose -- they only price a piece of the critical path; bench them with tools/variant_sweep.sh.
#   bash tools/ablate.sh NAME 'sed-expr' [NAME 'sed-expr' ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/mujoco_playground_amd/csrc/build/variants
mkdir -p "$OUT"
pids=()
while [ $# -ge 2 ]; do
  name=$1; expr=$2; shift 2
  T=$(mktemp -d /tmp/abl_XXXX)
  mkdir -p "$T/mujoco_playground_amd"
  cp -r "$ROOT/mujoco_playground_amd/csrc" "$T/mujoco_playground_amd/csrc"
  rm -rf "$T/mujoco_playground_amd/csrc/build"
  cp -r "$ROOT/include" "$T/include"
  (cd "$T/mujoco_playground_amd/csrc" && sed -i -E "$expr" ackphys_step.hip ackphys_quad.inc &&
   /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fno-fast-math -fno-slp-vectorize -Wno-unused-result \
     -o "$OUT/$name.so" ackphys_step.hip && rm -rf "$T") &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
