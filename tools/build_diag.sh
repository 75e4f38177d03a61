#!/bin/bash
# Diagnostic (stamped) build of the step kernel -> diag_libs/libackphys_stamps.so (never loaded by the product)
#   bash tools/build_diag.sh [extra hipcc flags...]   (DIAG_OUT=name.so picks another output under diag_libs/)
set -e
cd "$(dirname "$0")/../mujoco_playground_amd/csrc"
mkdir -p ../../diag_libs
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fno-fast-math -fno-slp-vectorize -DAK_STAMPS "$@" \
  -o ../../diag_libs/${DIAG_OUT:-libackphys_stamps.so} ackphys_step.hip
