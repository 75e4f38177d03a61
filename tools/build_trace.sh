#!/bin/bash
# Diagnostic build with per-iteration Newton printf for env 0 -> csrc/build/libackphys_trace.so
set -e
cd "$(dirname "$0")/../mujoco_playground_amd/csrc"
mkdir -p build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fno-fast-math -fno-slp-vectorize -DAK_TRACE \
  -o build/libackphys_trace.so ackphys_step.hip
