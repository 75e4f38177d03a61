#!/bin/bash
# r01f GPU probe: step-kernel stamps (lane + quad), PPO kernel timing + grad stamps.
set -o pipefail
V=mujoco_playground_amd/csrc/build/variants
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/stamps.py > gpurun_out/r01f_stamps_lane.txt 2>&1 &&
timeout -k 10 120 python -u tools/stamps.py quad > gpurun_out/r01f_stamps_quad.txt 2>&1 &&
timeout -k 10 120 python -u tools/ppo_kbench.py mujoco_playground_amd/csrc/build/libackppo.so > gpurun_out/r01f_ppo_kbench.txt 2>&1 &&
timeout -k 10 60 python -u tools/ppo_kbench.py --stamps $V/libackppo_stamps.so >> gpurun_out/r01f_ppo_kbench.txt 2>&1
