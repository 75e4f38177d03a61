#!/bin/bash
# r01f GPU probe: PPO kernel builds (event-timed), grad stamps, PPO GPU tests.
set -o pipefail
V=mujoco_playground_amd/csrc/build/variants
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/ppo_kbench.py $V/libackppo_base.so $V/libackppo_pf.so > gpurun_out/kbench.txt 2>&1 &&
timeout -k 10 60 python -u tools/ppo_kbench.py --stamps $V/libackppo_stamps.so >> gpurun_out/kbench.txt 2>&1 &&
timeout -k 10 200 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_obstacles.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_ppo.txt 2>&1
