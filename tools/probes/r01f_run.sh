#!/bin/bash
# r01f GPU probe: PPO kernel builds (event-timed), grad stamps, PPO GPU tests, bench (no CPU leg).
set -o pipefail
V=mujoco_playground_amd/csrc/build/variants
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_ppo.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_ppo.log 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u tools/ppo_kbench.py $V/libackppo_st3.so $V/libackppo_st5.so > gpurun_out/kbench.log 2>&1 &&
timeout -k 10 60 python -u tools/ppo_kbench.py --stamps $V/libackppo_stamps.so >> gpurun_out/kbench.log 2>&1 || exit 1
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err
