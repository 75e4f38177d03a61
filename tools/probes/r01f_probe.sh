#!/bin/bash
# r01f GPU probe: PPO kernel variants (policy-tile wave count, reduce fix), grad phase stamps,
# product GPU tests, quad Newton start-rule variants (bench + full GPU suite on the probe build).
set -o pipefail
D=mujoco_playground_amd/csrc/build
V=$D/variants
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/ppo_kbench.py $V/libackppo_head.so $V/libackppo_w4.so $V/libackppo_w8.so \
  $V/libackppo_w16.so > gpurun_out/kbench.log 2>&1 &&
timeout -k 10 60 python -u tools/ppo_kbench.py --stamps $V/libackppo_stamps.so >> gpurun_out/kbench.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_base.log 2>&1 &&
bash tools/variant_sweep.sh qbase qsmooth > gpurun_out/sweep.log 2>&1 || exit 1
cp $D/libackphys.so /tmp/keep.so && cp $V/qsmooth.so $D/libackphys.so
timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_qsmooth.log 2>&1
rc=$?
cp /tmp/keep.so $D/libackphys.so
exit $rc
