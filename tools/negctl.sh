#!/bin/bash
# Negative control (GPU box): run one parity test against a deliberately wrong prebuilt variant
# (csrc/build/variants/<name>.so); the test is expected to FAIL. The product library is restored.
#   bash tools/negctl.sh NAME 'pytest node id'
D=mujoco_playground_amd/csrc/build
cp $D/libackphys.so /tmp/libackphys.orig.so && cp $D/variants/$1.so $D/libackphys.so
timeout -k 10 200 python -u -m pytest "$2" -x -q --timeout 120 --timeout-method thread > gpurun_out/negctl_$1.log 2>&1
rc=$?
cp /tmp/libackphys.orig.so $D/libackphys.so
tail -3 gpurun_out/negctl_$1.log
if [ $rc -eq 0 ]; then echo "NEGCTL $1: test PASSED against the wrong variant (not discriminating)"; else echo "NEGCTL $1: test failed as expected (rc $rc)"; fi
