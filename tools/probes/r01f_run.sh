#!/bin/bash
# r01f GPU probe: quad step-kernel phase stamps.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/stamps.py quad > gpurun_out/r01f_stamps_quad2.txt 2>&1
