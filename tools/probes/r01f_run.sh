#!/bin/bash
# r01f GPU probe: PPO GPU tests, then the bench without the CPU leg.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_ppo.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_ppo.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/bench_nocpu.json 2> gpurun_out/bench_nocpu.err
