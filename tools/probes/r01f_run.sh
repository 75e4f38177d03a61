#!/bin/bash
# r01f GPU probe: bench with the graph-captured step loop (default) and per-call launches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-cpu --no-ppo > gpurun_out/bench_graph.json 2> gpurun_out/bench_graph.err &&
timeout -k 10 300 python -u bench.py --no-cpu --no-ppo --no-graph > gpurun_out/bench_nograph.json 2> gpurun_out/bench_nograph.err
