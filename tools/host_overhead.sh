#!/bin/bash
# per-call vs graph-replayed timed loop, long and driver-short runs (GPU box, repo root)
set -o pipefail
mkdir -p gpurun_out
for args in "--steps 1000 --warmup 50" "--steps 1000 --warmup 50 --graph" "--steps 20 --warmup 5" "--steps 20 --warmup 5 --graph"; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-ppo --no-secondary --no-obstacles $args > gpurun_out/ho.json 2> gpurun_out/ho.err || { tail -5 gpurun_out/ho.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ho.json')); print('$args', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step', round(d['roofline']['kernel_ms']*1e3,2), 'us kernel')"
done
