#!/bin/bash
# contacts-off step kernel under the lane mappings (64 / 16 envs per wave), GPU box, repo root
set -o pipefail
mkdir -p gpurun_out
for v in auto lane16 auto lane16; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-ppo --no-secondary --no-obstacles --variant $v > gpurun_out/lv.json 2> gpurun_out/lv.err || { tail -5 gpurun_out/lv.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/lv.json')); print('$v', round(d['value']/1e6,1), 'M/s', round(d['roofline']['kernel_ms']*1e3,2), 'us kernel')"
done
