#!/bin/bash
# quick GPU check: parity tests + short benches of the three step kernels (GPU box, repo root)
# usage: bash tools/quick_gpu.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-q}; K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${KARG[@]}" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_$TAG.log | head -20; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu --no-ppo --steps 500 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 1; }
python - <<PY
import json; d=json.load(open('gpurun_out/bench_$TAG.json'))
print('lane-off', round(d['value']/1e6,2), 'M/s', round(d['roofline']['kernel_ms']*1e3,2), 'us;',
      'quad-on', round(d['secondary']['value']/1e6,2), round(d['secondary']['kernel_ms']*1e3,2), 'us;',
      'obst', round(d['obstacles']['value']/1e6,2), round(d['obstacles']['kernel_ms']*1e3,2), 'us;', 'parity', d['parity'])
PY
