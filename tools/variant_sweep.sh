#!/bin/bash
# Bench several prebuilt step-kernel builds back to back on one box (GPU box, repo root).
#   bash tools/variant_sweep.sh A B C ...   (csrc/build/variants/<name>.so, built on the CPU side)
# Each variant is copied over csrc/build/libackphys.so, benched (contacts off lane, contacts on
# quad, obstacles), and the product library restored at the end.
set -o pipefail
D=mujoco_playground_amd/csrc/build
mkdir -p gpurun_out
cp $D/libackphys.so /tmp/libackphys.orig.so
rc=0
for v in "$@"; do
  cp $D/variants/$v.so $D/libackphys.so
  timeout -k 10 240 python -u bench.py --no-cpu --no-ppo --steps 1000 > gpurun_out/sweep_$v.json 2> gpurun_out/sweep_$v.err \
    || { echo "variant $v failed"; tail -5 gpurun_out/sweep_$v.err; rc=1; break; }
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.load(open(f'gpurun_out/sweep_{v}.json'))
print(v, 'lane-off', round(d['value'] / 1e6, 2), 'M/s', round(d['roofline']['kernel_ms'] * 1e3, 2), 'us;',
      'quad-on', round(d['secondary']['value'] / 1e6, 2), round(d['secondary']['kernel_ms'] * 1e3, 2), 'us;',
      'obst', round(d['obstacles']['value'] / 1e6, 2), round(d['obstacles']['kernel_ms'] * 1e3, 2), 'us')
PY
done
cp /tmp/libackphys.orig.so $D/libackphys.so
exit $rc
