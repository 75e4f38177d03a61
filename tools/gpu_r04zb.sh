# round 4: the driver's bench shape (--steps 20 --warmup 5) and the short-window probe, default
# and with spin-wait synchronisation
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r04zb_bench20.json 2> gpurun_out/r04zb_bench20.err || { echo BENCH_FAIL; tail -20 gpurun_out/r04zb_bench20.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04zb_bench20.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'kern_ms', d['roofline']['kernel_ms'])
print('secondary', d['secondary']['value'], d['secondary']['ms_per_step'], d['secondary']['kernel_ms'])
o=d['obstacles']; print('obst', o['value'], o['ms_per_step'], o['kernel_ms'])"
timeout -k 10 200 python -u tools/probes/short_window_probe.py > gpurun_out/r04zb_window.log 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/r04zb_window.log; exit 1; }
timeout -k 10 200 python -u tools/probes/short_window_probe.py spin > gpurun_out/r04zb_window_spin.log 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/r04zb_window_spin.log; exit 1; }
grep -h prelude gpurun_out/r04zb_window.log gpurun_out/r04zb_window_spin.log | grep '"fast": true'
grep -h hipSet gpurun_out/r04zb_window_spin.log
