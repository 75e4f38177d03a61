# round 4 close: every GPU test, smoke and the bench line at HEAD
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r04zg_pytest.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/r04zg_pytest.log; exit 1; }
tail -2 gpurun_out/r04zg_pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04zg_smoke.log 2>&1 && tail -1 gpurun_out/r04zg_smoke.log || { echo SMOKE_FAIL; tail -20 gpurun_out/r04zg_smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/r04zg_bench.json 2> gpurun_out/r04zg_bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/r04zg_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04zg_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'kern_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])
print('secondary', d['secondary']['value'])
p=d['ppo']; print('ppo', p['value'], p['update_us_per_minibatch'], p['rollout_env_steps_per_s'])
o=d['obstacles']; print('obst', o['value'], 'ppo rollout', o['ppo']['rollout_env_steps_per_s'], o['ppo']['value'])
print('cpu', d['cpu_baseline'])"
