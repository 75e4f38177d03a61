# round 4: the PPO observation wave on octets of lanes (observe_oct): PPO rollout parity (both scenes,
# variants), stamps, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ppo_rollout.py tests/test_gpu_ppo.py tests/test_gpu_variant.py -q --timeout 240 --timeout-method thread > gpurun_out/r04u_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r04u_tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" gpurun_out/r04u_tests.log | head -20; exit $rc; fi
timeout -k 10 200 python -u tools/probes/ppo_rollout_stamps.py flat > gpurun_out/r04u_ppo_stamps.log 2>&1 && timeout -k 10 200 python -u tools/probes/ppo_rollout_stamps.py obstacles >> gpurun_out/r04u_ppo_stamps.log 2>&1 || { echo PPOSTAMPS_FAIL; tail -20 gpurun_out/r04u_ppo_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04u_ppo_stamps.log
timeout -k 10 400 python -u bench.py > gpurun_out/r04u_bench.json 2> gpurun_out/r04u_bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/r04u_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04u_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'kern_ms', d['roofline']['kernel_ms'])
print('secondary', d['secondary']['value'], d['secondary']['kernel_ms'])
p=d['ppo']; print('ppo', p['value'], p['update_us_per_minibatch'], p['rollout_env_steps_per_s'])
o=d['obstacles']; print('obst', o['value'], o['kernel_ms'], 'ppo rollout', o['ppo']['rollout_env_steps_per_s'], o['ppo']['value'])"
