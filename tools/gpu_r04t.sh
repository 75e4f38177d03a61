# round 4: Adam step fused into the next gradient launch (blocked norm from the reduction):
# PPO tests, update timing + trace, PPO rollout policy stamps, grad stamps, bench
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_ppo_rollout.py tests/test_gpu_dropin.py -q --timeout 240 --timeout-method thread > gpurun_out/r04t_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r04t_tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|error" gpurun_out/r04t_tests.log | head -20; exit $rc; fi
timeout -k 10 120 python -u tools/probes/ppo_update_timeline.py > gpurun_out/r04t_ppo_timing.log 2>&1 || { echo TIMING_FAIL; tail -20 gpurun_out/r04t_ppo_timing.log; exit 1; }
grep epoch_buffers gpurun_out/r04t_ppo_timing.log
(cd /tmp && TMPDIR=/tmp timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r04t_trace -o t -- python3 $R/tools/probes/ppo_update_timeline.py --only 1,0,1 > $R/gpurun_out/r04t_trace.log 2>&1) || { echo TRACE_FAIL; tail -20 gpurun_out/r04t_trace.log; exit 1; }
python3 tools/probes/ppo_update_timeline.py --trace gpurun_out/r04t_trace > gpurun_out/r04t_trace_summary.log 2>&1 && head -14 gpurun_out/r04t_trace_summary.log
timeout -k 10 200 python -u tools/probes/ppo_rollout_stamps.py flat > gpurun_out/r04t_ppo_stamps.log 2>&1 && timeout -k 10 200 python -u tools/probes/ppo_rollout_stamps.py obstacles >> gpurun_out/r04t_ppo_stamps.log 2>&1 || { echo PPOSTAMPS_FAIL; tail -20 gpurun_out/r04t_ppo_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04t_ppo_stamps.log
timeout -k 10 400 python -u bench.py > gpurun_out/r04t_bench.json 2> gpurun_out/r04t_bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/r04t_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04t_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'kern_ms', d['roofline']['kernel_ms'])
print('secondary', d['secondary']['value'], d['secondary']['kernel_ms'])
p=d['ppo']; print('ppo', p['value'], p['update_us_per_minibatch'], p['rollout_env_steps_per_s'])
o=d['obstacles']; print('obst', o['value'], o['kernel_ms'], 'ppo rollout', o['ppo']['rollout_env_steps_per_s'], o['ppo']['value'])"
