# round 4: policy_forward with typed address spaces (PPO rollout), grad defaults NT=2 / no prefetch /
# R1_V=1 against variants, PPO tests, update timing + kernel traces (image on / off), PPO rollout
# stamps, full bench
set -o pipefail
mkdir -p gpurun_out
B=mujoco_playground_amd/csrc/build
R=$GRAFT_REPO_ROOT
timeout -k 10 150 python -u tools/ppo_kbench.py $B/libackppo.so $B/libackppo_v4.so $B/libackppo_nt1.so > gpurun_out/r04l_kbench.log 2>&1 || { echo KBENCH_FAIL; tail -20 gpurun_out/r04l_kbench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04l_kbench.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_ppo_rollout.py -q --timeout 240 --timeout-method thread > gpurun_out/r04l_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r04l_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/probes/ppo_update_timeline.py > gpurun_out/r04l_ppo_timing.log 2>&1 || { echo TIMING_FAIL; tail -20 gpurun_out/r04l_ppo_timing.log; exit 1; }
grep fuse gpurun_out/r04l_ppo_timing.log
for cfg in 0,1 0,0; do
  n=r04l_trace_${cfg/,/}
  (cd /tmp && TMPDIR=/tmp timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/$n -o t -- python3 $R/tools/probes/ppo_update_timeline.py --only $cfg > $R/gpurun_out/$n.log 2>&1) || { echo TRACE_FAIL; tail -20 gpurun_out/$n.log; exit 1; }
  python3 tools/probes/ppo_update_timeline.py --trace gpurun_out/$n > gpurun_out/${n}_summary.log 2>&1 && head -12 gpurun_out/${n}_summary.log
done
timeout -k 10 200 python -u tools/probes/ppo_rollout_stamps.py flat > gpurun_out/r04l_ppo_stamps.log 2>&1 && timeout -k 10 200 python -u tools/probes/ppo_rollout_stamps.py obstacles >> gpurun_out/r04l_ppo_stamps.log 2>&1 || { echo PPOSTAMPS_FAIL; tail -20 gpurun_out/r04l_ppo_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04l_ppo_stamps.log
timeout -k 10 400 python -u bench.py > gpurun_out/r04l_bench.json 2> gpurun_out/r04l_bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/r04l_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04l_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'kern_ms', d['roofline']['kernel_ms'])
print('secondary', d['secondary']['value'], d['secondary']['kernel_ms'], 'cp', (d['secondary'].get('roofline') or {}).get('critical_path'))
p=d['ppo']; print('ppo', p['value'], p['update_us_per_minibatch'], p['rollout_env_steps_per_s'])
o=d['obstacles']; print('obst', o['value'], o['kernel_ms'], 'ppo rollout', o['ppo']['rollout_env_steps_per_s'], o['ppo']['value'])"
