# round 4: the octet observation build (csrc/build/libackphys_oct.so) against the per-step path:
# diff probe, then the fused-rollout parity tests with it in place of the default library
set -o pipefail
mkdir -p gpurun_out
B=mujoco_playground_amd/csrc/build
timeout -k 10 200 python -u tools/probes/ppo_fused_diff.py flat libackphys_oct.so > gpurun_out/r04w_diff.log 2>&1 || { echo DIFF_FAIL; tail -20 gpurun_out/r04w_diff.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04w_diff.log | head -12
cp $B/libackphys_oct.so $B/libackphys.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_ppo_rollout.py tests/test_gpu_ppo.py tests/test_gpu_variant.py -q --timeout 240 --timeout-method thread > gpurun_out/r04w_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r04w_tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" gpurun_out/r04w_tests.log | head -20; exit $rc; fi
timeout -k 10 200 python -u tools/probes/ppo_rollout_stamps.py obstacles > gpurun_out/r04w_ppo_stamps.log 2>&1 || true
timeout -k 10 400 python -u bench.py --no-cpu --no-per-step --no-buffer-leg > gpurun_out/r04w_bench.json 2> gpurun_out/r04w_bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/r04w_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04w_bench.json').read().strip().splitlines()[-1])
p=d['ppo']; print('ppo', p['value'], p['update_us_per_minibatch'], p['rollout_env_steps_per_s'])
o=d['obstacles']; print('obst', o['value'], o['kernel_ms'], 'ppo rollout', o['ppo']['rollout_env_steps_per_s'], o['ppo']['value'])"
