# round 4: the noinline probe after the value-semantics fix + PPO tests (grad1 + fused Adam) + kernel A/B + PPO bench leg
set -o pipefail
mkdir -p gpurun_out
B=mujoco_playground_amd/csrc/build
timeout -k 10 300 python -u tools/probes/noinline_probe.py find $B/libackphys_noinl.so > gpurun_out/r04e_noinl_find.log 2>&1 || { echo FIND_FAIL; tail -20 gpurun_out/r04e_noinl_find.log; exit 1; }
tail -3 gpurun_out/r04e_noinl_find.log
timeout -k 10 60 python -u tools/probes/noinline_dump.py $B/libackphys_stamps_noinl.so noinl_fixed > gpurun_out/r04e_dump.log 2>&1 || { echo DUMP_FAIL; tail -20 gpurun_out/r04e_dump.log; exit 1; }
grep -E "qacc |lane 0 slot 0" gpurun_out/r04e_dump.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_ppo_rollout.py -v --timeout 240 --timeout-method thread > gpurun_out/r04e_ppo_tests.log 2>&1
rc=$?
grep -E "FAILED|passed|failed|Error" gpurun_out/r04e_ppo_tests.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended with $rc: stopping"; exit $rc; fi
timeout -k 10 90 python -u tools/ppo_kbench.py $B/libackppo.so $B/libackppo_g2.so > gpurun_out/r04e_kbench.log 2>&1 && timeout -k 10 60 python -u tools/ppo_kbench.py --stamps $B/libackppo_stamps.so >> gpurun_out/r04e_kbench.log 2>&1 || { echo KBENCH_FAIL; tail -20 gpurun_out/r04e_kbench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04e_kbench.log
timeout -k 10 300 python -u bench.py --steps 100 --no-cpu --no-secondary --no-obstacles --no-per-step --no-buffer-leg > gpurun_out/r04e_bench.json 2> gpurun_out/r04e_bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/r04e_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04e_bench.json').read().strip().splitlines()[-1]); p=d['ppo']
print('ppo', p['value'], 'update us/mb', p['update_us_per_minibatch'], 'rollout', p['rollout_env_steps_per_s'], 'dp ratio', p['dp_update_path']['ratio_to_single_rank_update'])"
exit $rc
