# round 4: noinline dumps (inline vs noinline diagnostic builds) + PPO tests with the fused Adam step + PPO bench leg
set -o pipefail
mkdir -p gpurun_out
B=mujoco_playground_amd/csrc/build
timeout -k 10 60 python -u tools/probes/noinline_dump.py $B/libackphys_stamps.so inl > gpurun_out/r04d_dump.log 2>&1 || { echo DUMP_FAIL; tail -20 gpurun_out/r04d_dump.log; exit 1; }
timeout -k 10 60 python -u tools/probes/noinline_dump.py $B/libackphys_stamps_noinl.so noinl >> gpurun_out/r04d_dump.log 2>&1 || { echo DUMP2_FAIL; tail -20 gpurun_out/r04d_dump.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04d_dump.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_ppo_rollout.py -v --timeout 240 --timeout-method thread > gpurun_out/r04d_ppo_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/r04d_ppo_tests.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended with $rc: stopping"; exit $rc; fi
timeout -k 10 90 python -u tools/ppo_kbench.py $B/libackppo_g1.so $B/libackppo.so > gpurun_out/r04d_kbench.log 2>&1 && timeout -k 10 60 python -u tools/ppo_kbench.py --stamps $B/libackppo_stamps.so >> gpurun_out/r04d_kbench.log 2>&1 || { echo KBENCH_FAIL; tail -20 gpurun_out/r04d_kbench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04d_kbench.log
timeout -k 10 300 python -u bench.py --steps 100 --no-cpu --no-secondary --no-obstacles --no-per-step --no-buffer-leg > gpurun_out/r04d_bench.json 2> gpurun_out/r04d_bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/r04d_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04d_bench.json').read().strip().splitlines()[-1]); p=d['ppo']
print('ppo', p['value'], 'update us/mb', p['update_us_per_minibatch'], 'rollout', p['rollout_env_steps_per_s'], 'dp ratio', p['dp_update_path']['ratio_to_single_rank_update'])"
exit $rc
