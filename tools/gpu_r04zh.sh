# round 4: the reduction with 16-B loads (AK_PPO_RA_VEC=1, 256 threads, libackppo_vec.so) against
# the scalar form (the default build)
set -o pipefail
mkdir -p gpurun_out
B=mujoco_playground_amd/csrc/build
cp $B/libackppo.so $B/libackppo_ra0.so && cp $B/libackppo_vec.so $B/libackppo.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py -q --timeout 240 --timeout-method thread > gpurun_out/r04zh_pytest.log 2>&1
rc=$?
tail -2 gpurun_out/r04zh_pytest.log
[ $rc -eq 0 ] || { cp $B/libackppo_ra0.so $B/libackppo.so; echo TEST_FAIL; tail -30 gpurun_out/r04zh_pytest.log; exit 1; }
timeout -k 10 150 python -u tools/ppo_kbench.py $B/libackppo_vec.so $B/libackppo_ra0.so $B/libackppo_vec.so $B/libackppo_ra0.so > gpurun_out/r04zh_kbench.log 2>&1 || { echo KBENCH_FAIL; tail -20 gpurun_out/r04zh_kbench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04zh_kbench.log | tail -4
L="--no-cpu --no-secondary --no-obstacles --no-per-step --no-buffer-leg"
for i in 1 2; do
  for v in vec ra0; do
    cp $B/libackppo_$v.so $B/libackppo.so
    timeout -k 10 300 python -u bench.py $L > gpurun_out/r04zh_$v$i.json 2> gpurun_out/r04zh_$v$i.err || { cp $B/libackppo_ra0.so $B/libackppo.so; echo BENCH_FAIL; tail -20 gpurun_out/r04zh_$v$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04zh_$v$i.json').read().strip().splitlines()[-1]); p=d['ppo']
print('$v$i', round(p['value']/1e6,2), round(p['update_us_per_minibatch'],2), round(p['dp_update_path']['update_us_per_minibatch'],2))"
  done
done
cp $B/libackppo_ra0.so $B/libackppo.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py -q --timeout 240 --timeout-method thread > gpurun_out/r04zh_pytest_ra0.log 2>&1 || { echo TEST_RA0_FAIL; tail -30 gpurun_out/r04zh_pytest_ra0.log; exit 1; }
tail -1 gpurun_out/r04zh_pytest_ra0.log
