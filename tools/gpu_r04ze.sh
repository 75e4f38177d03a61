# round 4: the data-parallel update's Adam launch forming the norm blocks itself (one launch fewer
# after the gradient's all-reduce) -- PPO GPU tests, then the bench's PPO leg with it and without
set -o pipefail
mkdir -p gpurun_out
B=mujoco_playground_amd/csrc/build
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py -q --timeout 240 --timeout-method thread > gpurun_out/r04ze_pytest.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/r04ze_pytest.log; exit 1; }
tail -2 gpurun_out/r04ze_pytest.log
L="--no-cpu --no-secondary --no-obstacles --no-per-step --no-buffer-leg"
timeout -k 10 300 python -u bench.py $L > gpurun_out/r04ze_bench.json 2> gpurun_out/r04ze_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r04ze_bench.err; exit 1; }
cp $B/libackppo.so $B/libackppo_default.so && cp $B/libackppo_dpnb.so $B/libackppo.so
timeout -k 10 300 python -u bench.py $L > gpurun_out/r04ze_bench_nb.json 2> gpurun_out/r04ze_bench_nb.err
rc=$?
cp $B/libackppo_default.so $B/libackppo.so
[ $rc -eq 0 ] || { echo BENCH_NB_FAIL; tail -20 gpurun_out/r04ze_bench_nb.err; exit 1; }
python3 -c "
import json
for f in ['gpurun_out/r04ze_bench.json','gpurun_out/r04ze_bench_nb.json']:
  d=json.loads(open(f).read().strip().splitlines()[-1]); p=d['ppo']
  print(f, p['value'], p['update_us_per_minibatch'], p['dp_update_path']['update_us_per_minibatch'])"
