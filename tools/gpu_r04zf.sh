# round 4: the data-parallel update with and without the self-norm Adam launch, alternating runs
set -o pipefail
mkdir -p gpurun_out
B=mujoco_playground_amd/csrc/build
L="--no-cpu --no-secondary --no-obstacles --no-per-step --no-buffer-leg"
cp $B/libackppo.so $B/libackppo_sn.so
for i in 1 2 3; do
  for v in sn dpnb; do
    cp $B/libackppo_$v.so $B/libackppo.so
    timeout -k 10 300 python -u bench.py $L > gpurun_out/r04zf_$v$i.json 2> gpurun_out/r04zf_$v$i.err || { cp $B/libackppo_sn.so $B/libackppo.so; echo BENCH_FAIL; tail -20 gpurun_out/r04zf_$v$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04zf_$v$i.json').read().strip().splitlines()[-1]); p=d['ppo']
print('$v$i', round(p['value']/1e6,2), round(p['update_us_per_minibatch'],2), round(p['dp_update_path']['update_us_per_minibatch'],2))"
  done
done
cp $B/libackppo_sn.so $B/libackppo.so
