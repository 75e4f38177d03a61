# round 4: full-size parity tests + variants-agree (tightened) + bench with the rollout-buffer leg
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_full.py "tests/test_gpu_parity.py::test_variants_agree_at_4096" tests/test_gpu_ppo.py tests/test_gpu_ppo_rollout.py -v -s --timeout 240 --timeout-method thread > gpurun_out/r04a_parity_full.log 2>&1
rc=$?
grep -E "full_size_parity|variants_agree|PASSED|FAILED|passed|failed|Error" gpurun_out/r04a_parity_full.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended with $rc: stopping"; exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/r04a_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r04a_bench.json'))
print('value', d['value'], 'kern_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])
print('buffer', {k: d['rollout_buffer'][k] for k in ('value','kernel_ms','achieved_GBps','frac')})
print('secondary', d['secondary']['value'], d['secondary']['kernel_ms'])
print('ppo', d['ppo']['value'], d['ppo']['update_us_per_minibatch'], d['ppo']['rollout_env_steps_per_s'], d['ppo']['dp_update_path'])
print('obst', d['obstacles']['value'], d['obstacles']['ppo']['rollout_env_steps_per_s'])
"
exit $rc
