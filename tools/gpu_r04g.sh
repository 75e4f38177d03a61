# round 4: all GPU tests + bench (REG0 back in the PPO kernels, opaque slot selection) + PMC of the rollout-buffer leg
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r04g_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r04g_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended with $rc: stopping"; exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/r04g_bench.json 2> gpurun_out/r04g_bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/r04g_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04g_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'kern_ms', d['roofline']['kernel_ms'])
print('buffer', {k: d['rollout_buffer'][k] for k in ('value','kernel_ms','achieved_GBps','frac')})
print('secondary', d['secondary']['value'], d['secondary']['kernel_ms'])
p=d['ppo']; print('ppo', p['value'], p['update_us_per_minibatch'], p['rollout_env_steps_per_s'])
o=d['obstacles']; print('obst', o['value'], o['kernel_ms'], 'ppo rollout', o['ppo']['rollout_env_steps_per_s'], o['ppo']['value'])"
timeout -k 10 300 python3 tools/profile_pmc.py 20,1000 --buffers > gpurun_out/r04g_pmc_buf.log 2>&1 || { echo PMC_FAIL; tail -20 gpurun_out/r04g_pmc_buf.log; exit 1; }
grep -o '"hbm_bytes_per_step": [0-9.]*' gpurun_out/r04g_pmc_buf.log
timeout -k 10 400 python3 tools/profile_mfma.py > gpurun_out/r04g_mfma.log 2>&1 || { echo MFMA_FAIL; tail -20 gpurun_out/r04g_mfma.log; exit 1; }
grep -E '"mfma_util"|"mfma_tflops"|median_duration' gpurun_out/r04g_mfma.log
exit $rc
