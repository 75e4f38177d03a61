# GPU: all GPU tests, the rollout probe, the fused PPO rollout bench leg (each under its own limit)
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_all.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/probes/rollout_probe.py > gpurun_out/rollout_probe.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu --steps 300 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || exit $?
python3 - <<'PY'
import json
d = json.load(open('gpurun_out/bench_quick.json'))
print('value', round(d['value'] / 1e6, 1), 'M; contacts on', round(d['secondary']['value'] / 1e6, 1), 'M;',
      'obst', round(d['obstacles']['value'] / 1e6, 1), 'M; ppo rollout', round(d['ppo']['rollout_env_steps_per_s'] / 1e6, 1),
      'M; ppo obst rollout', round(d['obstacles']['ppo']['rollout_env_steps_per_s'] / 1e6, 1), 'M')
PY
