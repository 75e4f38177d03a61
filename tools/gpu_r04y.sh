# round 4: octet observation in the PPO observation wave + box rays without FMA contraction: every GPU
# test, the fused-rollout diff (obstacles), PPO rollout stamps, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/probes/ppo_fused_diff.py obstacles > gpurun_out/r04y_diff.log 2>&1 || { echo DIFF_FAIL; tail -20 gpurun_out/r04y_diff.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04y_diff.log | head -8
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r04y_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r04y_pytest.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|differs" gpurun_out/r04y_pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04y_smoke.log 2>&1 && tail -1 gpurun_out/r04y_smoke.log || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 200 python -u tools/probes/ppo_rollout_stamps.py obstacles > gpurun_out/r04y_ppo_stamps.log 2>&1 && grep -E "observation|policy  |dyn: loaded|past barrier" gpurun_out/r04y_ppo_stamps.log | head -6
timeout -k 10 400 python -u bench.py > gpurun_out/r04y_bench.json 2> gpurun_out/r04y_bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/r04y_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04y_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'secondary', d['secondary']['value'])
p=d['ppo']; print('ppo', p['value'], p['update_us_per_minibatch'], p['rollout_env_steps_per_s'])
o=d['obstacles']; print('obst', o['value'], 'ppo rollout', o['ppo']['rollout_env_steps_per_s'], o['ppo']['value'])"
