# round 4 final: (a) the octet-observation build's parity (diff probe + fused-rollout tests with it in
# place of the default library, then the default restored), (b) every GPU test, smoke, the bench
# line, a kernel-trace summary of the bench command
set -o pipefail
mkdir -p gpurun_out
B=mujoco_playground_amd/csrc/build
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/probes/ppo_fused_diff.py flat libackphys_oct.so > gpurun_out/r04x_diff.log 2>&1 || { echo DIFF_FAIL; tail -20 gpurun_out/r04x_diff.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04x_diff.log | head -6
cp $B/libackphys.so $B/libackphys_default.so && cp $B/libackphys_oct.so $B/libackphys.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo_rollout.py tests/test_gpu_variant.py -q --timeout 240 --timeout-method thread > gpurun_out/r04x_oct_tests.log 2>&1
orc=$?
tail -2 gpurun_out/r04x_oct_tests.log
if [ $orc -ne 0 ] && [ $orc -ne 1 ]; then exit $orc; fi
if [ $orc -eq 0 ]; then
  timeout -k 10 200 python -u tools/probes/ppo_rollout_stamps.py obstacles > gpurun_out/r04x_oct_stamps.log 2>&1 && grep -E "observation|policy:|dyn: loaded|past barrier" gpurun_out/r04x_oct_stamps.log | head -8
  timeout -k 10 300 python -u bench.py --no-cpu --no-per-step --no-buffer-leg --no-secondary > gpurun_out/r04x_oct_bench.json 2> gpurun_out/r04x_oct_bench.err && python3 -c "
import json; d=json.loads(open('gpurun_out/r04x_oct_bench.json').read().strip().splitlines()[-1])
p=d['ppo']; print('OCT ppo', p['value'], p['rollout_env_steps_per_s'])
o=d['obstacles']; print('OCT obst ppo rollout', o['ppo']['rollout_env_steps_per_s'], o['ppo']['value'])"
fi
cp $B/libackphys_default.so $B/libackphys.so
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r04x_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r04x_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04x_smoke.log 2>&1 && tail -1 gpurun_out/r04x_smoke.log || { echo SMOKE_FAIL; tail -20 gpurun_out/r04x_smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/r04x_bench.json 2> gpurun_out/r04x_bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/r04x_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04x_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'kern_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])
print('secondary', d['secondary']['value'])
p=d['ppo']; print('ppo', p['value'], p['update_us_per_minibatch'], p['rollout_env_steps_per_s'])
o=d['obstacles']; print('obst', o['value'], 'ppo rollout', o['ppo']['rollout_env_steps_per_s'], o['ppo']['value'])"
(cd /tmp && TMPDIR=/tmp timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04x_prof -o b -- python3 $R/bench.py --no-cpu > $R/gpurun_out/r04x_prof.log 2>&1) || { echo PROF_FAIL; tail -5 gpurun_out/r04x_prof.log; }
exit $rc
