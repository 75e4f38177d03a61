# round 4: noinline probe after the opaque-value fix, quad parity tests, PPO update timing (fused vs not) + kernel trace
set -o pipefail
mkdir -p gpurun_out
B=mujoco_playground_amd/csrc/build
timeout -k 10 240 python -u tools/probes/noinline_probe.py find $B/libackphys_noinl.so > gpurun_out/r04f_noinl_find.log 2>&1 || { echo FIND_FAIL; tail -20 gpurun_out/r04f_noinl_find.log; exit 1; }
tail -3 gpurun_out/r04f_noinl_find.log
timeout -k 10 120 python -u tools/probes/ppo_update_timeline.py > gpurun_out/r04f_ppo_timing.log 2>&1 || { echo TIMING_FAIL; tail -20 gpurun_out/r04f_ppo_timing.log; exit 1; }
grep fuse gpurun_out/r04f_ppo_timing.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04f_trace -o t -- python3 $GRAFT_REPO_ROOT/tools/probes/ppo_update_timeline.py > $GRAFT_REPO_ROOT/gpurun_out/r04f_trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r04f_trace.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/probes/ppo_update_timeline.py --trace gpurun_out/r04f_trace > gpurun_out/r04f_trace_summary.log 2>&1 && cat gpurun_out/r04f_trace_summary.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_obstacles.py tests/test_gpu_rollout.py tests/test_gpu_ppo_rollout.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r04f_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r04f_tests.log
exit $rc
