# round 4: vectorised reduction A/B (R1_V 1 / 2 / 4) + Adam operand prefetch; PPO tests; update timing
set -o pipefail
mkdir -p gpurun_out
B=mujoco_playground_amd/csrc/build
timeout -k 10 120 python -u tools/ppo_kbench.py $B/libackppo_r1v1.so $B/libackppo_r1v2.so $B/libackppo.so > gpurun_out/r04h_kbench.log 2>&1 || { echo KBENCH_FAIL; tail -20 gpurun_out/r04h_kbench.log; exit 1; }
cat gpurun_out/r04h_kbench.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_ppo_rollout.py -q --timeout 240 --timeout-method thread > gpurun_out/r04h_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r04h_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/probes/ppo_update_timeline.py > gpurun_out/r04h_ppo_timing.log 2>&1 || { echo TIMING_FAIL; tail -20 gpurun_out/r04h_ppo_timing.log; exit 1; }
cat gpurun_out/r04h_ppo_timing.log
