# round 4: reduction A/B (R1_V 1 / 2 / 4), grad variants (two-tile workgroups, tile prefetch), PPO tests
# on the default build and on the two-tile build, update timing; PPO rollout stamps; critical path of
# the quad / obstacle rollout kernels and the obstacle kernel's PMC (tools/gpu_r04j.sh)
set -o pipefail
mkdir -p gpurun_out
B=mujoco_playground_amd/csrc/build
timeout -k 10 150 python -u tools/ppo_kbench.py $B/libackppo_r1v1.so $B/libackppo_r1v2.so $B/libackppo.so $B/libackppo_pf0.so $B/libackppo_nt2.so $B/libackppo_nt2pf0.so > gpurun_out/r04k_kbench.log 2>&1 || { echo KBENCH_FAIL; tail -20 gpurun_out/r04k_kbench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04k_kbench.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_ppo_rollout.py -q --timeout 240 --timeout-method thread > gpurun_out/r04k_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r04k_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/probes/ppo_update_timeline.py > gpurun_out/r04k_ppo_timing.log 2>&1 || { echo TIMING_FAIL; tail -20 gpurun_out/r04k_ppo_timing.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04k_ppo_timing.log
cp $B/libackppo.so $B/libackppo_default.so && cp $B/libackppo_nt2.so $B/libackppo.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py -q --timeout 240 --timeout-method thread > gpurun_out/r04k_tests_nt2.log 2>&1
rc=$?
tail -3 gpurun_out/r04k_tests_nt2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/probes/ppo_update_timeline.py > gpurun_out/r04k_ppo_timing_nt2.log 2>&1 || { echo TIMING2_FAIL; tail -20 gpurun_out/r04k_ppo_timing_nt2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04k_ppo_timing_nt2.log
cp $B/libackppo_default.so $B/libackppo.so
timeout -k 10 200 python -u tools/probes/ppo_rollout_stamps.py flat > gpurun_out/r04k_ppo_stamps.log 2>&1 && timeout -k 10 200 python -u tools/probes/ppo_rollout_stamps.py obstacles >> gpurun_out/r04k_ppo_stamps.log 2>&1 || { echo PPOSTAMPS_FAIL; tail -20 gpurun_out/r04k_ppo_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04k_ppo_stamps.log
bash tools/gpu_r04j.sh
