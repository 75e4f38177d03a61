# round 4: grad-kernel timeline (2 vs 1 workgroups per CU) + the noinline wall-contact probe
set -o pipefail
mkdir -p gpurun_out
B=mujoco_playground_amd/csrc/build
timeout -k 10 60 python -u tools/ppo_kbench.py --stamps $B/libackppo_stamps.so > gpurun_out/r04c_stamps.log 2>&1 || { echo STAMPS_FAIL; tail -20 gpurun_out/r04c_stamps.log; exit 1; }
timeout -k 10 60 python -u tools/ppo_kbench.py --stamps $B/libackppo_stamps1cu.so > gpurun_out/r04c_stamps1cu.log 2>&1 || { echo STAMPS1_FAIL; tail -20 gpurun_out/r04c_stamps1cu.log; exit 1; }
grep batch gpurun_out/r04c_stamps.log gpurun_out/r04c_stamps1cu.log
timeout -k 10 300 python -u tools/probes/noinline_probe.py find $B/libackphys_noinl.so > gpurun_out/r04c_noinl_find.log 2>&1 || { echo FIND_FAIL; tail -20 gpurun_out/r04c_noinl_find.log; exit 1; }
tail -8 gpurun_out/r04c_noinl_find.log
if [ -f gpurun_out/noinl_case.npz ]; then
  timeout -k 10 120 python -u tools/probes/noinline_probe.py step $B/libackphys_noinl.so noinl > gpurun_out/r04c_noinl_step.log 2>&1 || { echo STEP_FAIL; tail -20 gpurun_out/r04c_noinl_step.log; exit 1; }
  timeout -k 10 120 python -u tools/probes/noinline_probe.py step $B/libackphys.so inl >> gpurun_out/r04c_noinl_step.log 2>&1 || { echo STEP2_FAIL; tail -20 gpurun_out/r04c_noinl_step.log; exit 1; }
  cat gpurun_out/r04c_noinl_step.log | grep -v amdgpu.ids
fi
