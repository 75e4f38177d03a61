# round 4: PPO grad kernel A/B (one net per workgroup vs two-net workgroup) + PPO GPU tests,
# then the full-size parity tests and the bench (tools/gpu_r04a.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/ppo_kbench.py mujoco_playground_amd/csrc/build/libackppo_g0.so mujoco_playground_amd/csrc/build/libackppo.so > gpurun_out/r04b_kbench.log 2>&1 || { echo KBENCH_FAIL; tail -20 gpurun_out/r04b_kbench.log; exit 1; }
cat gpurun_out/r04b_kbench.log
timeout -k 10 60 python -u tools/ppo_kbench.py --stamps mujoco_playground_amd/csrc/build/libackppo_stamps.so > gpurun_out/r04b_stamps.log 2>&1 || { echo STAMPS_FAIL; tail -20 gpurun_out/r04b_stamps.log; exit 1; }
cat gpurun_out/r04b_stamps.log
bash tools/gpu_r04a.sh
