# round 4: PPO rollout policy sub-phase stamps; then the D = 10 maze training (tools/gpu_r04n_train.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/probes/ppo_rollout_stamps.py flat > gpurun_out/r04p_ppo_stamps.log 2>&1 && timeout -k 10 200 python -u tools/probes/ppo_rollout_stamps.py obstacles >> gpurun_out/r04p_ppo_stamps.log 2>&1 || { echo PPOSTAMPS_FAIL; tail -20 gpurun_out/r04p_ppo_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04p_ppo_stamps.log
bash tools/gpu_r04n_train.sh
