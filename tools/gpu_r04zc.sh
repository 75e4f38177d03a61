# round 4: the gradient launch with the first tile's sample indices loaded before the weight
# staging (AK_GRAD1_PREFETCH=2) against the default
set -o pipefail
mkdir -p gpurun_out
B=mujoco_playground_amd/csrc/build
timeout -k 10 150 python -u tools/ppo_kbench.py $B/libackppo.so $B/libackppo_pf2.so $B/libackppo.so $B/libackppo_pf2.so > gpurun_out/r04zc_kbench.log 2>&1 || { echo KBENCH_FAIL; tail -20 gpurun_out/r04zc_kbench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04zc_kbench.log | tail -40
