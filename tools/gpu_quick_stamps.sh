# GPU: all GPU tests, the rollout probe, then rollout stamps (each only if the previous step ended normally)
bash tools/gpu_quick.sh || exit $?
STAMPS_ROLLOUT=8 timeout -k 10 200 python -u tools/stamps.py > gpurun_out/stamps_roll.log 2>&1 || exit $?
head -16 gpurun_out/stamps_roll.log
