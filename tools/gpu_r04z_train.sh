# round 4: the whole maze (D = 10) with the entropy floor at -0.7
set -o pipefail
mkdir -p gpurun_out
C="--scene obstacles --action-repeat 10 --nohit-clear --collision-threshold 0.1 --envs 4096 --n-steps 64 --max-episode-steps 1500 --eval-every 250"
timeout -k 10 600 python -u tools/train_ppo.py $C --goal-cells 10 --iters 3000 --log-std-min -0.7 --out gpurun_out/r04_maze_g10_lsmin07.jsonl > gpurun_out/r04z_train.log 2>&1 || { echo TRAIN_FAIL; tail -20 gpurun_out/r04z_train.log; exit 1; }
tail -1 gpurun_out/r04_maze_g10_lsmin07.jsonl | head -c 300; echo
