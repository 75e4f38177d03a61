# round 4: the whole maze (D = 10) with the -1.0 entropy floor, (a) a goal curriculum 3 -> 10,
# (b) gamma 0.995
set -o pipefail
mkdir -p gpurun_out
C="--scene obstacles --action-repeat 10 --nohit-clear --collision-threshold 0.1 --envs 4096 --n-steps 64 --max-episode-steps 1500 --eval-every 250 --log-std-min -1.0"
timeout -k 10 560 python -u tools/train_ppo.py $C --goal-cells 10 --goal-cells-start 3 --goal-cells-every 300 --iters 4000 --out gpurun_out/r04_maze_g10_curr_lsmin10.jsonl > gpurun_out/r04zd_train_a.log 2>&1 || { echo TRAIN_A_FAIL; tail -20 gpurun_out/r04zd_train_a.log; exit 1; }
timeout -k 10 560 python -u tools/train_ppo.py $C --goal-cells 10 --gamma 0.995 --iters 4000 --out gpurun_out/r04_maze_g10_g995_lsmin10.jsonl > gpurun_out/r04zd_train_b.log 2>&1 || { echo TRAIN_B_FAIL; tail -20 gpurun_out/r04zd_train_b.log; exit 1; }
