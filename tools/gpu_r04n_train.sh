# round 4: the whole maze (D = 10 goal cells) with the entropy floor, and D = 6 with a higher floor
set -o pipefail
mkdir -p gpurun_out
C="--scene obstacles --action-repeat 10 --nohit-clear --collision-threshold 0.1 --envs 4096 --n-steps 64 --max-episode-steps 1500 --eval-every 250"
timeout -k 10 420 python -u tools/train_ppo.py $C --goal-cells 10 --iters 2500 --log-std-min -1.0 --out gpurun_out/r04_maze_g10_lsmin10.jsonl > gpurun_out/r04n_a.log 2>&1 || { echo A_FAIL; tail -20 gpurun_out/r04n_a.log; exit 1; }
tail -1 gpurun_out/r04_maze_g10_lsmin10.jsonl | head -c 300; echo
timeout -k 10 330 python -u tools/train_ppo.py $C --goal-cells 6 --iters 2000 --log-std-min -0.7 --out gpurun_out/r04_maze_g6_lsmin07.jsonl > gpurun_out/r04n_b.log 2>&1 || { echo B_FAIL; tail -20 gpurun_out/r04n_b.log; exit 1; }
tail -1 gpurun_out/r04_maze_g6_lsmin07.jsonl | head -c 300; echo
