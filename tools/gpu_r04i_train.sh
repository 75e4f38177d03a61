# round 4, VERDICT r03 item 8: the maze task at D = 6 goal cells with the opt-in log_std floor
# (the r03 D = 6 run collapsed to std 0.01 at 20 % success). Common: obstacle scene, R = 10,
# nohit_clear, collision threshold 0.1, 4096 envs, n_steps 64, 1500-step episodes.
set -o pipefail
mkdir -p gpurun_out
C="--scene obstacles --action-repeat 10 --nohit-clear --collision-threshold 0.1 --envs 4096 --n-steps 64 --max-episode-steps 1500 --eval-every 200"
timeout -k 10 330 python -u tools/train_ppo.py $C --goal-cells 6 --iters 2000 --log-std-min -1.0 --out gpurun_out/r04_maze_g6_lsmin10.jsonl > gpurun_out/r04i_a.log 2>&1 || { echo A_FAIL; tail -20 gpurun_out/r04i_a.log; exit 1; }
tail -1 gpurun_out/r04_maze_g6_lsmin10.jsonl | head -c 400; echo
timeout -k 10 330 python -u tools/train_ppo.py $C --goal-cells 6 --iters 2000 --log-std-min -1.6 --out gpurun_out/r04_maze_g6_lsmin16.jsonl > gpurun_out/r04i_b.log 2>&1 || { echo B_FAIL; tail -20 gpurun_out/r04i_b.log; exit 1; }
tail -1 gpurun_out/r04_maze_g6_lsmin16.jsonl | head -c 400; echo
timeout -k 10 330 python -u tools/train_ppo.py $C --goal-cells 6 --goal-cells-start 1 --goal-cells-every 150 --iters 2000 --log-std-min -1.0 --out gpurun_out/r04_maze_g6_curr_lsmin10.jsonl > gpurun_out/r04i_c.log 2>&1 || { echo C_FAIL; tail -20 gpurun_out/r04i_c.log; exit 1; }
tail -1 gpurun_out/r04_maze_g6_curr_lsmin10.jsonl | head -c 400; echo
