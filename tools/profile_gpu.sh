#!/bin/bash
# rocprofv3 kernel-trace summary of bench.py (run on the GPU box from the repo root).
# usage: tools/profile_gpu.sh <tag>
set -e
TAG=${1:-run}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o prof -- \
  python3 $ROOT/bench.py --no-cpu --steps 300 --warmup 30 > $OUT/bench_stdout.json 2> $OUT/stderr.log
find $OUT -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
# a rollout launch runs K steps: list each rollout dispatch (timed launches: K = 300)
python3 $ROOT/tools/dispatch_summary.py $OUT > $OUT/rollout_dispatches.csv
cat $OUT/kernel_stats.csv | head -20
