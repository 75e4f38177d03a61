# round 4 close: kernel-trace summary of the bench command at the octet-observation build
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
(cd /tmp && TMPDIR=/tmp timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04za_prof -o b -- python3 $R/bench.py --no-cpu > $R/gpurun_out/r04za_prof.log 2>&1) || { echo PROF_FAIL; tail -20 gpurun_out/r04za_prof.log; exit 1; }
find gpurun_out/r04za_prof -name "*kernel_stats.csv" | head -3
