#!/bin/bash
# Round-3 GPU check (run through gpurun from the repo root): GPU tests, smoke, the post-reset
# probe, the counter list, the default bench and the driver's short bench. Each step has its own
# time limit and the chain stops at the first failure.
#   tools/gpu_r03.sh [tag]
set -o pipefail
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
step() {  # step <name> <timeout> <cmd...>: stdout+stderr to $OUT/<name>.log
  local name=$1 t=$2
  shift 2
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  tail -4 $OUT/$name.log
  return $rc
}
step pytest_gpu 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit $?
step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
if [ -z "$SKIP_PROBES" ]; then
  step counters 60 rocprofv3 -L || true
  step post_reset 300 python -u tools/probes/post_reset_probe.py || exit $?
fi
step bench 500 python -u bench.py || exit $?
step bench_short 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
if [ -n "$PROFILE" ]; then
  step prof 400 bash tools/profile_gpu.sh $TAG || exit $?
  step pmc 900 python3 tools/profile_pmc.py || exit $?
  step mfma 400 python3 tools/profile_mfma.py || exit $?
  STAMPS_ROLLOUT=8 STAMPS_JSON=$OUT/critical_path.json step stamps 300 python -u tools/stamps.py || exit $?
fi
echo ALL_OK
