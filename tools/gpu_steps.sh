#!/bin/bash
# One parametrised GPU-box runner (replaces the per-round tools/gpu_r0*.sh one-offs).
#   bash tools/gpu_steps.sh TAG STEP [STEP ...]
# Run from the repo root on the GPU box (gpurun). Each step has its own time limit, writes under
# gpurun_out/TAG_*, and the first failing step ends the script (no GPU step runs after a failure).
# Steps:
#   tests[=EXPR]       pytest -m gpu (optionally -k EXPR)
#   smoke              __graft_entry__.smoke()
#   bench[=ARGS]       python bench.py ARGS (comma-separated flags, e.g. bench=--steps,20,--warmup,5)
#   prof               rocprofv3 --kernel-trace --stats of the default bench command
#   pmc                tools/profile_pmc.py (separate --pmc passes)
#   py=SCRIPT,ARGS     python3 -u SCRIPT ARGS
#   profpy=SCRIPT,ARGS rocprofv3 --kernel-trace --stats of python3 SCRIPT ARGS
#   mfma               tools/profile_mfma.py
#   kbench             tools/ppo_kbench.py
#   quad=LIB:EPW,...   tools/probes/quad_time.py over step-library builds (diag_libs/*.so)
#   stamps=ARGS        tools/stamps.py ARGS (comma-separated)
#   stalls[=RUNS]      tools/profile_stalls.py (SQ wait / issue counters of the rollout kernels)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
run() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "STEP_FAIL $name rc=$rc"; tail -30 "gpurun_out/${TAG}_${name}.log"; exit 1; fi
  tail -3 "gpurun_out/${TAG}_${name}.log"
}
for step in "$@"; do
  key=${step%%=*}; val=""; [ "$key" != "$step" ] && val=${step#*=}
  case $key in
    tests)
      if [ -n "$val" ]; then run tests 1100 python -u -m pytest tests -m gpu -x -v -k "$val" --timeout 240 --timeout-method thread
      else run tests 1100 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread; fi ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    bench)
      # bench with flags writes TAG_bench_<flags>.json, so two bench steps of one call keep both lines
      bn="${TAG}_bench"; [ -n "$val" ] && bn="${TAG}_bench_$(echo "$val" | tr -c 'a-zA-Z0-9\n' '_' | tr -s '_')"
      timeout -k 10 600 python -u bench.py ${val//,/ } > "gpurun_out/${bn}.json" 2> "gpurun_out/${bn}.err" \
        || { echo "STEP_FAIL bench"; tail -30 "gpurun_out/${bn}.err"; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', sys.argv[1], round(d['value']/1e6,1), 'M', {k: (round(d[k]['value']/1e6,2) if d.get(k) else None) for k in ('secondary','obstacles','ppo')})" "gpurun_out/${bn}.json" ;;
    prof)
      (cd /tmp && TMPDIR=/tmp timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_prof" -o b -- python3 "$R/bench.py" --no-cpu > "$R/gpurun_out/${TAG}_prof.log" 2>&1) \
        || { echo "STEP_FAIL prof"; tail -20 "gpurun_out/${TAG}_prof.log"; exit 1; }
      find "gpurun_out/${TAG}_prof" -name "*kernel_stats.csv" | head -3 ;;
    profpy)  # rocprofv3 kernel trace + stats of a python script: profpy=SCRIPT,ARGS...
      (cd /tmp && TMPDIR=/tmp timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_profpy" -o p -- python3 "$R/"${val//,/ } > "$R/gpurun_out/${TAG}_profpy.log" 2>&1) \
        || { echo "STEP_FAIL profpy"; tail -20 "gpurun_out/${TAG}_profpy.log"; exit 1; }
      tail -3 "gpurun_out/${TAG}_profpy.log" ;;
    py) run py 600 python3 -u ${val//,/ } ;;
    pmc) run pmc 900 python3 tools/profile_pmc.py ;;
    mfma) run mfma 600 python3 tools/profile_mfma.py ;;
    kbench) run kbench 600 python3 tools/ppo_kbench.py ${val//,/ } ;;
    quad) run quad 900 python3 -u tools/probes/quad_time.py ${val//,/ } ;;
    stamps) run stamps 900 python3 -u tools/stamps.py ${val//,/ } ;;
    stalls) run stalls 600 python3 -u tools/profile_stalls.py "$TAG" ${val//,/ } ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo ALL_OK
