set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log | tail -3
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench.err; exit 1; }
TAG=${1:-r01}
bash tools/profile_gpu.sh $TAG > gpurun_out/prof.log 2>&1 || { echo PROF_FAIL; tail gpurun_out/prof.log; exit 1; }
timeout -k 10 500 python3 tools/profile_pmc.py > gpurun_out/pmc.log 2>&1 || { echo PMC_FAIL; tail gpurun_out/pmc.log; exit 1; }
echo ALL_OK
