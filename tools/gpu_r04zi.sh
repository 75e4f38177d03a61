# round 4 final: every GPU test and smoke at HEAD
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r04zi_pytest.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/r04zi_pytest.log; exit 1; }
tail -1 gpurun_out/r04zi_pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04zi_smoke.log 2>&1 && tail -1 gpurun_out/r04zi_smoke.log || { echo SMOKE_FAIL; tail -20 gpurun_out/r04zi_smoke.log; exit 1; }
