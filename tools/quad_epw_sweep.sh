# GPU: rollout tests and probe per envs-per-quad-wave setting (ACKPHYS_QUAD_EPW, rollout launches only)
mkdir -p gpurun_out
for epw in 8 16 12; do
  ACKPHYS_QUAD_EPW=$epw timeout -k 10 200 python -u -m pytest tests/test_gpu_rollout.py -x -q --timeout 120 --timeout-method thread > gpurun_out/epw_tests_$epw.log 2>&1 || { echo "tests failed epw=$epw"; tail -20 gpurun_out/epw_tests_$epw.log; exit 1; }
  echo "epw=$epw tests ok"
  ACKPHYS_QUAD_EPW=$epw timeout -k 10 200 python -u tools/probes/rollout_probe.py > gpurun_out/epw_probe_$epw.log 2>&1 || exit $?
  grep -v "contacts off" gpurun_out/epw_probe_$epw.log | grep K
done
