# GPU: all GPU tests, then the rollout probe (only if the tests ended normally: pass or assertion failures)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -6 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended with $rc: stopping"; exit $rc; fi
timeout -k 10 200 python -u tools/probes/rollout_probe.py > gpurun_out/rollout_probe.log 2>&1
rc2=$?
tail -12 gpurun_out/rollout_probe.log
exit $(( rc > rc2 ? rc : rc2 ))
