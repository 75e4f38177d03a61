set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
bash tools/variant_sweep.sh qbase qsmooth > gpurun_out/sweep.log 2>&1 || exit 1
exit $rc
