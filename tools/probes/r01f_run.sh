#!/bin/bash
# r01f GPU probe: quad race variant sweep, then the full GPU suite + smoke on the product build.
set -o pipefail
mkdir -p gpurun_out
bash tools/variant_sweep.sh qbase qrace > gpurun_out/sweep.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_race.txt 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_race.txt 2>&1
exit $(( rc > 0 ? rc : $? ))
