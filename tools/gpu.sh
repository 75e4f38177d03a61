#!/bin/bash
# run a command on the GPU box via gpurun; stale gpurun_out/*.log files are removed first so a
# transient failure cannot be mistaken for fresh results. usage: tools/gpu.sh <timeout_s> '<cmd>'
T=${1:-600}; shift
rm -f gpurun_out/*.log gpurun_out/*.json 2>/dev/null
timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > gpurun_out/call.txt 2>&1
grep -E "status=|GPU-minutes left|stopped responding|refused" gpurun_out/call.txt | tail -3
