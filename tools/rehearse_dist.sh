#!/bin/bash
# bench.py under torchrun with 2 ranks sharing the one GPU of a gpurun box (gloo collectives):
# rehearses the N>1 code path (sharding, barrier/max timing, episode gather, DP PPO all-reduces).
set -o pipefail
mkdir -p gpurun_out
export ACKPHYS_DIST_BACKEND=gloo ACKPHYS_DEVICE_OVERRIDE=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 100 --warmup 10 --no-cpu > gpurun_out/dist2.json 2> gpurun_out/dist2.err \
  || { tail -20 gpurun_out/dist2.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/dist2.json').read().strip().splitlines()[-1]); print('n_gpus', d['n_gpus'], 'value', round(d['value']/1e6,1), 'M/s', 'ppo', round(d['ppo']['value']/1e6,2), d['ppo']['config'], 'obst ppo', round(d['obstacles']['ppo']['value']/1e6,2))"
