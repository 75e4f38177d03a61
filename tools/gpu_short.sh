# GPU: the driver's exact bench command, and the headline-only short window with/without the secondary leg first
mkdir -p gpurun_out
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', round(d['value']/1e6,1), 'M', 'ms/step', round(d['ms_per_step']*1e3,3), 'kernel us', round(d['roofline']['kernel_ms']*1e3,3))" "$1" "$2"; }
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/driver_bench.json 2> gpurun_out/driver_bench.err || { tail gpurun_out/driver_bench.err; exit 1; }
show gpurun_out/driver_bench.json "driver command:"
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-ppo --no-obstacles > gpurun_out/sb1.json 2>> gpurun_out/driver_bench.err || exit 1
show gpurun_out/sb1.json "secondary first:"
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-ppo --no-obstacles --no-secondary > gpurun_out/sb2.json 2>> gpurun_out/driver_bench.err || exit 1
show gpurun_out/sb2.json "headline alone:"
