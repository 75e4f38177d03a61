# GPU: the driver's short bench window, and the window-cost probe
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-ppo --no-obstacles --no-secondary > gpurun_out/short_bench_$i.json 2> gpurun_out/short_bench.err || { tail gpurun_out/short_bench.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('short bench value', round(d['value']/1e6,1), 'M', 'ms/step', d['ms_per_step']*1e3, 'kernel us', d['roofline']['kernel_ms']*1e3, 'per-step-launch', round(d['per_step_launch']['value']/1e6,1))" gpurun_out/short_bench_$i.json
done
timeout -k 10 200 python -u tools/probes/window_probe.py > gpurun_out/window_probe.log 2>&1 || exit $?
cat gpurun_out/window_probe.log | grep -v amdgpu.ids
