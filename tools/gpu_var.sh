summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['value'], 'Mpps step', d['ms_per_step'], 'span', r['gpu_span_ms_per_step'], 'kern', r['kernel_ms'])" $1; }
mkdir -p gpurun_out
for i in 1 2 3 4; do
timeout -k 10 200 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu --grid-waves 4096 > gpurun_out/cp_c3_$i.json 2>&1 || exit 3; summ gpurun_out/cp_c3_$i.json; done
nproc; uptime
