summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['value'], 'Mpps step', d['ms_per_step'], 'span', r['gpu_span_ms_per_step'], 'kern', r['kernel_ms'])" $1; }
mkdir -p gpurun_out
export BT_DEBUG_TIMING=1
for cfg in c3 c3 c3 c4 c4 c2; do
timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu > gpurun_out/dbg.json 2> gpurun_out/dbg.err || exit 3; summ gpurun_out/dbg.json; grep -E '^\[' gpurun_out/dbg.err | tail -3; done
