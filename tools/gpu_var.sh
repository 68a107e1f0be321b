summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['value'], 'Mpps step', d['ms_per_step'], 'kern', r['kernel_ms'], 'frac', r['frac'])" $1; }
mkdir -p gpurun_out
for fl in 0 16; do GW=0 FLAGS=$fl timeout -k 10 300 python tools/variance3.py || exit 3; done
for fl in 0 16; do GW=0 FLAGS=$fl timeout -k 10 300 python tools/variance3.py || exit 3; done
for cfg in c2 c3; do for fl in 16 0 16 0; do
timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --flags $fl > gpurun_out/t_${cfg}_$fl.json 2>&1 || exit 3; summ gpurun_out/t_${cfg}_$fl.json; done; done
