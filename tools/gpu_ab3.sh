mkdir -p gpurun_out
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['value'], 'Mpps step', d['ms_per_step'], 'kern', r['kernel_ms'], 'ms frac', r['frac'])" $1; }
for i in 1 2 3; do
  BT_LIB_PATH=$PWD/tools/calib/libbeatrice_gpu_r01a.so timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu --grid-waves 8192 > gpurun_out/old_$i.json 2>&1 || exit 3
  summ gpurun_out/old_$i.json
  timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu --grid-waves 8192 > gpurun_out/new_$i.json 2>&1 || exit 3
  summ gpurun_out/new_$i.json
done
timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu --grid-waves 8192 --packets 4194304 > gpurun_out/new_4m.json 2>&1 && summ gpurun_out/new_4m.json
rocm-smi --showclocks --showpower 2>&1 | head -30 > gpurun_out/smi.txt; grep -E 'sclk|mclk|Power' gpurun_out/smi.txt | head
