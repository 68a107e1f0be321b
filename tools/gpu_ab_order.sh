# A/B: cyclic vs blocked tile order (alternating processes, 3 pairs per config)
mkdir -p gpurun_out/ab
run() { timeout -k 10 120 "$@" > gpurun_out/ab/last.json 2>&1 || exit 3; python3 -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/ab/last.json') if l.startswith('{')][-1]); r=d['roofline']
print(sys.argv[1][50:], 'kern', r['kernel_ms'], 'step', d['ms_per_step'], 'gap', d['timing']['gap_ms'])" "$*" | tee -a gpurun_out/ab/order.txt; }
for c in c2f c3 c4; do for rep in 1 2 3; do
run python3 bench.py --configs none --no-cpu --steps 20 --warmup 3 --config $c
run python3 bench.py --configs none --no-cpu --steps 20 --warmup 3 --config $c --flags 2
done; done
