# A/B for the headline c2f kernel: which outputs / tile order cost what.
mkdir -p gpurun_out/ab
run() { timeout -k 10 120 env "$@" > gpurun_out/ab/last.json 2>&1 || exit 3; python3 -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/ab/last.json') if l.startswith('{')][-1]); r=d['roofline']
print(sys.argv[1][60:], 'kern', r['kernel_ms'], 'step', d['ms_per_step'])" "$*" | tee -a gpurun_out/ab/summary3.txt; }
B="python3 bench.py --configs none --no-cpu --steps 20 --warmup 3 --config c2f"
for rep in 1 2; do
run X=1 $B
run X=1 $B --outputs records,decide,verdict
run X=1 $B --outputs records,verdict,pass_idx
run X=1 $B --outputs records,verdict
run X=1 $B --outputs decide,verdict,pass_idx
run X=1 $B --flags 2
run X=1 $B --flags 2 --grid-waves 2048
done
