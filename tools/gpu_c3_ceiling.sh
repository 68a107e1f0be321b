# C3's main kernel next to the pure data-movement kernel with its access pattern
# (tools/calib/gather_mix), alternating, on one box: bash tools/gpu_c3_ceiling.sh [REPS]
REPS=${1:-3}
mkdir -p gpurun_out/ceil
for rep in $(seq $REPS); do
  timeout -k 10 120 tools/calib/gather_mix > gpurun_out/ceil/gather_$rep.txt 2>&1 || exit 3
  grep -E 'blocks/CU' gpurun_out/ceil/gather_$rep.txt | sed "s/^/rep $rep /"
  timeout -k 10 120 python3 bench.py --configs none --no-cpu --steps 20 --warmup 3 --config c3 > gpurun_out/ceil/c3_$rep.json 2>&1 || exit 3
  python3 -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']
print('rep', sys.argv[2], 'c3 kern', r['kernel_ms'], 'step', d['ms_per_step'], 'traffic', r.get('traffic'), 'floor', r.get('traffic_floor'))" gpurun_out/ceil/c3_$rep.json $rep
done
