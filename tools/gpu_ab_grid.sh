# A/B of the persistent grid size (waves) against the default, alternating processes:
# bash tools/gpu_ab_grid.sh "c3 c4" "2048 1536" [PAIRS]
CFGS=${1:-"c3 c4"}; GRIDS=${2:-2048}; PAIRS=${3:-3}
mkdir -p gpurun_out/ab
run() { timeout -k 10 120 python3 bench.py --configs none --no-cpu --steps 20 --warmup 3 --config $c --grid-waves $1 > gpurun_out/ab/last.json 2>&1 || { tail -3 gpurun_out/ab/last.json; exit 3; }; python3 -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/ab/last.json') if l.startswith('{')][-1]); r=d['roofline']
print(sys.argv[1], 'kern', r['kernel_ms'], 'step', d['ms_per_step'])" "grid $1 $c" | tee -a gpurun_out/ab/ab_grid.txt; }
for c in $CFGS; do for rep in $(seq $PAIRS); do
run 0
for g in $GRIDS; do run $g; done
done; done
