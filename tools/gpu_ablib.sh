# A/B of an alternative library build (tools/build_ab.sh NAME ...) against the tree's own,
# alternating processes: bash tools/gpu_ablib.sh NAME "c3 c4" [PAIRS] ["extra bench args"]
NAME=$1; CFGS=${2:-"c3 c4"}; PAIRS=${3:-3}; EXTRA=${4:-}
mkdir -p gpurun_out/ab
run() { timeout -k 10 120 env "$@" > gpurun_out/ab/last.json 2>&1 || { tail -3 gpurun_out/ab/last.json; exit 3; }; python3 -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/ab/last.json') if l.startswith('{')][-1]); r=d['roofline']
print(sys.argv[1], 'kern', r['kernel_ms'], 'step', d['ms_per_step'])" "$TAG $c" | tee -a gpurun_out/ab/ablib_$NAME.txt; }
for c in $CFGS; do for rep in $(seq $PAIRS); do
TAG=base run X=1 python3 bench.py --configs none --no-cpu --steps 20 --warmup 3 --config $c $EXTRA
TAG=$NAME run BT_LIB_PATH=beatrice_amd/ab/$NAME/libbeatrice_gpu.so python3 bench.py --configs none --no-cpu --steps 20 --warmup 3 --config $c $EXTRA
done; done
