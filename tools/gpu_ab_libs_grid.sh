# A/B of several library builds x grid sizes on one config, alternating processes:
#   bash tools/gpu_ab_libs_grid.sh CFG "libA libB ..." "GRIDS" REPS
# (lib = a directory name under beatrice_amd/ab/; GRID 0 = the library's default)
CFG=$1; LIBS=$2; GRIDS=$3; REPS=${4:-2}
mkdir -p gpurun_out/ab
for rep in $(seq $REPS); do for g in $GRIDS; do for L in $LIBS; do
  BT_LIB_PATH=$PWD/beatrice_amd/ab/$L/libbeatrice_gpu.so timeout -k 10 120 python3 bench.py --configs none --no-cpu --steps 20 --warmup 3 --config $CFG --grid-waves $g > gpurun_out/ab/last.json 2>&1 || { tail -5 gpurun_out/ab/last.json; exit 3; }
  python3 -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/ab/last.json') if l.startswith('{')][-1]); r=d['roofline']
print(sys.argv[1], 'kern', r['kernel_ms'], 'step', d['ms_per_step'], 'mpps', d['value'])" "$CFG grid $g $L" | tee -a gpurun_out/ab/ab_libs_grid.txt
done; done; done
