# Sweep of the fixed-stride kernel's knobs (c2f / c2): prefetch on/off, nt header loads,
# grid (auto = residency, 2048 waves = 2 blocks/CU), alternating in one box.
#   bash tools/gpu_sweep_fixed.sh "<configs>" [reps]
mkdir -p gpurun_out/sweep
CFGS=${1:-"c2f c2"}; REPS=${2:-2}
summ() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print('%-5s %-22s %9.1f Mpps step %.4f kern %.4f' % (sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], r['kernel_ms']))" $1 $2 $3; }
for cfg in $CFGS; do
  for i in $(seq $REPS); do
    for gw in 0 2048; do
      for fl in 0 1 64 65; do
        f=gpurun_out/sweep/${cfg}_${gw}_${fl}_$i.json
        timeout -k 10 200 python bench.py --configs none --config $cfg --steps 20 --warmup 3 --no-cpu --grid-waves $gw --flags $fl > $f 2>&1 || { tail -5 $f; exit 3; }
        summ $f $cfg "gw=$gw flags=$fl"
      done
    done
  done
done
