# A/B of one build under two environment settings, alternating processes on one box:
#   bash tools/gpu_abenv.sh "<envA>" "<envB>" "<configs>" [reps] [extra bench args]
# e.g. bash tools/gpu_abenv.sh "BT_NO_PIPE=1" "BT_NO_PIPE=0" "c3 c4" 3
mkdir -p gpurun_out
EA=$1; EB=$2; CFGS=$3; REPS=${4:-3}; shift 4; EXTRA="$@"
summ() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(sys.argv[2], sys.argv[3], d['value'], 'Mpps step', d['ms_per_step'], 'kern', r['kernel_ms'])" $1 $2 $3; }
for cfg in $CFGS; do
  for i in $(seq $REPS); do
    for v in A B; do
      E=$EA; [ $v = B ] && E=$EB
      env $E timeout -k 10 200 python bench.py --configs none --config $cfg --steps 20 --warmup 3 --no-cpu $EXTRA > gpurun_out/abe_${cfg}_${v}_$i.json 2>&1 || { tail -5 gpurun_out/abe_${cfg}_${v}_$i.json; exit 3; }
      summ gpurun_out/abe_${cfg}_${v}_$i.json $cfg $v
    done
  done
done
