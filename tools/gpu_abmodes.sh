# A/B of bench.py's step-timing modes on one box, alternating processes:
#   default                       pipelined compaction, no per-kernel events in the timed region
#   --no-pipeline                 compaction on the main stream
#   --no-pipeline --kernel-events-in-timed   round 2's first form (events on every main kernel)
#   pipedev: --kernel-events-in-timed (pipelined, events on every main kernel)
#   MODES="piped pipedev" selects a subset
#   bash tools/gpu_abmodes.sh "<configs>" [reps]
mkdir -p gpurun_out/abm
CFGS=${1:-"c2f c3"}; REPS=${2:-2}
summ() { python3 -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; t=d['timing']; k=t['kernel_pass']
print('%-4s %-10s %9.1f Mpps step %.4f kern %.4f | kernel pass: step %.4f gap/step %.4f' % (sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], r['kernel_ms'], k['ms_per_step'], k['gap_ms'] / d['steps']))" $1 $2 $3; }
for cfg in $CFGS; do
  for i in $(seq $REPS); do
    for m in ${MODES:-piped serial events}; do
      case $m in piped) A="";; serial) A="--no-pipeline";; events) A="--no-pipeline --kernel-events-in-timed";;
                 pipedev) A="--kernel-events-in-timed";; esac
      f=gpurun_out/abm/${cfg}_${m}_$i.json
      timeout -k 10 200 python bench.py --configs none --config $cfg --steps 20 --warmup 3 --no-cpu $A > $f 2>&1 || { tail -5 $f; exit 3; }
      summ $f $cfg $m
    done
  done
done
