# A/B of bt_opts flag sets on one build, alternating processes on one box:
#   bash tools/gpu_abflags.sh "<configs>" "<flags list>" [reps] [extra bench args]
# e.g. bash tools/gpu_abflags.sh "c2f c3" "0 64 4096 8192" 2
mkdir -p gpurun_out/abf
CFGS=$1; FLS=$2; REPS=${3:-2}; shift 3; EXTRA="$@"
summ() { python3 -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; t=d['timing']
print('%-4s flags=%-6s %9.1f Mpps step %.4f kern %.4f gap/step %.4f' % (sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], r['kernel_ms'], t['gap_ms'] / d['steps']))" $1 $2 $3; }
for cfg in $CFGS; do
  for i in $(seq $REPS); do
    for fl in $FLS; do
      f=gpurun_out/abf/${cfg}_${fl}_$i.json
      timeout -k 10 200 python bench.py --configs none --config $cfg --steps 20 --warmup 3 --no-cpu --flags $fl $EXTRA > $f 2>&1 || { tail -5 $f; exit 3; }
      summ $f $cfg $fl
    done
  done
done
