# round 4: C4's main kernel next to the pure data-movement kernels with its access pattern
# (tools/calib/gather_c4: one round / two dependent rounds), alternating, on one box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 tools/calib/gather_c4 > $O/gather_c4_$rep.txt 2>&1 || { cat $O/gather_c4_$rep.txt; exit 3; }
  cat $O/gather_c4_$rep.txt
  timeout -k 10 200 python3 bench.py --configs none --no-cpu --steps 20 --warmup 3 --config c4 > $O/c4_$rep.json 2>&1 || exit 3
  python3 -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']
print('rep', sys.argv[2], 'c4 kern', r['kernel_ms'], 'step', d['ms_per_step'], 'traffic', r.get('traffic'), 'floor', r.get('traffic_floor'))" $O/c4_$rep.json $rep
done
echo ALL-DONE
