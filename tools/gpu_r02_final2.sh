# Round-2 closing evidence, part 2 (after part 1's traffic.json is committed): the default
# bench line, the 2-rank rehearsal on one device, the end-to-end table.
OUT=gpurun_out/r02/final
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 3; }
python3 -c "
import json; d=json.loads([l for l in open('$OUT/bench_default.json') if l.startswith('{')][-1])
print('head', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['traffic_bytes_per_packet'])
for k,c in d['configs'].items(): print(k, c['value'], c['ms_per_step'], c['roofline']['kernel_ms'], c['roofline']['frac'], c['roofline'].get('traffic_bytes_per_packet'), (c.get('cpu_baseline') or {}).get('value'))"
BT_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --cpu-seconds 2 > $OUT/bench_2rank_one_gpu.json 2> $OUT/bench_2rank.err || { tail $OUT/bench_2rank.err; exit 4; }
tail -c 300 $OUT/bench_2rank_one_gpu.json
rm -f gpurun_out/e2e.jsonl
bash tools/gpu_e2e.sh > $OUT/e2e.txt 2>&1 || { tail -5 $OUT/e2e.txt; exit 5; }
cp gpurun_out/e2e.jsonl $OUT/e2e.jsonl
tail -9 $OUT/e2e.txt
