# Round-2 closing evidence after the pipelined compaction (part 2, extractor grid 4 blocks/CU): the default bench line
# (the driver's command) and the 2- and 4-rank rehearsals of the --gpus N path on one device.
OUT=gpurun_out/r02/final9
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 3; }
BT_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --cpu-seconds 2 > $OUT/bench_2rank_one_gpu.json 2> $OUT/bench_2rank.err || { tail $OUT/bench_2rank.err; exit 4; }
BT_BENCH_DEVICE=0 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --cpu-seconds 2 > $OUT/bench_4rank_one_gpu.json 2> $OUT/bench_4rank.err || { tail $OUT/bench_4rank.err; exit 5; }
python3 - <<'PY'
import json
for f in ("bench_default", "bench_2rank_one_gpu", "bench_4rank_one_gpu"):
    d = json.loads([l for l in open(f"gpurun_out/r02/final9/{f}.json") if l.startswith("{")][-1])
    print(f, d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d["roofline"]["traffic_source"], d["timing"]["wall_over_span"], (d.get("cpu_baseline") or {}).get("value"))
    for k, v in d["configs"].items():
        print("  ", k, v["value"], v["ms_per_step"], v["scaling"], v["roofline"]["kernel_ms"], v["roofline"]["frac"], v["roofline"].get("traffic_bytes_per_packet"), (v.get("cpu_baseline") or {}).get("value"))
PY
