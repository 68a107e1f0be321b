# N=1 default bench line + a 2-rank rehearsal of the --gpus 2 path with both ranks on device 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r02
timeout -k 10 400 python3 bench.py > gpurun_out/r02/bench_default.json 2> gpurun_out/r02/bench_default.err || { tail -5 gpurun_out/r02/bench_default.err; exit 3; }
BT_BENCH_DEVICE=0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --no-cpu > gpurun_out/r02/bench_2rank_one_gpu.json 2> gpurun_out/r02/bench_2rank.err || { tail -20 gpurun_out/r02/bench_2rank.err; exit 4; }
python3 - <<'PY'
import json
for f in ("bench_default", "bench_2rank_one_gpu"):
    d = json.loads([l for l in open(f"gpurun_out/r02/{f}.json") if l.startswith("{")][-1])
    print(f, d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["traffic_source"], d["timing"]["wall_over_span"])
    for k, v in d["configs"].items():
        print("  ", k, v["value"], v["ms_per_step"], v["scaling"], v["roofline"]["frac"], v.get("per_rank"))
PY
