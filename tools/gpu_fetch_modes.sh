# FETCH_SIZE of the C4 main kernel under the load-mode A/B knobs (bt_opts.flags)
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c4}
for fl in ${FLAGS:-0 1024 2048 128 1025}; do
  timeout -k 10 200 python bench.py --config $CFG --steps 20 --warmup 3 --no-cpu --flags $fl > gpurun_out/fm_$fl.json 2>&1 || exit 3
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/fm_fetch_$fl -o run -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu --flags $fl > /dev/null 2>&1 || exit 4
  python3 - $fl <<'PY'
import csv, glob, json, sys
fl = sys.argv[1]
per = {}
for f in glob.glob(f"gpurun_out/fm_fetch_{fl}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "parse_filter_" in r.get("Kernel_Name", "") and r.get("Counter_Name") == "FETCH_SIZE":
            k = (f, r.get("Dispatch_Id"))
            per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
vals = sorted(per.values())
d = json.loads(open(f"gpurun_out/fm_{fl}.json").read().strip().splitlines()[-1])
n = d["config"]["packets_per_gpu"]
print(f"flags {fl}: kern {d['roofline']['kernel_ms']} ms, read {2 * 1024 * vals[len(vals) // 2] / n:.1f} B/pkt (2 x FETCH, {len(vals)} dispatches)")
PY
done
