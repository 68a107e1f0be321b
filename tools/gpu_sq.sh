# SQ counters of the main kernel (one 8-counter pass per config): where wave time goes.
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in ${CFGS:-c2 c3}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/sq_$c -o run -- python3 bench.py --config $c --configs none --steps 3 --warmup 1 --no-cpu > /dev/null 2>&1 || exit 4
  python3 - $c <<'PY'
import csv, glob, sys
c = sys.argv[1]
per = {}
for f in glob.glob(f"gpurun_out/sq_{c}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "parse_filter_" in r.get("Kernel_Name", "") or "extract_tile" in r.get("Kernel_Name", ""):
            per.setdefault(r["Dispatch_Id"], {}).setdefault(r["Counter_Name"], 0.0)
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
d = per[sorted(per, key=int)[-1]]
wc = d["SQ_WAVE_CYCLES"]
print(c, {k: round(v / 1e6, 2) for k, v in sorted(d.items())}, "(millions)")
print(c, "wait_any %.2f  wait_inst %.2f  active %.2f of wave cycles; VALU insts per packet %.1f" % (
    d["SQ_WAIT_ANY"] / wc, d["SQ_WAIT_INST_ANY"] / wc, d["SQ_ACTIVE_INST_ANY"] / wc, d["SQ_INSTS_VALU"] / (1 << 24)))
PY
done
