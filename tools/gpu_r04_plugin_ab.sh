# A/B of two plugin builds (beatrice_amd/ab/plugin_{base,new}.so), alternating processes on one box:
# surface_bench plugin (C2 / C3, 1 / 8 / 16 producers), with CPU time, faults and cgroup throttling
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04plugin_ab}
mkdir -p "$OUT"
for rep in 1 2; do
  for v in ${VARIANTS:-base new}; do
    BEATRICE_GPU_DEBUG=1 timeout -k 10 300 tools/surfaces/surface_bench plugin --seconds 2 --threads 16 \
      --plugin beatrice_amd/ab/plugin_$v.so >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "$v failed $?"; tail -20 "$OUT/ab.err"; exit 1; }
  done
done
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["plugin"].split("/")[-1], r["config"], r["threads"], round(r["mpps"], 1), "cpu", r["cpu_s"], "sys", r["sys_s"],
          "minflt", r["minflt"], "thr_ms", r["cgroup_throttled_ms"])
PY
