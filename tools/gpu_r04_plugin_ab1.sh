# the same A/B at one producer (surface_bench plugin --threads 1 runs it twice per process), 3 pairs
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04plugin_ab1}
mkdir -p "$OUT"
for rep in 1 2 3; do
  for v in ${VARIANTS:-base new}; do
    BEATRICE_GPU_DEBUG=1 timeout -k 10 300 tools/surfaces/surface_bench plugin --seconds 2 --threads 1 \
      --plugin beatrice_amd/ab/plugin_$v.so >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "$v failed $?"; tail -20 "$OUT/ab.err"; exit 1; }
  done
done
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["plugin"].split("/")[-1], r["config"], r["threads"], round(r["mpps"], 1), "cpu", r["cpu_s"], "minflt", r["minflt"])
PY
