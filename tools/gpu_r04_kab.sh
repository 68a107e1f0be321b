# device-resident A/B of two libbeatrice_gpu.so builds (beatrice_amd/ab/prev against the tree's),
# alternating processes on one box: bench.py's c2f / c2 / c3 / c4 main-kernel times
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04kab}
mkdir -p "$OUT"
bash tools/ab_cmd.sh "$OUT" ${REPS:-3} "prev|BT_LIB_PATH=$PWD/beatrice_amd/ab/prev/libbeatrice_gpu.so|" "cur||" \
  -- python bench.py --configs c2,c3,c4 --no-cpu --group-ingest-packets 0 --steps 20 || exit 1
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    es = [("c2f", d)] + list(d["configs"].items())
    print(d["variant"], d["rep"], " ".join(f"{k} {e['roofline']['kernel_ms']:.4f}" for k, e in es))
PY
