# the plugin's time budget at 1 / 8 / 16 producers (BEATRICE_GPU_DEBUG: where the classifier
# threads' time went), 2 and 4 classifier threads, one box
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04plugin}
mkdir -p "$OUT"
for w in 2 4; do
  BEATRICE_GPU_DEBUG=1 BEATRICE_GPU_WORKERS=$w timeout -k 10 300 tools/surfaces/surface_bench plugin --seconds 2 --threads 16 \
    > "$OUT/plugin_w$w.jsonl" 2> "$OUT/plugin_w$w.err" || { echo "w$w failed $?"; tail -20 "$OUT/plugin_w$w.err"; exit 1; }
  cat "$OUT/plugin_w$w.jsonl"; grep gpu_parse_filter "$OUT/plugin_w$w.err"
done
