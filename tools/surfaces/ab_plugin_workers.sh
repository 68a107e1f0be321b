# A/B of the plugin's classifier threads (BEATRICE_GPU_WORKERS 1 / 2 / 4), surface_bench plugin,
# two alternating repetitions in one call.   bash tools/surfaces/ab_plugin_workers.sh [OUT]
OUT=${1:-gpurun_out/ab_workers}
mkdir -p "$OUT"
for rep in 1 2; do
  for w in 1 2 4; do
    BEATRICE_GPU_WORKERS=$w timeout -k 10 300 tools/surfaces/surface_bench plugin --seconds 1.5 2>/dev/null \
      | sed "s/^{/{\"workers\": $w, \"rep\": $rep, /" >> "$OUT/ab_workers.jsonl" || exit 3
  done
done
