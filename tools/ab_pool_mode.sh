# A/B of the host pool's scheduling (BT_POOL_FIXED=1: round 2's fixed index per worker, the
# caller waits for every worker; unset: claimed indices) on the host-gather end-to-end path
# (C2 / C3) and the plugin, alternating.   bash tools/ab_pool_mode.sh OUT
OUT=${1:-gpurun_out/ab_pool_mode}
mkdir -p "$OUT"
for rep in 1 2; do
  for mode in fixed claim; do
    if [ $mode = fixed ]; then export BT_POOL_FIXED=1; else unset BT_POOL_FIXED; fi
    for cfg in c2 c3; do
      timeout -k 10 300 python tools/e2e.py --config $cfg --reps 2 \
        | sed "s/^{/{\"pool\": \"$mode\", \"rep\": $rep, /" >> "$OUT/e2e.jsonl" || exit 3
    done
    timeout -k 10 300 tools/surfaces/surface_bench plugin --seconds 1.5 2>/dev/null \
      | sed "s/^{/{\"pool\": \"$mode\", \"rep\": $rep, /" >> "$OUT/plugin.jsonl" || exit 3
  done
done
