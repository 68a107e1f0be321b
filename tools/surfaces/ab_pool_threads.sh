# A/B of the context's host pool size (BT_HOST_THREADS 8 vs 16) on the surfaces that share
# the host with their callers: 16 callers of one GpuPacketFilter (surface_bench mt) and the
# plugin fed from 1 and 16 onPacket threads, two alternating repetitions in one call.
#   bash tools/surfaces/ab_pool_threads.sh [OUT]
OUT=${1:-gpurun_out/r03b/v6}
mkdir -p "$OUT"
for rep in 1 2; do
  for t in 8 16; do
    for m in mt plugin; do
      BT_HOST_THREADS=$t timeout -k 10 300 tools/surfaces/surface_bench $m --seconds 1.5 2>/dev/null \
        | sed "s/^{/{\"pool\": $t, \"rep\": $rep, /" >> "$OUT/ab_threads.jsonl" || exit 3
    done
  done
done
