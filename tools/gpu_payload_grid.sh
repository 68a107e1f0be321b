# c3_payload bench steps under BT_PAYLOAD_GRID settings (blocks per CU for PAYLOAD programs;
# 0 = residency, -1 = one block per 4 tiles), alternating processes:
#   OUT=gpurun_out/x GRIDS="0 3 -1" ROUNDS=2 bash tools/gpu_payload_grid.sh
set -o pipefail
OUT=${OUT:-gpurun_out/payload_grid}
mkdir -p "$OUT"
for r in $(seq ${ROUNDS:-2}); do
  for g in ${GRIDS:-0 3 -1}; do
    BT_PAYLOAD_GRID=$g timeout -k 10 300 python bench.py --config c3_payload --configs none --no-cpu \
      --group-ingest-packets 0 > "$OUT/grid_${g}_$r.json" 2> "$OUT/grid_${g}_$r.err" || { tail -20 "$OUT/grid_${g}_$r.err"; exit 3; }
    python3 tools/summ.py "$OUT/grid_${g}_$r.json" | grep head | sed "s/^/grid $g: /"
  done
done
