# Runs surface_bench once per mode given (e.g. "mt plugin parser"), appending every JSON line to
# OUT/surfaces.jsonl; SURF_SECONDS (default 2) per measurement.
#   bash tools/surfaces/run_modes.sh OUT mode...
OUT=$1; shift
mkdir -p "$OUT"
for m in "$@"; do
  timeout -k 10 400 tools/surfaces/surface_bench $m --seconds ${SURF_SECONDS:-2} >> "$OUT/surfaces.jsonl" 2>> "$OUT/surfaces.err" || exit 3
done
