# A/B(/C...) of one command under several settings, in alternating processes on one box.
# Every JSON line the command prints is tagged {"variant": <label>, "rep": <r>, ...} and
# appended to OUT/ab.jsonl (stderr to OUT/ab.err).
#   bash tools/ab_cmd.sh OUT REPS "label|ENV=v ...|extra args" ... -- command args...
# e.g. the host pool's scheduling on the host-gather path and the plugin:
#   bash tools/ab_cmd.sh gpurun_out/ab 2 "fixed|BT_POOL_FIXED=1|" "claim||" -- python tools/e2e.py --config c3 --reps 2
#   bash tools/ab_cmd.sh gpurun_out/ab 2 "p8|BT_HOST_THREADS=8|" "p16|BT_HOST_THREADS=16|" -- tools/surfaces/surface_bench mt --seconds 1.5
#   bash tools/ab_cmd.sh gpurun_out/ab 2 "w1|BEATRICE_GPU_WORKERS=1|" "w2||" "w4|BEATRICE_GPU_WORKERS=4|" -- tools/surfaces/surface_bench plugin --seconds 1.5
#   bash tools/ab_cmd.sh gpurun_out/ab 2 "1M||--chunk 1048576" "256k||--chunk 262144" -- python tools/e2e.py --config c2 --reps 2
#   bash tools/ab_cmd.sh gpurun_out/ab 2 "r02|BT_LIB_PATH=$PWD/beatrice_amd/ab/r02/libbeatrice_gpu.so|" "current||" -- python tools/e2e.py --config c3 --reps 2
OUT=$1; REPS=$2; shift 2
V=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done
shift
[ ${#V[@]} -gt 0 ] && [ $# -gt 0 ] || { echo "usage: ab_cmd.sh OUT REPS variant... -- command..."; exit 2; }
mkdir -p "$OUT"
for rep in $(seq "$REPS"); do
  for v in "${V[@]}"; do
    IFS='|' read -r label envs extra <<< "$v"
    env $envs timeout -k 10 300 "$@" $extra 2>> "$OUT/ab.err" | grep '^{' \
      | sed "s/^{/{\"variant\": \"$label\", \"rep\": $rep, /" >> "$OUT/ab.jsonl" || { echo "variant $label failed"; exit 3; }
  done
done
