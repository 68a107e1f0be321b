# Host-gather end-to-end path (tools/e2e.py default mode) by staging chunk size, C2 and C3
# verdicts, alternating: bash tools/e2e_chunk_ab.sh OUT
OUT=${1:-gpurun_out/e2e_chunk}
mkdir -p "$OUT"
for rep in 1 2; do
  for cfg in c2 c3; do
    for ch in 1048576 262144 131072; do
      timeout -k 10 300 python tools/e2e.py --config $cfg --chunk $ch --reps 2 \
        | sed "s/^{/{\"chunk_ab\": $ch, \"rep\": $rep, /" >> "$OUT/e2e_chunk.jsonl" || exit 3
    done
  done
done
