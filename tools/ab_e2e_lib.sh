# Same-box A/B of the host-gather end-to-end path against another build of the library
# (BT_LIB_PATH, e.g. round 2's in beatrice_amd/ab/r02), alternating, C3 and C4:
#   bash tools/ab_e2e_lib.sh OUT beatrice_amd/ab/r02/libbeatrice_gpu.so
OUT=${1:-gpurun_out/ab_e2e_lib}; OTHER=$2
mkdir -p "$OUT"
for rep in 1 2; do
  for which in other current; do
    for cfg in c3 c4; do
      if [ $which = other ]; then
        BT_LIB_PATH=$PWD/$OTHER timeout -k 10 300 python tools/e2e.py --config $cfg --reps 2 \
          | sed "s/^{/{\"lib\": \"$which\", \"rep\": $rep, /" >> "$OUT/e2e.jsonl" || exit 3
      else
        timeout -k 10 300 python tools/e2e.py --config $cfg --reps 2 \
          | sed "s/^{/{\"lib\": \"$which\", \"rep\": $rep, /" >> "$OUT/e2e.jsonl" || exit 3
      fi
    done
  done
done
