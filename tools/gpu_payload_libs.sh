# PAYLOAD A/B of library builds in alternating processes on one box (tools/payload_ab.py per
# build, BT_LIB_PATH):
#   OUT=gpurun_out/x LIBS="base bytes" VARIANTS=first,caret_x ROUNDS=2 bash tools/gpu_payload_libs.sh
# LIBS name builds under beatrice_amd/ab/<name>/ (tools/build_ab.sh); "main" = the in-tree library.
set -o pipefail
OUT=${OUT:-gpurun_out/payload_libs}
mkdir -p "$OUT"
for r in $(seq ${ROUNDS:-2}); do
  for lib in $LIBS; do
    L=$PWD/beatrice_amd/ab/$lib/libbeatrice_gpu.so
    [ "$lib" = main ] && L=$PWD/beatrice_amd/libbeatrice_gpu.so
    echo "== round $r $lib $(date +%T)"
    # lib@G: the build with BT_PAYLOAD_GRID=G
    G=""; case $lib in *@*) G=${lib#*@}; L=${L%/*}; L=$PWD/beatrice_amd/$( [ "${lib%@*}" = main ] && echo "" || echo "ab/${lib%@*}/")libbeatrice_gpu.so;; esac
    BT_PAYLOAD_GRID=$G BT_LIB_PATH=$L timeout -k 10 300 python tools/payload_ab.py --variants ${VARIANTS:-first,caret_x} \
      --rounds ${AB_ROUNDS:-2} > "$OUT/${lib}_$r.jsonl" 2> "$OUT/${lib}_$r.err" || { tail -20 "$OUT/${lib}_$r.err"; exit 3; }
    python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['variant'], 'rec' if d['records'] else 'flt', d['kernel_ms_median'], d.get('decisions_equal_to_dfa_form'))
" "$OUT/${lib}_$r.jsonl" $lib
  done
done
