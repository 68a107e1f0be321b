# c3_payload bench steps of library builds in alternating processes (BT_LIB_PATH):
#   OUT=gpurun_out/x LIBS="main payrow" ROUNDS=2 bash tools/gpu_payload_bench_libs.sh
# LIBS name builds under beatrice_amd/ab/<name>/ (tools/build_ab.sh); "main" = the in-tree library.
set -o pipefail
OUT=${OUT:-gpurun_out/payload_bench_libs}
mkdir -p "$OUT"
for r in $(seq ${ROUNDS:-2}); do
  for lib in $LIBS; do
    L=$PWD/beatrice_amd/ab/$lib/libbeatrice_gpu.so
    [ "$lib" = main ] && L=$PWD/beatrice_amd/libbeatrice_gpu.so
    BT_LIB_PATH=$L timeout -k 10 300 python bench.py --config ${CFG:-c3_payload} --configs none --no-cpu \
      --group-ingest-packets 0 > "$OUT/${lib}_$r.json" 2> "$OUT/${lib}_$r.err" || { tail -20 "$OUT/${lib}_$r.err"; exit 3; }
    python3 tools/summ.py "$OUT/${lib}_$r.json" | grep head | sed "s/^/$lib: /"
  done
done
