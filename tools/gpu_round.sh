# One parameterized GPU-box script for the round's evidence (run through gpurun):
#
#   OUT=gpurun_out/r03/x STEPS="tests bounds smoke bench" bash tools/gpu_round.sh
#
# Steps (in the order given; the first failure ends the call — nothing runs after a GPU
# failure):
#   tests   python -m pytest tests -m gpu (release library)         -> $OUT/pytest_gpu.log
#   bounds  the same suite on the BT_DEBUG_BOUNDS build (beatrice_amd/dbg, make -C
#           beatrice_amd/csrc debug): every kernel access checked   -> $OUT/pytest_bounds.log
#   smoke   __graft_entry__.smoke()                                   -> $OUT/smoke.log
#   bench   the default `python bench.py` line                       -> $OUT/bench_default.json
#   multi   2- and 4-rank rehearsals on the one device (bench.py --gpus N spawning its
#           ranks, BT_BENCH_DEVICE=0)                                -> $OUT/bench_{2,4}rank_one_gpu.json
#   prof    rocprofv3 kernel stats + PMC traffic (tools/gpu_prof.sh) -> $OUT/prof/
#   sq      SQ counters of the main kernels (tools/gpu_sq.sh)        -> $OUT/sq.txt
#   e2e     end-to-end (PCIe) table (tools/e2e.py)                   -> $OUT/e2e.jsonl
#   surfaces  the drop-in C++ surfaces timed next to the reference  -> $OUT/surfaces.json
#             (SURF_ARGS: surface_bench arguments, default "all")
# CFGS (default "c2f c2 c3 c4 c1") selects the configs of prof / sq.
set -o pipefail
OUT=${OUT:-gpurun_out/round}
STEPS=${STEPS:-"tests smoke bench"}
CFGS=${CFGS:-"c2f c2 c3 c4 c1"}
mkdir -p "$OUT"
export TMPDIR=/tmp
PYTEST="python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
fail() { echo "step $1 failed (rc $2)"; tail -40 "$3" 2>/dev/null; exit "$2"; }
for step in $STEPS; do
  echo "== $step $(date +%T)"
  case $step in
    tests)
      timeout -k 10 900 $PYTEST > "$OUT/pytest_gpu.log" 2>&1 || fail tests $? "$OUT/pytest_gpu.log"
      tail -2 "$OUT/pytest_gpu.log" ;;
    bounds)
      [ -f beatrice_amd/dbg/libbeatrice_gpu.so ] || { echo "no bounds build (make -C beatrice_amd/csrc debug)"; exit 9; }
      BT_LIB_PATH=$PWD/beatrice_amd/dbg/libbeatrice_gpu.so LD_LIBRARY_PATH=$PWD/beatrice_amd/dbg:$LD_LIBRARY_PATH \
        timeout -k 10 1200 $PYTEST > "$OUT/pytest_bounds.log" 2>&1 || fail bounds $? "$OUT/pytest_bounds.log"
      grep -c "BT_DEBUG_BOUNDS" "$OUT/pytest_bounds.log" | sed 's/^/bounds reports: /'
      tail -2 "$OUT/pytest_bounds.log" ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || fail smoke $? "$OUT/smoke.log"
      tail -1 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 600 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || fail bench $? "$OUT/bench_default.err"
      python3 tools/summ.py "$OUT/bench_default.json" ;;
    multi)
      for n in 2 4; do
        BT_BENCH_DEVICE=0 timeout -k 10 600 python bench.py --gpus $n \
          > "$OUT/bench_${n}rank_one_gpu.json" 2> "$OUT/bench_${n}rank.err" || fail multi$n $? "$OUT/bench_${n}rank.err"
        python3 tools/summ.py "$OUT/bench_${n}rank_one_gpu.json"
      done ;;
    prof)
      bash tools/gpu_prof.sh "$OUT/prof" $CFGS || fail prof $? /dev/null ;;
    sq)
      CFGS="$CFGS" bash tools/gpu_sq.sh > "$OUT/sq.txt" 2>&1 || fail sq $? "$OUT/sq.txt"
      cat "$OUT/sq.txt" ;;
    e2e)
      rm -f "$OUT/e2e.jsonl"
      # E2E_MODES: ';'-separated e2e.py option sets (default: host gather, zero-copy, ring)
      IFS=';' read -r -a modes <<< "${E2E_MODES:- ;--zero-copy;--tpacket}"
      for cfg in ${E2E_CFGS:-c2 c3 c4}; do
        for mode in "${modes[@]}"; do
          timeout -k 10 400 python tools/e2e.py --config $cfg $mode --reps 2 >> "$OUT/e2e.jsonl" 2> "$OUT/e2e.err" \
            || fail "e2e $cfg $mode" $? "$OUT/e2e.err"
        done
      done
      cat "$OUT/e2e.jsonl" ;;
    surfaces)
      timeout -k 10 900 tools/surfaces/surface_bench ${SURF_ARGS:-all} > "$OUT/surfaces.json" 2> "$OUT/surfaces.err" || fail surfaces $? "$OUT/surfaces.err"
      cat "$OUT/surfaces.json" ;;
    *) echo "unknown step $step"; exit 8 ;;
  esac
done
echo "== done $(date +%T)"
