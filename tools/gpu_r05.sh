# Round 5's GPU experiments, one case per call (run through gpurun):
#
#   OUT=gpurun_out/r05/x bash tools/gpu_r05.sh CASE
#
# Cases:
#   c2f_split  where the headline's extra time over parse-only goes: c2 (parse only), c2f
#              and c2f with its filter outputs dropped (--outputs), alternating processes,
#              ROUNDS rounds; then two SQ-counter passes of c2f and c2     
#   ab         AB_LIB (a build under beatrice_amd/ab/) against the in-tree library: first the
#              fixed-stride / full-size parity tests on AB_LIB (AB_TESTS, a -k expression),
#              then tools/gpu_abx.sh over AB_CFGS (default c2f), AB_REPS rounds
#   e2e_outs   host-gather e2e (tools/e2e.py, capture on the device's node) with output arrays
#              allocated once against fresh per call, alternating, E2E_REPS pairs per config
#   fuzz       fresh-seed randomized sweeps sized to the call: FUZZ_SECONDS (S) for the entry-form
#              sweep, S/3 for the PAYLOAD sweep, S for the C++ adapter sweep, each under its own
#              timeout; refuses to start unless S + S/3 + S + 240 s of start-up fits GPURUN_LIMIT
#              (the --timeout given to gpurun for this call)
#   e2e_thp    host-gather and zero-copy e2e with the bound capture on transparent huge pages
#              (--hugepages) against 4-KiB pages, alternating, E2E_REPS pairs per config
#   abn        timing only: the in-tree library and every build named in AB_NAMES
#              (beatrice_amd/ab/<name>/), alternating processes, AB_REPS rounds of AB_CFGS
#   e2e_envab  host-gather e2e (tools/e2e.py --data-node auto, E2E_ARGS appended) with and
#              without AB_ENV, alternating processes, E2E_REPS rounds of E2E_CFGS
#   envab      timing only: the in-tree library with and without AB_ENV (e.g. BT_XCD_ORDER=1),
#              alternating processes, AB_REPS rounds of AB_CFGS, 50 steps each
# Every GPU step runs under its own timeout; the first failure ends the call.
set -o pipefail
OUT=${OUT:-gpurun_out/r05}
mkdir -p "$OUT"
export TMPDIR=/tmp
fail() { echo "step $1 failed (rc $2)"; tail -30 "$3" 2>/dev/null; exit "$2"; }

sq_pass() {   # sq_pass NAME CONFIG COUNTERS...: one rocprofv3 PMC pass of a bench config
  local name=$1 cfg=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/sq_${cfg}_$name" -o run -- \
    python3 bench.py --config $cfg --configs none --steps 5 --warmup 2 --no-cpu > /dev/null 2> "$OUT/sq_${cfg}_$name.err" \
    || fail "sq $cfg $name" $? "$OUT/sq_${cfg}_$name.err"
}

case $1 in
  envab)
    for r in $(seq 1 ${AB_REPS:-3}); do
      for cfg in ${AB_CFGS:-c2f}; do
        for v in base env; do
          e=""; [ $v = env ] && e="${AB_ENV:?AB_ENV=NAME=VALUE}"
          env $e timeout -k 10 150 python3 bench.py --config $cfg --configs none --no-cpu --steps 50 --warmup 5 \
            > "$OUT/envab_${r}_${cfg}_$v.json" 2> "$OUT/envab.err" || fail "envab $cfg $v" $? "$OUT/envab.err"
          python3 - "$OUT/envab_${r}_${cfg}_$v.json" "$cfg $v" "$r" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print(f"round {sys.argv[3]} {sys.argv[2]:10s} kernel {r['kernel_ms']:.4f} ms (min {r['kernel_ms_min']:.4f}) "
      f"step {d['ms_per_step']:.4f} value {d['value']}", flush=True)
PY
        done
      done
    done ;;
  c2f_split)
    for r in $(seq 1 ${ROUNDS:-3}); do
      for v in c2 c2f c2f:records c2f:records,decide c2f:records,verdict; do
        cfg=${v%%:*}; outs=${v#*:}
        extra=""; [ "$outs" != "$v" ] && extra="--outputs $outs"
        timeout -k 10 120 python3 bench.py --config $cfg --configs none --no-cpu --steps 50 --warmup 5 $extra \
          > "$OUT/split_${r}_${v//[:,]/_}.json" 2> "$OUT/split.err" || fail "split $v" $? "$OUT/split.err"
        python3 - "$OUT/split_${r}_${v//[:,]/_}.json" "$v" "$r" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print(f"round {sys.argv[3]} {sys.argv[2]:22s} kernel {r['kernel_ms']:.4f} ms (min {r['kernel_ms_min']:.4f}) "
      f"step {d['ms_per_step']:.4f} frac {r['frac']}", flush=True)
PY
      done
    done
    for cfg in c2f c2; do
      sq_pass a $cfg SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU
      sq_pass b $cfg SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH
      sq_pass g $cfg GRBM_GUI_ACTIVE GRBM_COUNT
    done
    python3 tools/sq_summary.py "$OUT" c2f c2 | tee "$OUT/sq_summary.txt" ;;
  ab)
    L=${AB_LIB:?AB_LIB=beatrice_amd/ab/<name>/libbeatrice_gpu.so}
    BT_LIB_PATH=$PWD/$L timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -m gpu -x -q \
      -p no:cacheprovider --timeout 300 --timeout-method thread -k "${AB_TESTS:-fixed_stride or full_size or tile_groups}" \
      > "$OUT/ab_pytest.log" 2>&1 || fail "ab pytest" $? "$OUT/ab_pytest.log"
    tail -1 "$OUT/ab_pytest.log"
    bash tools/gpu_abx.sh beatrice_amd/libbeatrice_gpu.so $L "${AB_CFGS:-c2f}" ${AB_REPS:-4} --steps 50 \
      | tee "$OUT/ab.txt" || fail ab $? "$OUT/ab.txt" ;;
  abn)
    for r in $(seq 1 ${AB_REPS:-3}); do
      for cfg in ${AB_CFGS:-c2f}; do
        for v in base ${AB_NAMES:?AB_NAMES}; do
          L=$PWD/beatrice_amd/libbeatrice_gpu.so; [ $v != base ] && L=$PWD/beatrice_amd/ab/$v/libbeatrice_gpu.so
          BT_LIB_PATH=$L timeout -k 10 200 python bench.py --configs none --config $cfg --steps 50 --warmup 3 --no-cpu \
            > "$OUT/abn_${cfg}_${v}_$r.json" 2> "$OUT/abn.err" || fail "abn $cfg $v" $? "$OUT/abn.err"
          python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(sys.argv[2], sys.argv[3], sys.argv[4], 'step', d['ms_per_step'], 'kern', r['kernel_ms'], 'frac', r['frac'])" \
            "$OUT/abn_${cfg}_${v}_$r.json" $r $cfg $v | tee -a "$OUT/abn.txt"
        done
      done
    done ;;
  e2e_envab)
    for r in $(seq 1 ${E2E_REPS:-2}); do
      for cfg in ${E2E_CFGS:-c2 c3 c4}; do
        for v in base env; do
          e=""; [ $v = env ] && e="${AB_ENV:?AB_ENV=NAME=VALUE}"
          echo "{\"round\": $r, \"variant\": \"$v\"}" >> "$OUT/e2e_envab.jsonl"
          env $e timeout -k 10 300 python tools/e2e.py --config $cfg --data-node auto --reps 5 ${E2E_ARGS:-} \
            >> "$OUT/e2e_envab.jsonl" 2> "$OUT/e2e_envab.err" || fail "e2e $cfg $v" $? "$OUT/e2e_envab.err"
          tail -1 "$OUT/e2e_envab.jsonl" | cut -c1-160
        done
      done
    done ;;
  e2e_outs)
    for r in $(seq 1 ${E2E_REPS:-2}); do
      for cfg in ${E2E_CFGS:-c2 c3 c4}; do
        for v in once fresh; do
          extra=""; [ $v = fresh ] && extra="--fresh-outputs"
          timeout -k 10 300 python tools/e2e.py --config $cfg --data-node auto --reps 5 $extra \
            >> "$OUT/e2e_outs.jsonl" 2> "$OUT/e2e_outs.err" || fail "e2e $cfg $v" $? "$OUT/e2e_outs.err"
          tail -2 "$OUT/e2e_outs.jsonl" | cut -c1-160
        done
      done
    done ;;
  fuzz)
    S=${FUZZ_SECONDS:-120}; LIMIT=${GPURUN_LIMIT:?GPURUN_LIMIT = the gpurun --timeout of this call}
    need=$(( S + S / 3 + S + 240 ))
    [ $need -le $LIMIT ] || { echo "fuzz: ${need} s of sweeps + start-up exceed the call's ${LIMIT} s"; exit 7; }
    BT_FUZZ_SECONDS=$S BT_FUZZ_SEED=random timeout -k 10 $(( S + S / 3 + 120 )) python -u -m pytest tests/test_gpu_fuzz.py \
      -m gpu -s -q -p no:cacheprovider --timeout $(( S + 120 )) --timeout-method thread > "$OUT/fuzz_gpu.log" 2>&1 \
      || fail "fuzz gpu" $? "$OUT/fuzz_gpu.log"
    grep -iE "rounds|passed|failed" "$OUT/fuzz_gpu.log" | tail -6
    BT_FUZZ_SECONDS=$S BT_FUZZ_SEED=random timeout -k 10 $(( S + 100 )) python -u -m pytest tests/test_cpp_adapter.py \
      -k randomized -m gpu -s -q -p no:cacheprovider --timeout $(( S + 90 )) --timeout-method thread \
      > "$OUT/fuzz_adapter.log" 2>&1 || fail "fuzz adapter" $? "$OUT/fuzz_adapter.log"
    grep -iE "rounds|passed|failed" "$OUT/fuzz_adapter.log" | tail -4 ;;
  e2e_thp)
    for r in $(seq 1 ${E2E_REPS:-2}); do
      for cfg in ${E2E_CFGS:-c2 c3 c4}; do
        for mode in "" "--zero-copy"; do
          for v in thp small; do
            extra=""; [ $v = thp ] && extra="--hugepages"
            timeout -k 10 300 python tools/e2e.py --config $cfg --data-node auto --reps 5 $mode $extra \
              | sed "s/^{/{\"pages\": \"$v\", /" >> "$OUT/e2e_thp.jsonl" 2> "$OUT/e2e_thp.err" || fail "e2e $cfg $v" $? "$OUT/e2e_thp.err"
          done
        done
      done
    done
    tail -4 "$OUT/e2e_thp.jsonl" | cut -c1-120 ;;
  *) echo "unknown case $1"; exit 8 ;;
esac
echo "== done $(date +%T)"
