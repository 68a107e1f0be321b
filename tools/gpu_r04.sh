# Round 4's experiments and closing evidence, one case per gpurun call (each on one box, A/Bs in
# alternating processes through tools/ab_cmd.sh):
#   bash tools/gpu_r04.sh CASE [OUT]      (OUT defaults to gpurun_out/r04-CASE)
# Cases and the DESIGN.md section each feeds:
#   e2e-closing    every e2e path, C2 / C3 / C4: host gather, zero-copy, ring in place / packed,
#                  groups of 2 / 4 on the shared device, the sparse-frame option (§6, §7)
#   surf-closing   every drop-in C++ surface, then rocprofv3 stats + PMC traffic (§6)
#   group-e2e      the group rows alone, 1 / 2 / 4 members (§7)
#   numa-ab        host-gather pool pinned to the device's node or not, C2 / C3 / C4 (§7)
#   serial-ab      shared-device members concurrent or serialised (zero-copy group) (§7)
#   group1-ab      host gather through one context against a group of one (§7)
#   c4-ceiling     C4's kernel next to tools/calib/gather_c4 (one / two dependent rounds) (§4.1, §6)
#   plugin-hot     the plugin fed hot frames, BEATRICE_GPU_PACK off / on (§6)
#   plugin-budget  the plugin's classifier time (BEATRICE_GPU_DEBUG), 2 and 4 classifier threads (§6)
#   plugin-ab      two plugin builds (beatrice_amd/ab/plugin_{base,new}.so; VARIANTS) (§6)
#   gather-nt-ab   host gather with plain / non-temporal staging stores (§6)
#   drain-nt-ab    the record drain with memcpy / non-temporal stores (§6)
#   lean-ab        GPU suite with the narrow lean round, then its e2e A/B (§9.2)
#   kernel-ab      device-resident A/B of beatrice_amd/ab/prev against the tree's library (§6)
#   route-ab       group tests, then concurrent callers routed whole / always split (§7)
#   single         single-packet and small-batch surfaces (§6)
#   pool-ab        the context's host pool at 8 (BT_HOST_THREADS=8, round 3's default) / the
#                  default (the usable CPUs, a share of 8 while other callers wait): host-gather e2e
#                  with the capture on the device's node, the plugin, one- and 16-caller classify (§6)
#   data-node-ab   host gather / zero-copy with the capture where its generator left it or moved
#                  onto the device's NUMA node (e2e.py --data-node auto) (§6)
set -o pipefail
export TMPDIR=/tmp
CASE=$1
OUT=${2:-gpurun_out/r04-$CASE}
mkdir -p "$OUT"
PYTEST="python -u -m pytest -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread"
summ_ab() {   # variant, rep, config, mode, Mpps of every JSON line of an ab.jsonl
  python3 - "$1" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    extra = {k: r[k] for k in ("members", "threads", "cpu_s", "cgroup_throttled_ms") if k in r}
    print(r["variant"], r["rep"], r.get("config"), r.get("mode", r.get("surface", ""))[:60], r.get("mpps"), extra)
PY
}
case $CASE in
  e2e-closing)
    OUT=$OUT STEPS="e2e" E2E_CFGS="c2 c3 c4" \
      E2E_MODES=" ;--zero-copy;--tpacket;--tpacket --gather --dense --mix 2;--group 2;--group 4;--group 1 --flags 0x10000" \
      bash tools/gpu_round.sh ;;
  surf-closing)
    OUT=$OUT STEPS="surfaces" SURF_ARGS="all --seconds 2" bash tools/gpu_round.sh || exit 1
    OUT=$OUT STEPS="prof" bash tools/gpu_round.sh ;;
  group-e2e)
    OUT=$OUT STEPS="e2e" E2E_CFGS="c2 c3 c4" E2E_MODES="--group 1;--group 2;--group 4" bash tools/gpu_round.sh ;;
  numa-ab)
    for cfg in c2 c3 c4; do
      bash tools/ab_cmd.sh "$OUT" 2 "pin||" "nopin|BT_NUMA_PIN=0|" -- python tools/e2e.py --config $cfg --reps 2 || exit 1
    done
    summ_ab "$OUT/ab.jsonl" ;;
  serial-ab)
    bash tools/ab_cmd.sh "$OUT" 2 "concurrent||" "serial|BT_GROUP_SHARED_SERIAL=1|" -- python tools/e2e.py --config c2 --group 2 --reps 2 \
      && summ_ab "$OUT/ab.jsonl" ;;
  group1-ab)
    for cfg in c2 c3; do
      bash tools/ab_cmd.sh "$OUT" 2 "single||" "group1||--group 1" -- python tools/e2e.py --config $cfg --reps 2 || exit 1
    done
    summ_ab "$OUT/ab.jsonl" ;;
  c4-ceiling)
    for rep in 1 2; do
      timeout -k 10 300 tools/calib/gather_c4 > "$OUT/gather_c4_$rep.txt" 2>&1 || { cat "$OUT/gather_c4_$rep.txt"; exit 3; }
      cat "$OUT/gather_c4_$rep.txt"
      timeout -k 10 200 python3 bench.py --configs none --no-cpu --steps 20 --warmup 3 --config c4 > "$OUT/c4_$rep.json" 2>&1 || exit 3
      python3 tools/summ.py "$OUT/c4_$rep.json"
    done ;;
  plugin-hot)
    bash tools/ab_cmd.sh "$OUT" 2 "pack0|BEATRICE_GPU_PACK=0|" "pack1|BEATRICE_GPU_PACK=1|" -- tools/surfaces/surface_bench plugin-hot --seconds 2 \
      && summ_ab "$OUT/ab.jsonl" ;;
  plugin-budget)
    for w in 2 4; do
      BEATRICE_GPU_DEBUG=1 BEATRICE_GPU_WORKERS=$w timeout -k 10 300 tools/surfaces/surface_bench plugin --seconds 2 --threads 16 \
        > "$OUT/plugin_w$w.jsonl" 2> "$OUT/plugin_w$w.err" || { tail -20 "$OUT/plugin_w$w.err"; exit 1; }
      cat "$OUT/plugin_w$w.jsonl"; grep gpu_parse_filter "$OUT/plugin_w$w.err"
    done ;;
  plugin-ab)
    V=()
    for v in ${VARIANTS:-base new}; do V+=("$v||--plugin beatrice_amd/ab/plugin_$v.so"); done
    BEATRICE_GPU_DEBUG=1 bash tools/ab_cmd.sh "$OUT" ${REPS:-2} "${V[@]}" -- tools/surfaces/surface_bench plugin --seconds 2 --threads ${THREADS:-16} \
      && summ_ab "$OUT/ab.jsonl" ;;
  gather-nt-ab)
    for cfg in ${CFGS:-c2 c3 c4}; do
      bash tools/ab_cmd.sh "$OUT" ${REPS:-2} "plain|BT_GATHER_NT=0|" "nt|BT_GATHER_NT=1|" -- python tools/e2e.py --config $cfg --reps 3 || exit 1
    done
    summ_ab "$OUT/ab.jsonl" ;;
  drain-nt-ab)
    for cfg in ${CFGS:-c2 c3 c4}; do
      bash tools/ab_cmd.sh "$OUT" ${REPS:-3} "memcpy|BT_DRAIN_NT=0|" "nt|BT_DRAIN_NT=1|" -- python tools/e2e.py --config $cfg --reps 3 || exit 1
    done
    summ_ab "$OUT/ab.jsonl" ;;
  lean-ab)
    BT_LEAN_LO=12 BT_LEAN_END=38 timeout -k 10 600 $PYTEST tests > "$OUT/pytest_lean12_38.log" 2>&1 || { tail -30 "$OUT/pytest_lean12_38.log"; exit 1; }
    tail -2 "$OUT/pytest_lean12_38.log"
    for cfg in c2 c3 c4; do
      for mode in --zero-copy --tpacket; do
        bash tools/ab_cmd.sh "$OUT" 2 "lo0|BT_LEAN_LO=0 BT_LEAN_END=46|" "lo12|BT_LEAN_LO=12 BT_LEAN_END=46|" "lo12e38|BT_LEAN_LO=12 BT_LEAN_END=38|" \
          -- python tools/e2e.py --config $cfg $mode --reps 3 || exit 1
      done
    done
    summ_ab "$OUT/ab.jsonl" ;;
  kernel-ab)
    bash tools/ab_cmd.sh "$OUT" ${REPS:-3} "prev|BT_LIB_PATH=$PWD/beatrice_amd/ab/prev/libbeatrice_gpu.so|" "cur||" \
      -- python bench.py --configs c2,c3,c4 --no-cpu --group-ingest-packets 0 --steps 20 || exit 1
    python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    es = [("c2f", d)] + list(d["configs"].items())
    print(d["variant"], d["rep"], " ".join(f"{k} {e['roofline']['kernel_ms']:.4f}" for k, e in es))
PY
    ;;
  route-ab)
    timeout -k 10 400 $PYTEST tests/test_gpu_group.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
    tail -2 "$OUT/pytest.log"
    bash tools/ab_cmd.sh "$OUT" 2 "split|BT_GROUP_ROUTE_BELOW=0|" "routed||" -- tools/surfaces/surface_bench group --seconds 2 \
      && summ_ab "$OUT/ab.jsonl" ;;
  single)
    timeout -k 10 400 tools/surfaces/surface_bench single --seconds 1.5 > "$OUT/surf_single.jsonl" 2> "$OUT/surf_single.err" \
      || { tail "$OUT/surf_single.err"; exit 1; }
    cat "$OUT/surf_single.jsonl" ;;
  pool-ab)
    for cfg in c2 c3 c4; do
      bash tools/ab_cmd.sh "$OUT" 2 "p8|BT_HOST_THREADS=8|" "auto||" -- python tools/e2e.py --config $cfg --reps 3 --data-node auto || exit 1
    done
    bash tools/ab_cmd.sh "$OUT" 2 "p8|BT_HOST_THREADS=8|" "auto||" -- tools/surfaces/surface_bench plugin --seconds 2 --threads 16 || exit 1
    bash tools/ab_cmd.sh "$OUT" 2 "p8|BT_HOST_THREADS=8|" "auto||" -- tools/surfaces/surface_bench filter --seconds 2 || exit 1
    summ_ab "$OUT/ab.jsonl" ;;
  data-node-ab)
    for cfg in c2 c3 c4; do
      bash tools/ab_cmd.sh "$OUT" 2 "asis||" "local||--data-node auto" -- python tools/e2e.py --config $cfg --reps 3 || exit 1
    done
    summ_ab "$OUT/ab.jsonl" ;;
  *) echo "unknown case '$CASE' (see the header of tools/gpu_r04.sh)"; exit 2 ;;
esac
