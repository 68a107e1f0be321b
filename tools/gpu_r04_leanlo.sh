# lean round A that skips bytes 0..11 (BT_LEAN_LO=12) and ends at 38 B (BT_LEAN_END=38): the GPU
# suite with it on, then e2e zero-copy / TPACKET_V3 ring A/B, alternating processes on one box
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04leanlo}
mkdir -p "$OUT"
BT_LEAN_LO=12 BT_LEAN_END=38 timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > "$OUT/pytest_lean12_38.log" 2>&1 || { tail -30 "$OUT/pytest_lean12_38.log"; exit 1; }
tail -2 "$OUT/pytest_lean12_38.log"
for cfg in c2 c3 c4; do
  for mode in --zero-copy --tpacket; do
    bash tools/ab_cmd.sh "$OUT" 2 "lo0||" "lo12|BT_LEAN_LO=12|" "lo12e38|BT_LEAN_LO=12 BT_LEAN_END=38|" \
      -- python tools/e2e.py --config $cfg $mode --reps 3 || exit 1
  done
done
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys
from collections import defaultdict
d = defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l)
    if "verdicts" not in r["mode"] or "records" in r["mode"]: continue
    d[(r["config"], r["mode"][:40], r["variant"])].append(r["mpps"])
for k in sorted(d): print(k, d[k])
PY
