# A/B: non-temporal staging stores in the host gather (BT_GATHER_NT=1) against plain copies,
# alternating processes on one box, host-gather e2e for C2 / C3 / C4
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04nt}
for cfg in ${CFGS:-c2 c3 c4}; do
  bash tools/ab_cmd.sh "$OUT" ${REPS:-2} "plain|BT_GATHER_NT=0|" "nt|BT_GATHER_NT=1|" -- python tools/e2e.py --config $cfg --reps 3 || exit 1
done
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    if "zero-copy" in r["mode"]: continue
    print(r["variant"], r["rep"], r["config"], r["mode"], r["mpps"])
PY
