# A/B: non-temporal stores for the host pipeline's record drain (BT_DRAIN_NT=1) against memcpy,
# alternating processes on one box, host-gather e2e (records + verdicts rows) for C2 / C3 / C4
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04drain}
for cfg in ${CFGS:-c2 c3 c4}; do
  bash tools/ab_cmd.sh "$OUT" ${REPS:-3} "memcpy|BT_DRAIN_NT=0|" "nt|BT_DRAIN_NT=1|" -- python tools/e2e.py --config $cfg --reps 3 || exit 1
done
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    if "zero-copy" in r["mode"]: continue
    print(r["variant"], r["rep"], r["config"], r["mode"], r["mpps"])
PY
