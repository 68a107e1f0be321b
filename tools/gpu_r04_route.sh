# group routing: the group GPU tests, then an A/B of routed concurrent calls (default) against
# always splitting (BT_GROUP_ROUTE_BELOW=0), surface_bench group (1 / 2 / 4 shared-device members,
# 1 and 16 callers), alternating processes on one box
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04route}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_group.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
bash tools/ab_cmd.sh "$OUT" 2 "split|BT_GROUP_ROUTE_BELOW=0|" "routed||" -- tools/surfaces/surface_bench group --seconds 2 || exit 1
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["variant"], r["rep"], r["config"], "members", r.get("members"), "callers", r["threads"], round(r["mpps"], 1),
          "cpu/Mpkt", r.get("host_cpu_s_per_mpkt"))
PY
