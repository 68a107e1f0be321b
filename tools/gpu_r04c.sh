# round 4: A/B of the NUMA pinning (host gather) and of serialising shared-device members
# (group zero-copy), alternating processes on one box; then the small-call surfaces again.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
bash tools/ab_cmd.sh $O/pin 2 "pin||" "nopin|BT_NUMA_PIN=0|" -- python tools/e2e.py --config c2 --reps 2 || exit 1
bash tools/ab_cmd.sh $O/pin 1 "pin||" "nopin|BT_NUMA_PIN=0|" -- python tools/e2e.py --config c3 --reps 2 || exit 1
bash tools/ab_cmd.sh $O/serial 2 "concurrent||" "serial|BT_GROUP_SHARED_SERIAL=1|" -- python tools/e2e.py --config c2 --group 2 --reps 2 || exit 1
timeout -k 10 300 tools/surfaces/surface_bench single --seconds 1 > $O/surf_single.jsonl 2> $O/surf_single.err || exit 1
echo ALL-DONE
