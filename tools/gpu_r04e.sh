# round 4: host gather through one context against a group of one (same box, alternating)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
bash tools/ab_cmd.sh $O/g1 2 "single||" "group1||--group 1" -- python tools/e2e.py --config c2 --reps 2 || exit 1
bash tools/ab_cmd.sh $O/g1 1 "single||" "group1||--group 1" -- python tools/e2e.py --config c3 --reps 2 || exit 1
echo ALL-DONE
