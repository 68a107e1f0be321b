# round 4: the whole GPU suite, then the group e2e rows (1/2/4 members) and the NUMA A/B on C3
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
OUT=$O STEPS="tests" bash tools/gpu_round.sh || exit 1
OUT=$O STEPS="e2e" E2E_CFGS="c2 c3 c4" E2E_MODES="--group 1;--group 2;--group 4" bash tools/gpu_round.sh > $O/round_e2e.txt 2>&1 || { tail -5 $O/round_e2e.txt; exit 1; }
bash tools/ab_cmd.sh $O/pin 2 "pin||" "nopin|BT_NUMA_PIN=0|" -- python tools/e2e.py --config c3 --reps 2 || exit 1
bash tools/ab_cmd.sh $O/pin 2 "pin||" "nopin|BT_NUMA_PIN=0|" -- python tools/e2e.py --config c4 --reps 2 || exit 1
echo ALL-DONE
