# round 4: GPU suite on the release and the bounds-checked builds, then the group surfaces
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
OUT=$O STEPS="tests bounds" bash tools/gpu_round.sh || exit 1
timeout -k 10 400 tools/surfaces/surface_bench group --seconds 2 --packets 2097152 > $O/surf_group.jsonl 2> $O/surf_group.err || { tail $O/surf_group.err; exit 1; }
echo ALL-DONE
