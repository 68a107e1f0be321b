# round 4 closing evidence, one box: every drop-in C++ surface next to the reference, then the
# rocprofv3 kernel statistics + PMC traffic of the bench workloads
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04surf} STEPS="surfaces" SURF_ARGS="all --seconds 2" bash tools/gpu_round.sh || exit 1
OUT=${OUT:-gpurun_out/r04surf} STEPS="prof" bash tools/gpu_round.sh
