# Profiles of the current kernels (keyed traffic for bench.py) + SQ counters
export TMPDIR=/tmp
bash tools/gpu_prof.sh gpurun_out/r02/prof c2f c2 c3 c4 || exit 4
CFGS="c2f c3 c4" bash tools/gpu_sq.sh > gpurun_out/r02/sq.txt 2>&1 || exit 5
cat gpurun_out/r02/sq.txt
