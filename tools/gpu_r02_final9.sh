# Round-2 closing evidence after the pipelined compaction (part 1, extractor grid 4 blocks/CU): GPU suite, smoke, rocprofv3 stats + PMC traffic of every bench workload, SQ counters.
# of every bench workload (the kernels as committed), SQ counters.
OUT=gpurun_out/r02/final9
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 2; }
tail -1 $OUT/smoke.log
bash tools/gpu_prof.sh $OUT/prof c2f c2 c3 c4 c1 || exit 4
CFGS="c2f c2 c3 c4 c1" bash tools/gpu_sq.sh > $OUT/sq.txt 2>&1 || { tail -5 $OUT/sq.txt; exit 5; }
cat $OUT/sq.txt
