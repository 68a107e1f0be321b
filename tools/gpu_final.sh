# Round-end evidence: parity tests, smoke, bench lines for C2/C3/C4 (with the CPU
# baseline), rocprofv3 kernel stats + FETCH/WRITE PMC passes (tools/gpu_prof.sh).
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh || exit 1
for c in c3 c4; do timeout -k 10 300 python bench.py --config $c > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit 3; done
bash tools/gpu_prof.sh > gpurun_out/prof.log 2>&1 || exit 4
