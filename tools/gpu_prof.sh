# Profiles of the current kernels: rocprofv3 kernel stats + separate FETCH/WRITE PMC passes,
# one bench workload at a time (--configs none). Usage: bash tools/gpu_prof.sh [OUTDIR] [configs...]
# The stats run times PROF_STEPS (default 100) steps: rocprofv3's average covers every launch
# of the process, and the 10-15 launches the GPU runs slower a few ms after the host's
# bookkeeping idle ("rocprof average") would otherwise weigh 1 in 4.
OUT=${1:-gpurun_out/prof}; shift
CFGS=${*:-c2f c2 c3 c4 c1}
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in $CFGS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_$cfg -o run -- python3 bench.py --config $cfg --configs none --steps ${PROF_STEPS:-100} --warmup 3 --no-cpu > $OUT/${cfg}_bench_under_rocprof.json 2>&1 || exit 4
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_${cfg}_fetch -o run -- python3 bench.py --config $cfg --configs none --steps 3 --warmup 1 --no-cpu > /dev/null 2>&1 || exit 4
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_${cfg}_write -o run -- python3 bench.py --config $cfg --configs none --steps 3 --warmup 1 --no-cpu > /dev/null 2>&1 || exit 4
  python3 tools/pmc_traffic.py --fetch $OUT/pmc_${cfg}_fetch --write $OUT/pmc_${cfg}_write --config $cfg --out $OUT/traffic.json | cut -c1-200
  cp $OUT/stats_$cfg/run_kernel_stats.csv $OUT/${cfg}_kernel_stats.csv
  cp $OUT/stats_$cfg/run_kernel_trace.csv $OUT/${cfg}_kernel_trace.csv
  grep -E "parse_filter_(main|pipe)|extract_tile" $OUT/${cfg}_kernel_stats.csv | cut -d, -f2-5
done
