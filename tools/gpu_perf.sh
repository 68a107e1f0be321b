# Parity tests, then bench + rocprofv3 kernel stats for the configs given (default c2 c3 c4).
mkdir -p gpurun_out
export TMPDIR=/tmp
CFGS=${@:-c2 c3 c4}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for cfg in $CFGS; do
  timeout -k 10 300 python bench.py --config $cfg --no-cpu > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err || { tail gpurun_out/bench_$cfg.err; exit 3; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['value'], 'Mpps ms/step', d['ms_per_step'], 'kern', r['kernel_ms'], 'frac', r['frac'])" gpurun_out/bench_$cfg.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$cfg -o run -- python3 bench.py --config $cfg --steps 20 --warmup 3 --no-cpu > gpurun_out/prof_$cfg.json 2>&1 || exit 4
  cut -d, -f1-4 gpurun_out/prof_$cfg/run_kernel_stats.csv | cut -c1-160
done
