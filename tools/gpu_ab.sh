# A/B + PMC round: tests, prefetch A/B, grid sweep, PMC traffic passes.
mkdir -p gpurun_out
export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['value'], 'Mpps', 'kern', r['kernel_ms'], 'ms frac', r['frac'])" $1; }
timeout -k 10 480 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for cfg in c2 c3 c4; do
  timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu > gpurun_out/ab_${cfg}_pf.json 2>&1 || exit 3
  summ gpurun_out/ab_${cfg}_pf.json
  timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --no-prefetch > gpurun_out/ab_${cfg}_nopf.json 2>&1 || exit 3
  summ gpurun_out/ab_${cfg}_nopf.json
done
for gw in 2048 4096 16384; do
  timeout -k 10 200 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu --grid-waves $gw > gpurun_out/ab_c3_gw$gw.json 2>&1 || exit 3
  summ gpurun_out/ab_c3_gw$gw.json
done
for cfg in c2 c3; do
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${cfg}_fetch -o run -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu > gpurun_out/pmc_${cfg}_fetch.log 2>&1 || exit 4
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${cfg}_write -o run -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu > gpurun_out/pmc_${cfg}_write.log 2>&1 || exit 4
  python3 tools/pmc_traffic.py --fetch gpurun_out/pmc_${cfg}_fetch --write gpurun_out/pmc_${cfg}_write --config $cfg --out gpurun_out/traffic.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu > gpurun_out/prof_c3.log 2>&1 && echo prof-ok
