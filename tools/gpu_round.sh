# Full GPU round: parity tests (Python + C++), smoke, benches, e2e.
mkdir -p gpurun_out
export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; c=d.get('cpu_baseline') or {}; print(sys.argv[1], d['value'], 'Mpps step', d['ms_per_step'], 'span', r['gpu_span_ms_per_step'], 'kern', r['kernel_ms'], 'frac', r['frac'], 'cpu', c.get('value'))" $1; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -rs > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log
for cfg in c2 c3 c4; do
  timeout -k 10 300 python bench.py --config $cfg > gpurun_out/bench_$cfg.json 2>gpurun_out/bench_$cfg.err || exit 3
  summ gpurun_out/bench_$cfg.json
done
for cfg in c2 c3 c4; do timeout -k 10 300 python tools/e2e.py --config $cfg > gpurun_out/e2e_$cfg.json 2>&1 || exit 5; cat gpurun_out/e2e_$cfg.json; done
