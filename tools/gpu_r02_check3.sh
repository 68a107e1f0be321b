# Session-3 re-entry check: full -m gpu suite, smoke, default bench line
export TMPDIR=/tmp
mkdir -p gpurun_out/r02s3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r02s3/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r02s3/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r02s3/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02s3/smoke.log 2>&1 || { tail gpurun_out/r02s3/smoke.log; exit 1; }
tail -1 gpurun_out/r02s3/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r02s3/bench_default.json 2> gpurun_out/r02s3/bench_default.err || { tail gpurun_out/r02s3/bench_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r02s3/bench_default.json').read().strip().splitlines()[-1]); print('c2f', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac']); [print(k, v['value'], v['ms_per_step'], v['roofline']['kernel_ms'], v['roofline']['frac']) for k,v in d['configs'].items()]"
