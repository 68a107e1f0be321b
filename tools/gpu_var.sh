mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_payload.py tests/test_gpu_parity.py -q -x -p no:cacheprovider > gpurun_out/pytest_payload.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_payload.log; [ $rc -eq 0 ] || exit $rc
for re in 'GET|POST' 'HTTP/1\.[01] [1-5][0-9][0-9]'; do
  timeout -k 10 300 python bench.py --config c3 --no-cpu --payload "$re" > gpurun_out/bench_c3_payload.json 2>&1 || exit 4
  tail -1 gpurun_out/bench_c3_payload.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['config']['workload'][-40:], d['value'], 'kern', r['kernel_ms'], 'frac', r['frac'])"
done
timeout -k 10 300 python bench.py --config c3 --no-cpu | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c3 plain', d['value'], 'kern', r['kernel_ms'], 'frac', r['frac'])"
