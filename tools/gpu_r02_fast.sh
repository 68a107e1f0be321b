# Parity tests on the uniform-predicate filter + c2f/c3/c4 kernel times
export TMPDIR=/tmp
mkdir -p gpurun_out/r02
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r02/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r02/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r02/pytest_gpu.log
for c in c2f c3 c4; do
timeout -k 10 200 python3 bench.py --config $c --configs none --no-cpu > gpurun_out/r02/fast_$c.json 2>&1 || exit 3
python3 -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/r02/fast_$c.json') if l.startswith('{')][-1]); r=d['roofline']
print('$c', 'kern', r['kernel_ms'], 'step', d['ms_per_step'], 'Mpps', d['value'], 'frac', r['frac'])"
done
