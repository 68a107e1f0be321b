mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 480 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo smoke-ok &&
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 5 > gpurun_out/bench_c2.log 2>&1 && cat gpurun_out/bench_c2.log &&
  timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --cpu-seconds 5 > gpurun_out/bench_c3.log 2>&1 && cat gpurun_out/bench_c3.log &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/prof_c2.log 2>&1 && echo prof-ok
fi
