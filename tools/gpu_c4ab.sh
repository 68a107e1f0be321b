timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash tools/gpu_abx.sh tools/ab/rows.so tools/ab/line.so "c4 c3" 3 || exit 2
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_c4_fetch -o run -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu > /dev/null 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_c4_write -o run -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu > /dev/null 2>&1 || exit 4
python3 tools/pmc_traffic.py --fetch gpurun_out/pmc_c4_fetch --write gpurun_out/pmc_c4_write --config c4 --out gpurun_out/traffic_new.json | cut -c1-300
