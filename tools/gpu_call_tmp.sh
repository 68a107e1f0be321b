set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 5; }
tail -3 gpurun_out/pytest_gpu.log
bash tools/gpu_abenv.sh "BT_NO_PIPE=1" "BT_NO_PIPE=0" "c3 c4" 3 || exit 6
