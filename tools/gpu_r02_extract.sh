# GPU: user-protocol extraction tests, then the rest of the suite
export TMPDIR=/tmp
mkdir -p gpurun_out/r02
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r02/pytest_extract.log 2>&1; rc=$?
tail -25 gpurun_out/r02/pytest_extract.log
exit $rc
