# Full -m gpu suite + smoke
export TMPDIR=/tmp
mkdir -p gpurun_out/r02
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r02/pytest_gpu.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r02/pytest_gpu.log | grep -v PASSED | head; tail -2 gpurun_out/r02/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02/smoke.log 2>&1 && tail -1 gpurun_out/r02/smoke.log
