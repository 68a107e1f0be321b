mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_payload.py tests/test_gpu_parity.py tests/test_cpp_adapter.py -q -x -p no:cacheprovider > gpurun_out/pytest_payload.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_payload.log; exit $rc
