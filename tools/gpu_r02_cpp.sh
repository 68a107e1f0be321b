# GPU: the C++ drop-in parity binaries
export TMPDIR=/tmp
mkdir -p gpurun_out/r02
timeout -k 10 600 ./tests/cpp/test_adapter beatrice_amd/libgpu_parse_filter_plugin.so > gpurun_out/r02/cpp_adapter.log 2>&1; rc=$?
tail -8 gpurun_out/r02/cpp_adapter.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 ./tests/cpp/test_plugin beatrice_amd/libgpu_parse_filter_plugin.so > gpurun_out/r02/cpp_plugin.log 2>&1; rc=$?
cat gpurun_out/r02/cpp_plugin.log
exit $rc
