set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04b
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py tests/test_cpp_adapter.py -k "mapped or small" -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r04b/pytest.log 2>&1 || { tail -30 gpurun_out/r04b/pytest.log; exit 1; }
tail -2 gpurun_out/r04b/pytest.log
OUT=gpurun_out/r04b STEPS="e2e" E2E_CFGS="c2 c3" E2E_MODES="--group 1;--group 2;--group 4" bash tools/gpu_round.sh > gpurun_out/r04b/round_e2e.txt 2>&1 || { tail -20 gpurun_out/r04b/round_e2e.txt; exit 1; }
timeout -k 10 400 tools/surfaces/surface_bench single --seconds 1.5 > gpurun_out/r04b/surf_single.jsonl 2> gpurun_out/r04b/surf_single.err || { tail gpurun_out/r04b/surf_single.err; exit 1; }
timeout -k 10 400 tools/surfaces/surface_bench group --seconds 2 --packets 2097152 > gpurun_out/r04b/surf_group.jsonl 2> gpurun_out/r04b/surf_group.err || { tail gpurun_out/r04b/surf_group.err; exit 1; }
echo ALL-DONE
