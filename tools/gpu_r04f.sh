# round 4: pipe2 (round B one tile ahead) parity, then A/B against pipe on C4 / C3; and the
# host gather through one context against a group of one
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
BT_PIPE2=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ring.py tests/test_gpu_group.py tests/test_gpu_staging.py tests/test_gpu_robustness.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_pipe2.log 2>&1 || { tail -30 $O/pytest_pipe2.log; exit 1; }
tail -1 $O/pytest_pipe2.log
bash tools/gpu_abenv.sh "BT_PIPE2=0" "BT_PIPE2=1" "c4 c3" 3 > $O/ab_pipe2.txt 2>&1 || { tail $O/ab_pipe2.txt; exit 1; }
cat $O/ab_pipe2.txt
bash tools/ab_cmd.sh $O/g1 2 "single||" "group1||--group 1" -- python tools/e2e.py --config c2 --reps 2 || exit 1
echo ALL-DONE
