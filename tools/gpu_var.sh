mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x -p no:cacheprovider -k "zero_copy" 2>&1 | tail -2
for cfg in c2 c3 c4; do timeout -k 10 300 python tools/e2e.py --config $cfg --zero-copy > gpurun_out/zc_$cfg.jsonl || exit 5; cat gpurun_out/zc_$cfg.jsonl; done
