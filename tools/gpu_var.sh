mkdir -p gpurun_out
timeout -k 10 120 ./tools/ringwalk/walk_scaling 3 8000000 1048576 16 pool || exit 3
for cfg in c2 c3 c4; do timeout -k 10 300 python tools/e2e.py --config $cfg --tpacket --host-threads 16 > gpurun_out/tp_$cfg.jsonl || exit 5; cat gpurun_out/tp_$cfg.jsonl; done
