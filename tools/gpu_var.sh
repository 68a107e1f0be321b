mkdir -p gpurun_out
for cfg in c2 c3; do for bb in 128 512; do timeout -k 10 300 python tools/e2e.py --config $cfg --tpacket --host-threads 16 --ring-batch-blocks $bb --reps 3 || exit 5; done; done
