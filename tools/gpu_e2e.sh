# End-to-end (PCIe-inclusive) rates: host gather, zero-copy, TPACKET_V3 ring; C2/C3/C4.
mkdir -p gpurun_out
for c in c2 c3 c4; do
  for m in "" "--zero-copy" "--tpacket"; do
    timeout -k 10 300 python tools/e2e.py --config $c $m --reps 2 >> gpurun_out/e2e.jsonl 2> gpurun_out/e2e_err.log || { tail -5 gpurun_out/e2e_err.log; exit 3; }
  done
done
cat gpurun_out/e2e.jsonl | cut -c1-260
