mkdir -p gpurun_out
for i in 1 2 3 4 5 6 7 8; do
  BT_DEBUG_TIMING=1 timeout -k 10 200 python bench.py --config c4 --steps 30 --warmup 3 --no-cpu > gpurun_out/dbg_$i.json 2> gpurun_out/dbg_$i.err || exit 3
  echo "run $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dbg_$i.json)"; grep -E "bench\]|bt_time_device" gpurun_out/dbg_$i.err | tail -2
done
