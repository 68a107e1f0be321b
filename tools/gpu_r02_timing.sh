# Round 2: host facts + default bench (headline + configs) + timing breakdown repeats
set -o pipefail
mkdir -p gpurun_out/r02
{ nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; free -g; } > gpurun_out/r02/host.txt 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/r02/bench_default.json 2> gpurun_out/r02/bench_default.err || exit 3
for i in 1 2 3; do
  BT_DEBUG_TIMING=1 timeout -k 10 200 python3 bench.py --configs none --no-cpu --config c2 > gpurun_out/r02/dbg_c2_$i.json 2> gpurun_out/r02/dbg_c2_$i.err || exit 4
done
echo done
