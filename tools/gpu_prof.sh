# Profiles for the current kernel: rocprofv3 kernel stats + separate FETCH/WRITE PMC passes.
mkdir -p gpurun_out
export TMPDIR=/tmp
(amd-smi process 2>&1 || rocm-smi --showpids 2>&1) | head -30 > gpurun_out/gpu_procs_before.txt
for cfg in c2 c3 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$cfg -o run -- python3 bench.py --config $cfg --steps 20 --warmup 3 --no-cpu > gpurun_out/prof_$cfg.json 2>&1 || exit 4
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${cfg}_fetch -o run -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu > /dev/null 2>&1 || exit 4
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${cfg}_write -o run -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu > /dev/null 2>&1 || exit 4
  python3 tools/pmc_traffic.py --fetch gpurun_out/pmc_${cfg}_fetch --write gpurun_out/pmc_${cfg}_write --config $cfg --out gpurun_out/traffic.json | cut -c1-200
  grep -E "parse_filter_(main|pipe)" gpurun_out/prof_$cfg/run_kernel_stats.csv | cut -d, -f2-5
  tail -1 gpurun_out/prof_$cfg.json | cut -c1-100
done
(python3 bench.py --config c3 --steps 200 --warmup 3 --no-cpu > /dev/null 2>&1 &) ; sleep 6; (amd-smi process 2>&1 || rocm-smi --showpids 2>&1) | head -40 > gpurun_out/gpu_procs_during.txt; sleep 8
cat gpurun_out/gpu_procs_during.txt | head -40
