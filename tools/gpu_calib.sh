mkdir -p gpurun_out
export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['value'], 'Mpps step', d['ms_per_step'], 'kern', r['kernel_ms'], 'ms frac', r['frac'])" $1; }
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1; grep -o 'TCC_EA0_[A-Z0-9_]*' gpurun_out/counters_list.txt | sort -u | tr '\n' ' '; echo
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib_fetch -o run -- ./tools/calib/fetch_calib > gpurun_out/calib.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d gpurun_out/calib_rdreq -o run -- ./tools/calib/fetch_calib >> gpurun_out/calib.log 2>&1 || echo rdreq-pass-failed
python3 tools/calib/analyze.py gpurun_out/calib_fetch/run_counter_collection.csv
for gw in 4096 8192 16384 32768; do
  timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu --grid-waves $gw > gpurun_out/gs_c2_$gw.json 2>&1 || exit 3
  summ gpurun_out/gs_c2_$gw.json
done
for gw in 4096 8192; do
  for cfg in c3 c4; do
  timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --grid-waves $gw > gpurun_out/gs_${cfg}_$gw.json 2>&1 || exit 3
  summ gpurun_out/gs_${cfg}_$gw.json
  done
done
