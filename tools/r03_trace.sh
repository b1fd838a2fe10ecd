#!/bin/bash
# kernel-trace stats of the C3 bench (tree as is) + LDS-occupancy probe of the factor kernels
export TMPDIR=/tmp
mkdir -p gpurun_out/r03t
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!; trap "kill $HB" EXIT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03t/trace -o run -- python3 bench.py --steps 10 --warmup 2 --profile-only > gpurun_out/r03t/trace.log 2>&1 || exit 1
python tools/rocpd_summary.py stats gpurun_out/r03t/trace/run_results.db gpurun_out/r03t/kernel_stats.csv > /dev/null
rm -rf gpurun_out/r03t/trace
head -30 gpurun_out/r03t/kernel_stats.csv
for pad in 0 3000 8000; do
  UNO_KKT_LDS_PAD_LDS=$pad timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-shipped > gpurun_out/r03t/pad$pad.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/r03t/pad$pad.json').read().strip().splitlines()[-1]); k=d['roofline']['kernel_ms_per_step']; print('pad $pad', d['value'], k['factor_lds'])"
done
