#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!; trap "kill $HB" EXIT
UNO_KKT_SWEEP_NOATOMIC=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03s/na -o run -- python3 bench.py --steps 5 --warmup 1 --profile-only > gpurun_out/r03s/na.log 2>&1 || exit 1
python tools/rocpd_summary.py stats gpurun_out/r03s/na/run_results.db gpurun_out/r03s/na_stats.csv > /dev/null; rm -rf gpurun_out/r03s/na
grep -i "sweep\|pack" gpurun_out/r03s/na_stats.csv
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/r03s/f -o run -- python3 bench.py --steps 2 --warmup 1 --profile-only > gpurun_out/r03s/f.log 2>&1 || exit 1
python tools/rocpd_summary.py bykernel gpurun_out/r03s/f/run_results.db > gpurun_out/r03s/fetch.txt; rm -rf gpurun_out/r03s/f
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/r03s/w -o run -- python3 bench.py --steps 2 --warmup 1 --profile-only > gpurun_out/r03s/w.log 2>&1 || exit 1
python tools/rocpd_summary.py bykernel gpurun_out/r03s/w/run_results.db > gpurun_out/r03s/write.txt; rm -rf gpurun_out/r03s/w
grep -A1 "sweep\|pack\|solve_fwd\|factor_lds<64, 8>" gpurun_out/r03s/fetch.txt gpurun_out/r03s/write.txt
