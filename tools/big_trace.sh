#!/bin/bash
# kernel-trace statistics of the dense-front bench (bash tools/big_trace.sh N)
N=${1:-2048}
export TMPDIR=/tmp
mkdir -p gpurun_out/bigtrace
( while true; do date >> gpurun_out/heartbeat.log; sleep 50; done ) &
HB=$!; trap "kill $HB" EXIT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bigtrace/t$N -o run -- python3 tools/bigfront_bench.py $N 3 > gpurun_out/bigtrace/t$N.log 2>&1 && \
python tools/rocpd_summary.py stats gpurun_out/bigtrace/t$N/run_results.db gpurun_out/bigtrace/stats$N.csv && head -25 gpurun_out/bigtrace/stats$N.csv
