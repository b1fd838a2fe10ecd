#!/bin/bash
# round 3 diagnostics: per-front factor stamps, solve stamps, bench (with the shipped-mode leg), then the
# configs[2] whole solve through the GPU plugin with its full trace kept for comparison with the golden
mkdir -p gpurun_out/r03
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!; trap "kill $HB" EXIT
for M in 1 4 2; do MODE=$M timeout -k 10 200 python tools/stamps.py > gpurun_out/r03/stamps$M.log 2>&1 || { echo "stamps $M failed"; tail gpurun_out/r03/stamps$M.log; exit 1; }; done
timeout -k 10 200 python tools/solve_stamps.py > gpurun_out/r03/solve_stamps.log 2>&1 || { echo "solve stamps failed"; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/r03/bench1.json 2> gpurun_out/r03/bench1.err || { echo "bench failed"; tail -20 gpurun_out/r03/bench1.err; exit 1; }
tail -c 1500 gpurun_out/r03/bench1.json
timeout -k 10 720 ./oracle/_ref/uno_kkt_driver arrowband:1000000 linear_solver=HIPLDL logger=SILENT > gpurun_out/r03/c3_hipldl.json 2> gpurun_out/r03/c3_hipldl.err
echo "driver rc=$?"
