mkdir -p gpurun_out/d1
( while true; do date >> gpurun_out/heartbeat.log; sleep 50; done ) &
HB=$!; trap "kill $HB" EXIT
for M in 1 4 3; do MODE=$M timeout -k 10 200 python tools/stamps.py > gpurun_out/d1/stamps$M.log 2>&1 || exit 1; done
timeout -k 10 200 python tools/solve_stamps.py > gpurun_out/d1/solve_stamps.log 2>&1 || exit 1
bash tools/ab_opts.sh "" "mfma_fronts=1" > gpurun_out/d1/ab.log 2>&1
cat gpurun_out/d1/ab.log
timeout -k 10 200 python tools/bigfront_bench.py 2048 10 > gpurun_out/d1/bigfront2048.json 2>gpurun_out/d1/bigfront.err && cat gpurun_out/d1/bigfront2048.json
