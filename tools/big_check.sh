#!/bin/bash
# large-front path: GPU tests (default: the whole -m gpu suite), then dense-front throughput at several orders
mkdir -p gpurun_out/big
( while true; do date >> gpurun_out/heartbeat.log; sleep 50; done ) &
HB=$!; trap "kill $HB" EXIT
args=("$@"); [ ${#args[@]} -eq 0 ] && args=(tests -m gpu)
timeout -k 10 600 python -u -m pytest "${args[@]}" -x -q --timeout 300 --timeout-method thread > gpurun_out/big/tests.log 2>&1
rc=$?; tail -3 gpurun_out/big/tests.log; [ $rc -eq 0 ] || exit $rc
for n in 512 1024 2048 4096; do
  timeout -k 10 200 python tools/bigfront_bench.py $n 5 > gpurun_out/big/dense$n.json 2> gpurun_out/big/dense$n.err || { tail -5 gpurun_out/big/dense$n.err; exit 1; }
  cat gpurun_out/big/dense$n.json
done
