#!/bin/bash
# a-posteriori large-front steps: big-front GPU tests, then dense-front throughput with and without them
mkdir -p gpurun_out/app
( while true; do date >> gpurun_out/heartbeat.log; sleep 50; done ) &
HB=$!; trap "kill $HB" EXIT
args=("$@"); [ ${#args[@]} -eq 0 ] && args=(tests/test_big_fronts.py -m gpu)
timeout -k 10 600 python -u -m pytest "${args[@]}" -x -q --timeout 300 --timeout-method thread > gpurun_out/app/tests.log 2>&1
rc=$?; tail -5 gpurun_out/app/tests.log; [ $rc -eq 0 ] || exit $rc
for n in 512 1024 2048 4096; do
  timeout -k 10 200 python tools/bigfront_bench.py $n 5 > gpurun_out/app/dense$n.json 2> gpurun_out/app/dense$n.err || { tail -5 gpurun_out/app/dense$n.err; exit 1; }
  cat gpurun_out/app/dense$n.json
done
for n in 1024 4096; do
  UNO_KKT_OPTIONS=big_app=0 timeout -k 10 200 python tools/bigfront_bench.py $n 3 > gpurun_out/app/dense${n}_off.json 2> gpurun_out/app/dense${n}_off.err || { tail -5 gpurun_out/app/dense${n}_off.err; exit 1; }
  cat gpurun_out/app/dense${n}_off.json
done
