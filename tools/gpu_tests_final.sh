#!/bin/bash
# the whole -m gpu suite on the final tree (the 1e6 drop-in test runs ~6 min silently: heartbeat)
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!; trap "kill $HB" EXIT
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 1000 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests_final.log; exit $rc
