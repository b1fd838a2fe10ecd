#!/bin/bash
# parity tests of the final tree, lpos16 A/B, then the round-3 profile set
mkdir -p gpurun_out/ab3
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!; trap "kill $HB" EXIT
TESTS="tests/test_gpu_parity.py tests/test_null_threshold.py tests/test_big_fronts.py tests/test_distributed.py -m gpu" bash tools/ab3.sh "l16|" "l32|--opt lpos16=0" "l16b|" "l32b|--opt lpos16=0" || exit 1
kill $HB; trap - EXIT
bash tools/profile_r03.sh
