#!/bin/bash
# The whole GPU suite on the final tree with a heartbeat, log into gpurun_out/r06/tests
mkdir -p gpurun_out/r06/tests
( while true; do date >> gpurun_out/r06/tests/heartbeat.log; sleep 30; done ) &
HB=$!; trap "kill $HB" EXIT
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 1000 --timeout-method thread > gpurun_out/r06/tests/pytest.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r06/tests/pytest.log | tail -3; exit $rc
