#!/bin/bash
# GPU tests with a heartbeat (the drop-in runs print nothing for minutes): bash tools/gpu_tests.sh TAG [pytest args]
T=${1:-tests}; shift
mkdir -p gpurun_out/$T
( while true; do date >> gpurun_out/$T/heartbeat.log; sleep 30; done ) &
HB=$!; trap "kill $HB" EXIT
timeout -k 10 1100 python -u -m pytest "$@" -m gpu -x -v --timeout 1000 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/$T/pytest.log | tail -40; exit $rc
