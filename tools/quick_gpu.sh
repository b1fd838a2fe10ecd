# quick GPU iteration: parity tests that cover the numerics, then the kernel trace of the bench
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 50; done ) &
HB=$!; trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_null_threshold.py tests/test_big_fronts.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/quick_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/ktrace.sh "$@"
