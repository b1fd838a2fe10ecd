mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 50; done ) &
HB=$!; trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_big_fronts.py tests/test_gpu_parity.py tests/test_null_threshold.py -m gpu -v -rf --timeout 300 --timeout-method thread -x > gpurun_out/big_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/big_tests.log | tail -2
[ $rc -eq 0 ] || exit $rc
start=$(date +%s)
UNO_KKT_VERBOSE=2 timeout -k 10 240 oracle/_ref/uno_kkt_driver arrowband_ineq:100000 linear_solver=HIPLDL logger=SILENT > gpurun_out/ineq.out 2> gpurun_out/ineq.err
echo "ineq rc=$? $(( $(date +%s) - start )) s"
