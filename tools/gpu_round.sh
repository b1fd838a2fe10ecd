# GPU round script: heartbeat (the box kills commands silent for 180 s), gpu tests, bench.
# usage: bash tools/gpu_round.sh [pytest args...]   (default: the whole -m gpu suite)
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 50; done ) &
HB=$!
trap "kill $HB" EXIT
args=("$@"); [ ${#args[@]} -eq 0 ] && args=(tests -m gpu)
timeout -k 10 1000 python -u -m pytest "${args[@]}" -v -rf --timeout 400 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -3
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ -n "$NO_BENCH" ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
echo "bench rc=$?"; tail -c 3000 gpurun_out/bench.log
