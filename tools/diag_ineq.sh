# Drop-in diagnostics at KKT dimension 1e5: wall time and per-factorization log of the reference Uno core
# with the GPU plugin (UNO_KKT_VERBOSE=2), optionally with extra library options ($1, UNO_KKT_OPTIONS syntax).
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 50; done ) &
HB=$!; trap "kill $HB" EXIT
for model in arrowband:100000 arrowband_ineq:100000; do
  tag=${model%%:*}
  start=$(date +%s)
  UNO_KKT_OPTIONS="$1" UNO_KKT_VERBOSE=2 timeout -k 10 200 oracle/_ref/uno_kkt_driver $model linear_solver=HIPLDL logger=SILENT \
    > gpurun_out/$tag.out 2> gpurun_out/$tag.err
  echo "$model rc=$? $(( $(date +%s) - start )) s"
done
