#!/bin/bash
# round 3 probe: whole solve at KKT dimension 1e5 with MUMPS-style delays (delay_relaxed=1) vs the shipped
# relaxation mode, merge-round counts and rebuild times, then the C3 bench line on this box
mkdir -p gpurun_out/r03
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!; trap "kill $HB" EXIT
for mode in 1 0; do
  s=$(date +%s.%N)
  UNO_KKT_VERBOSE=1 UNO_KKT_OPTIONS=delay_relaxed=$mode timeout -k 10 300 ./oracle/_ref/uno_kkt_driver arrowband:100000 linear_solver=HIPLDL logger=SILENT \
    > gpurun_out/r03/ab1e5_d$mode.json 2> gpurun_out/r03/ab1e5_d$mode.err || { echo "FAILED d$mode"; tail -5 gpurun_out/r03/ab1e5_d$mode.err; exit 1; }
  e=$(date +%s.%N)
  echo "delay_relaxed=$mode wall $(python -c "print(round($e - $s, 2))") s merges: $(grep -c 'merge round' gpurun_out/r03/ab1e5_d$mode.err)"
done
timeout -k 10 300 python bench.py > gpurun_out/r03/bench0.json 2> gpurun_out/r03/bench0.err || { echo "bench failed"; tail -20 gpurun_out/r03/bench0.err; exit 1; }
tail -c 600 gpurun_out/r03/bench0.json
