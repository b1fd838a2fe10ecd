#!/bin/bash
# whole ipopt-preset Uno solves through the GPU plugin (reference Uno core + HIPLDL), wall time per model
mkdir -p gpurun_out/whole
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!; trap "kill $HB" EXIT
for model in "$@"; do
  s=$(date +%s.%N)
  timeout -k 10 900 ./oracle/_ref/uno_kkt_driver $model linear_solver=HIPLDL logger=SILENT > gpurun_out/whole/$model.json 2> gpurun_out/whole/$model.err || { echo "FAILED $model"; tail -5 gpurun_out/whole/$model.err; exit 1; }
  e=$(date +%s.%N)
  echo "$model wall $(python -c "print(round($e - $s, 2))") s: $(tail -c 400 gpurun_out/whole/$model.json)"
done
