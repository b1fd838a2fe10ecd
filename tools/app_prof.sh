#!/bin/bash
# kernel-time breakdown of dense order-N fronts (rocpd databases; summarised on the host with
# tools/rocpd_summary.py stats)
export TMPDIR=/tmp
mkdir -p gpurun_out/app
for N in "$@"; do
  rm -rf gpurun_out/app/prof$N
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/app/prof$N -o run -- python3 tools/bigfront_bench.py $N 2 > gpurun_out/app/prof$N.log 2>&1 || exit 1
done
