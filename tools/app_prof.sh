#!/bin/bash
# kernel-time breakdown of the dense order-N front (rocpd database; summarised on the host)
export TMPDIR=/tmp
N=${1:-4096}
mkdir -p gpurun_out/app
rm -rf gpurun_out/app/prof$N
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/app/prof$N -o run -- python3 tools/bigfront_bench.py $N 2 > gpurun_out/app/prof$N.log 2>&1
