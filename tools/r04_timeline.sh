#!/bin/bash
# one-step kernel timeline of the C3 bench (rocprofv3 kernel trace): gpurun_out/tl/timeline.txt
export TMPDIR=/tmp
mkdir -p gpurun_out/tl
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl/trace -o run -- python3 bench.py --steps 6 --warmup 2 --profile-only > gpurun_out/tl/trace.log 2>&1 || exit 1
python tools/timeline.py gpurun_out/tl/trace/run_results.db 2 > gpurun_out/tl/timeline.txt
rm -rf gpurun_out/tl/trace
cat gpurun_out/tl/timeline.txt
