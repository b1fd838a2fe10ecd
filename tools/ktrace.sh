# Kernel-trace statistics of the bench (profile-only pass): gpurun_out/ktrace/kernel_stats.csv
# usage (on the GPU box): bash tools/ktrace.sh [extra bench args]
export TMPDIR=/tmp
mkdir -p gpurun_out/ktrace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ktrace/trace -o run -- python3 bench.py --steps 10 --warmup 2 --profile-only "$@" > gpurun_out/ktrace/trace.log 2>&1 && \
python tools/rocpd_summary.py stats gpurun_out/ktrace/trace/run_results.db gpurun_out/ktrace/kernel_stats.csv && \
head -25 gpurun_out/ktrace/kernel_stats.csv
