set -e
export TMPDIR=/tmp
R=gpurun_out/ipmprof
mkdir -p $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/trace -o run -- python3 bench.py --mode ipm --ipm-iters 3 > $R/out.json 2> $R/err.log
python tools/rocpd_summary.py stats $R/trace/run_results.db $R/kernel_stats.csv
rm -rf $R/trace
head -25 $R/kernel_stats.csv
