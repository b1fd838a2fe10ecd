#!/bin/bash
# Round profile: full bench line, rocprofv3 kernel-trace stats, and a separate PMC pass (HBM bytes).
# usage (on the GPU box): tools/profile_round.sh r01
set -e
R=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$R/trace -o run -- python3 bench.py --steps 10 --warmup 2 --profile-only > gpurun_out/$R/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/$R/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --profile-only > gpurun_out/$R/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/$R/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --profile-only > gpurun_out/$R/pmc_write.log 2>&1

python tools/rocpd_summary.py stats gpurun_out/$R/trace/run_results.db gpurun_out/$R/kernel_stats.csv
python tools/rocpd_summary.py pmc gpurun_out/$R/pmc_fetch/run_results.db gpurun_out/$R/pmc_fetch.json > /dev/null
python tools/rocpd_summary.py pmc gpurun_out/$R/pmc_write/run_results.db gpurun_out/$R/pmc_write.json > /dev/null
python tools/pmc_traffic.py gpurun_out/$R/pmc_fetch.json gpurun_out/$R/pmc_write.json gpurun_out/$R/pmc_traffic.json > /dev/null
echo done
