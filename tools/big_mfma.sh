#!/bin/bash
# MFMA activity of the large-front path: kernel trace + one PMC pass (SQ MFMA / VALU counters) of the
# dense-front bench (bash tools/big_mfma.sh N)
N=${1:-4096}
export TMPDIR=/tmp
mkdir -p gpurun_out/bigmfma
( while true; do date >> gpurun_out/heartbeat.log; sleep 50; done ) &
HB=$!; trap "kill $HB" EXIT
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/bigmfma/avail.txt 2>&1
grep -iE "MFMA|VALU_MFMA|SQ_BUSY_CU|GRBM_GUI" gpurun_out/bigmfma/avail.txt | head -30
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bigmfma/t -o run -- python3 tools/bigfront_bench.py $N 3 > gpurun_out/bigmfma/t.log 2>&1 && \
python tools/rocpd_summary.py stats gpurun_out/bigmfma/t/run_results.db gpurun_out/bigmfma/stats$N.csv && head -8 gpurun_out/bigmfma/stats$N.csv || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/bigmfma/p -o run -- python3 tools/bigfront_bench.py $N 2 > gpurun_out/bigmfma/p.log 2>&1 || { tail -5 gpurun_out/bigmfma/p.log; exit 1; }
python tools/rocpd_summary.py bykernel gpurun_out/bigmfma/p/run_results.db > gpurun_out/bigmfma/pmc_bykernel.txt 2>&1; head -60 gpurun_out/bigmfma/pmc_bykernel.txt
