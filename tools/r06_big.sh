#!/bin/bash
# Large fronts (dense order N, default 4096), round-6 tree: bench lines, kernel-trace stats and one MFMA / VALU PMC pass of
# tools/bigfront_bench.py, into gpurun_out/r06/bigfront
N=${1:-4096}
export TMPDIR=/tmp
R=gpurun_out/r06/bigfront
mkdir -p $R
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!; trap "kill $HB" EXIT
for n in 1024 2048 $N; do
  timeout -k 10 300 python3 tools/bigfront_bench.py $n 3 > $R/dense$n.json 2> $R/dense$n.err || { tail -5 $R/dense$n.err; exit 1; }
  tail -c 300 $R/dense$n.json; echo
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/t -o run -- python3 tools/bigfront_bench.py $N 3 > $R/t.log 2>&1 && \
python tools/rocpd_summary.py stats $R/t/run_results.db $R/dense${N}_kernel_stats.csv && head -12 $R/dense${N}_kernel_stats.csv || exit 1
rm -rf $R/t
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU SQ_WAVE_CYCLES --kernel-trace -d $R/p -o run -- python3 tools/bigfront_bench.py $N 2 > $R/p.log 2>&1 || { tail -5 $R/p.log; exit 1; }
python tools/rocpd_summary.py bykernel $R/p/run_results.db > $R/dense${N}_pmc_mfma.txt 2>&1
rm -rf $R/p
grep -A6 "k_app_update\|k_big_update" $R/dense${N}_pmc_mfma.txt | head -30
