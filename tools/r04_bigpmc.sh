#!/bin/bash
# Large fronts (dense order N, default 4096): HBM traffic and SQ counter passes of the a-posteriori kernels
# (tools/bigfront_bench.py), into gpurun_out/r04bigpmc
N=${1:-4096}
export TMPDIR=/tmp
R=gpurun_out/r04bigpmc
mkdir -p $R
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!; trap "kill $HB" EXIT
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/f -o run -- python3 tools/bigfront_bench.py $N 2 > $R/f.log 2>&1 || { tail -5 $R/f.log; exit 1; }
python tools/rocpd_summary.py bykernel $R/f/run_results.db > $R/dense${N}_fetch.txt 2>&1; rm -rf $R/f
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/w -o run -- python3 tools/bigfront_bench.py $N 2 > $R/w.log 2>&1 || { tail -5 $R/w.log; exit 1; }
python tools/rocpd_summary.py bykernel $R/w/run_results.db > $R/dense${N}_write.txt 2>&1; rm -rf $R/w
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --kernel-trace -d $R/s -o run -- python3 tools/bigfront_bench.py $N 2 > $R/s.log 2>&1 || { tail -5 $R/s.log; exit 1; }
python tools/rocpd_summary.py bykernel $R/s/run_results.db > $R/dense${N}_sq.txt 2>&1; rm -rf $R/s
for k in k_app_diag k_app_rows k_app_update k_app_exact k_big_update; do grep -A9 "$k" $R/dense${N}_fetch.txt $R/dense${N}_write.txt $R/dense${N}_sq.txt | grep -E "$k|FETCH|WRITE|SQ_" | head -14; done
