#!/bin/bash
# Round-6 evidence of the final tree (C3 unless noted), into gpurun_out/r06/final: bench line (CPU baseline +
# shipped-mode line), rocprofv3 kernel-trace stats, one-step timeline, FETCH_SIZE / WRITE_SIZE passes
# (steady-state factorizations -> pmc_traffic.json), two SQ counter passes, the same-size N=1 point of the
# distributed curve and the IPM-sequence leg.  Large fronts: tools/bigfront_bench.py.
set -e
export TMPDIR=/tmp
R=gpurun_out/r06/final
mkdir -p $R
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!; trap "kill $HB" EXIT
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $R/bench.json 2> $R/bench.err
tail -c 400 $R/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/trace -o run -- python3 bench.py --steps 10 --warmup 2 --profile-only > $R/trace.log 2>&1
python tools/rocpd_summary.py stats $R/trace/run_results.db $R/kernel_stats.csv
python tools/timeline.py $R/trace/run_results.db 2 > $R/timeline_one_step.txt
rm -rf $R/trace
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/pf -o run -- python3 bench.py --steps 6 --warmup 1 --profile-only > $R/pf.log 2>&1
python tools/rocpd_summary.py pmc_steady $R/pf/run_results.db $R/pmc_fetch.json > /dev/null
python tools/rocpd_summary.py bykernel $R/pf/run_results.db > $R/pmc_fetch_bykernel.txt
rm -rf $R/pf
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/pw -o run -- python3 bench.py --steps 6 --warmup 1 --profile-only > $R/pw.log 2>&1
python tools/rocpd_summary.py pmc_steady $R/pw/run_results.db $R/pmc_write.json > /dev/null
python tools/rocpd_summary.py bykernel $R/pw/run_results.db > $R/pmc_write_bykernel.txt
rm -rf $R/pw
python tools/pmc_traffic.py $R/pmc_fetch.json $R/pmc_write.json $R/pmc_traffic.json
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --kernel-trace -d $R/sa -o run -- python3 bench.py --steps 2 --warmup 1 --profile-only > $R/sa.log 2>&1
python tools/rocpd_summary.py bykernel $R/sa/run_results.db > $R/sq_a.txt
rm -rf $R/sa
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAVES --kernel-trace -d $R/sb -o run -- python3 bench.py --steps 2 --warmup 1 --profile-only > $R/sb.log 2>&1
python tools/rocpd_summary.py bykernel $R/sb/run_results.db > $R/sq_b.txt
rm -rf $R/sb
timeout -k 10 400 python bench.py --gpus 1 --mode dist --steps 20 --warmup 5 --no-cpu-baseline --no-shipped > $R/bench_dist1.json 2> $R/bench_dist1.err
tail -c 300 $R/bench_dist1.json
timeout -k 10 400 python bench.py --mode ipm > $R/bench_ipm.json 2> $R/bench_ipm.err
tail -c 300 $R/bench_ipm.json
echo done
