#!/bin/bash
# PMC passes (one rocprofv3 --pmc pass each; bench --profile-only): bash tools/r04_pmc.sh TAG [bench args]; summaries per kernel in gpurun_out/TAG/[abcd].txt
T=${1:-pmcs}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/$T
timeout -s KILL 60 rocprofv3 -L > gpurun_out/$T/counters.txt 2>&1
grep -oE "^\s*(TA|TD|TCP)_[A-Z_]+" gpurun_out/$T/counters.txt | sort -u | head -60 > gpurun_out/$T/ta_names.txt
B="python3 bench.py --steps 2 --warmup 1 --profile-only --no-shipped $*"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --kernel-trace -d gpurun_out/$T/a -o run -- $B > gpurun_out/$T/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAVES --kernel-trace -d gpurun_out/$T/b -o run -- $B > gpurun_out/$T/b.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUSY_avr --kernel-trace -d gpurun_out/$T/c -o run -- $B > gpurun_out/$T/c.log 2>&1 || echo "TA pass failed"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/$T/d -o run -- $B > gpurun_out/$T/d.log 2>&1 || exit 1
for p in a b c d; do
  [ -f gpurun_out/$T/$p/run_results.db ] && python tools/rocpd_summary.py bykernel gpurun_out/$T/$p/run_results.db > gpurun_out/$T/$p.txt 2>&1
done
grep -h -A9 -E "${PMC_GREP:-k_solve}" gpurun_out/$T/[abcd].txt | head -${PMC_LINES:-120}
