#!/bin/bash
# round 3: configs[2] whole solve through the GPU plugin with the per-iteration log and the inertia
# cross-check at the factorizations where its trace leaves the golden one; SQ counter passes of every kernel
export TMPDIR=/tmp
mkdir -p gpurun_out/r03 gpurun_out/r03/pmc_sq
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!; trap "kill $HB" EXIT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --kernel-trace -d gpurun_out/r03/pmc_sq/a -o run -- python3 bench.py --steps 2 --warmup 1 --profile-only > gpurun_out/r03/pmc_sq/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAVES --kernel-trace -d gpurun_out/r03/pmc_sq/b -o run -- python3 bench.py --steps 2 --warmup 1 --profile-only > gpurun_out/r03/pmc_sq/b.log 2>&1 || exit 1
python tools/rocpd_summary.py bykernel gpurun_out/r03/pmc_sq/a/run_results.db > gpurun_out/r03/pmc_sq_a.txt
python tools/rocpd_summary.py bykernel gpurun_out/r03/pmc_sq/b/run_results.db > gpurun_out/r03/pmc_sq_b.txt
rm -rf gpurun_out/r03/pmc_sq/a gpurun_out/r03/pmc_sq/b
UNO_KKT_CROSSCHECK=1051,1348 timeout -k 10 800 ./oracle/_ref/uno_kkt_driver arrowband:1000000 linear_solver=HIPLDL logger=INFO > gpurun_out/r03/c3_hipldl_info.log 2> gpurun_out/r03/c3_hipldl_info.err
echo "driver rc=$?"
