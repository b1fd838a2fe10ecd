# SQ counters of the factor kernels (one rocprofv3 --pmc pass each): bash tools/pmc_sq.sh [extra bench args]
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_sq
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --kernel-trace -d gpurun_out/pmc_sq/a -o run -- python3 bench.py --steps 2 --warmup 1 --profile-only "$@" > gpurun_out/pmc_sq/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAVES --kernel-trace -d gpurun_out/pmc_sq/b -o run -- python3 bench.py --steps 2 --warmup 1 --profile-only "$@" > gpurun_out/pmc_sq/b.log 2>&1 || exit 1
python tools/rocpd_summary.py bykernel gpurun_out/pmc_sq/a/run_results.db | grep -A8 "factor"
python tools/rocpd_summary.py bykernel gpurun_out/pmc_sq/b/run_results.db | grep -A8 "factor"
