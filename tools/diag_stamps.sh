# drop-in GPU tests + per-front stamps (all modes) of one C3 factorization; usage (GPU box): bash tools/diag_stamps.sh
NO_BENCH=1 bash tools/gpu_round.sh tests/test_uno_dropin.py -m gpu
for M in 1 3 4 2; do MODE=$M timeout -k 10 200 python tools/stamps.py > gpurun_out/stamps$M.log 2>&1 || exit 1; done
