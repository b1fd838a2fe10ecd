# quick parity tests + tile-kernel phase cycles + A/B against the register kernels (GPU box)
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_null_threshold.py tests/test_big_fronts.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -2 gpurun_out/quick_tests.log; [ $rc -eq 0 ] || exit $rc
MODE=5 timeout -k 10 200 python tools/stamps.py 2>&1 | grep -v amdgpu | head -5
bash tools/ab_opts.sh "" "mfma_fronts=0" "$@"
