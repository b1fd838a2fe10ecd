# parity tests (scaling bit-identity, null threshold, C3) + A/B of the equilibration paths (GPU box)
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_null_threshold.py tests/test_ipm_vectors.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -3 gpurun_out/quick_tests.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED\|assert" gpurun_out/quick_tests.log | head -60; exit $rc; }
bash tools/ab_opts.sh "" "front_sweeps=0" "$@"
