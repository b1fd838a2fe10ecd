mkdir -p gpurun_out/r04base
timeout -k 10 200 python tools/solve_stamps.py > gpurun_out/r04base/solve_stamps.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r04base/bench.json 2> gpurun_out/r04base/bench.err
rc=$?; cat gpurun_out/r04base/solve_stamps.log; exit $rc
