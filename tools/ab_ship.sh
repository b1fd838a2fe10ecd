# refinement-path A/B: the refinement / relaxation parity tests, a bench line, the shipped-mode timeline
set -e
export TMPDIR=/tmp
R=gpurun_out/${OUT:-abship}
mkdir -p $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "refine or relax or residual" > $R/t.log 2>&1
tail -2 $R/t.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/b.json 2> $R/b.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/trace -o run -- python3 bench.py --steps 10 --warmup 2 --profile-only --opt delay_relaxed=0 > $R/trace.log 2>&1
python tools/timeline.py $R/trace/run_results.db 2 > $R/timeline_ship.txt
rm -rf $R/trace
