# kernel trace of the C3 bench (3 steps): bash tools/ktrace_r06.sh TAG [bench args]; stats -> gpurun_out/r06/kt_TAG
set -e
export TMPDIR=/tmp
T=${1:-kt}; shift || true
R=gpurun_out/r06/kt_$T
mkdir -p $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline "$@" > $R/bench.log 2>&1
python3 tools/rocpd_summary.py stats $R/run_results.db $R/kernel_stats.csv

python3 - "$R/kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{float(r["AverageNs"])/1e3:9.1f} us avg  x{r["Calls"]:>5}  {r["Name"][:90]}')
PY
