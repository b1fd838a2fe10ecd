#!/bin/bash
# GPU tests, then the C3 bench line for each extra-argument set (usage: tools/ab.sh tag "args A" "args B" ...)
T=${1:-ab}; shift
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { echo TESTS FAILED; tail -n 40 gpurun_out/$T/pytest.log; exit 1; }
tail -n 2 gpurun_out/$T/pytest.log
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu-baseline $a > gpurun_out/$T/bench$i.json 2> gpurun_out/$T/bench$i.err || { echo "BENCH FAILED ($a)"; tail -n 20 gpurun_out/$T/bench$i.err; exit 1; }
  python - "$T" "$i" "$a" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/{sys.argv[1]}/bench{sys.argv[2]}.json"))
print(sys.argv[3], "| value", d["value"], "ms", d["ms_per_step"], d["roofline"]["kernel_ms_per_step"], "res", d["config"]["rel_residual"], d["config"].get("solve_schedule"))
PY
done
