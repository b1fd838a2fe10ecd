#!/bin/bash
# round-4 quick GPU loop: parity tests (file list in $TESTS), C3 solve stamps, bench line without CPU baseline
# usage: TESTS="tests/test_gpu_parity.py" bash tools/r04_quick.sh TAG [bench args...]
T=${1:-q}; shift
mkdir -p gpurun_out/$T
TESTS=${TESTS:-tests/test_gpu_parity.py}
timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/$T/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/$T/pytest.log | head -30; exit $rc; }
timeout -k 10 200 python tools/solve_stamps.py > gpurun_out/$T/solve_stamps.log 2>&1 || { tail -20 gpurun_out/$T/solve_stamps.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/solve_stamps.log
python - "$T" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/{sys.argv[1]}/bench.json"))
r = d["roofline"]
print("value", d["value"], "ms", d["ms_per_step"], r["kernel_ms_per_step"], "solve frac", r.get("solve_roofline", {}).get("frac"), "res", d["config"]["rel_residual"], "shipped", (d.get("shipped_plugin_mode") or {}).get("value"))
PY
