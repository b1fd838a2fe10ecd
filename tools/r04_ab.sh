#!/bin/bash
# GPU tests (file list in $TESTS), then per option set: solve stamps + bench line (usage: tools/r04_ab.sh TAG "opts A" "opts B" ...)
# an option set is a comma list name=value (UNO_KKT_OPTIONS format), "" = defaults
T=${1:-ab}; shift
mkdir -p gpurun_out/$T
TESTS=${TESTS:-tests/test_gpu_parity.py}
timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/$T/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/$T/pytest.log | head -30; exit $rc; }
i=0
for o in "$@"; do
  i=$((i+1))
  UNO_KKT_OPTIONS="$o" timeout -k 10 200 python tools/solve_stamps.py > gpurun_out/$T/stamps$i.log 2>&1 || { tail -20 gpurun_out/$T/stamps$i.log; exit 1; }
  UNO_KKT_OPTIONS="$o" timeout -k 10 300 python bench.py --no-cpu-baseline --no-shipped > gpurun_out/$T/bench$i.json 2> gpurun_out/$T/bench$i.err || { tail -20 gpurun_out/$T/bench$i.err; exit 1; }
  echo "== [$o]"; grep -E "total|level  [0-3] |level 17" gpurun_out/$T/stamps$i.log
  python - "$T" "$i" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/{sys.argv[1]}/bench{sys.argv[2]}.json"))
r = d["roofline"]
print("value", d["value"], "ms", d["ms_per_step"], r["kernel_ms_per_step"], "solve frac", r.get("solve_roofline", {}).get("frac"))
PY
done
