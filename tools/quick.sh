#!/bin/bash
# quick GPU check: gpu tests, bench line without CPU baseline, per-front stamps (usage: tools/quick.sh tag)
T=${1:-q}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { echo TESTS FAILED; tail -n 30 gpurun_out/$T/pytest.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo BENCH FAILED; tail -n 20 gpurun_out/$T/bench.err; exit 1; }
timeout -k 10 200 python tools/stamps.py > gpurun_out/$T/stamps1.log 2>&1
python - "$T" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/{sys.argv[1]}/bench.json"))
print("value", d["value"], "ms", d["ms_per_step"], d["roofline"]["kernel_ms_per_step"], "res", d["config"]["rel_residual"])
PY
head -n 8 gpurun_out/$T/stamps1.log
