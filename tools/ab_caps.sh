#!/bin/bash
# A/B of factor size-class caps on the C3 bench (UNO_KKT_CAPS, kkt_api.cpp build_plan): bash tools/ab_caps.sh "32,64,72,128" "..."
for c in "$@"; do
  echo -n "[caps $c] "
  UNO_KKT_CAPS="$c" timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | python -c '
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d["roofline"]
print(d["value"], "ms", d["ms_per_step"], {k: v for k, v in r["kernel_ms_per_step"].items() if v}, "inertia", d["config"]["inertia"])'
done
