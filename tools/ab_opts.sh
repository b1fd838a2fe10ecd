#!/bin/bash
# A/B of library options on the C3 bench (one GPU): bash tools/ab_opts.sh "opt=v,opt=v" "..." ("" = defaults)
for o in "$@"; do
  echo -n "[$o] "
  UNO_KKT_OPTIONS="$o" timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | python -c '
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d["roofline"]
print(d["value"], "ms", d["ms_per_step"], {k: v for k, v in r["kernel_ms_per_step"].items() if v}, "inertia", d["config"]["inertia"])'
done
