#!/bin/bash
# A/B lines of the C3 bench: bash tools/ab3.sh "label|--opt a=1 --opt b=2" ...   (first: parity tests)
mkdir -p gpurun_out/ab3
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!; trap "kill $HB" EXIT
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/ab3/tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab3/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for spec in "$@"; do
  label=${spec%%|*}; args=${spec#*|}
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-shipped $args > gpurun_out/ab3/$label.json 2> gpurun_out/ab3/$label.err || { echo "$label failed"; tail -5 gpurun_out/ab3/$label.err; exit 1; }
  python - "$label" <<'PY'
import json, sys
l = sys.argv[1]
d = json.loads(open(f"gpurun_out/ab3/{l}.json").read().strip().splitlines()[-1])
k = d["roofline"]["kernel_ms_per_step"]
print(f"{l:14s} {d['value']:8.2f}/s  {d['ms_per_step']:.4f} ms | scale {k['scale']:.4f} factor {k['factor_lds']:.4f} fwd {k['solve_fwd']:.4f} bwd {k['solve_bwd']:.4f}")
PY
done
