# A/B of two library builds on the C3 bench line: B = the in-tree libuno_kkt.so, A = $A_LIB (UNO_KKT_LIB,
# default the in-tree one), alternated twice; A_ARGS / B_ARGS: extra bench options per side (e.g. --opt x=0);
# optional pytest selection first (PYTEST_K) on the in-tree build
set -e
export TMPDIR=/tmp
R=gpurun_out/${OUT:-ablib}
mkdir -p $R
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "$PYTEST_K" > $R/t.log 2>&1
  tail -2 $R/t.log
fi
for i in 1 2; do
  UNO_KKT_LIB=${A_LIB:-} timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} ${A_ARGS} > $R/a$i.json 2> $R/a$i.err
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} ${B_ARGS} > $R/b$i.json 2> $R/b$i.err
done
python - <<'PY'
import json, os
R = os.environ.get("OUT", "ablib")
for tag in ("a1", "b1", "a2", "b2"):
    d = json.loads(open(f"gpurun_out/{R}/{tag}.json").read().strip().splitlines()[-1])
    k = d["roofline"]["kernel_ms_per_step"]
    sp = d.get("shipped_plugin_mode") or {}
    print(tag, d["value"], d["ms_per_step"], "scale", k["scale"], "factor", k["factor_lds"], "fwd", k["solve_fwd"], "bwd", k["solve_bwd"], "shipped", sp.get("value"))
PY
