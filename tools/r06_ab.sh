# A/B of the in-tree library (B) against $A_LIB (A) on the C3 bench line, alternated twice, after the parity files
# given in $TESTS (B_LIB: another library as B) (default: the GPU parity suite + null threshold):  OUT=name A_LIB=ab/x/libuno_kkt.so bash tools/r06_ab.sh
set -e
export TMPDIR=/tmp
R=gpurun_out/r06/${OUT:-ab}
mkdir -p $R
( while true; do date >> $R/heartbeat.log; sleep 30; done ) &  # long tests print nothing for minutes
HB=$!; trap "kill $HB" EXIT
TESTS=${TESTS:-tests/test_gpu_parity.py tests/test_null_threshold.py}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread $TESTS > $R/t.log 2>&1
  tail -2 $R/t.log
fi
for i in 1 2; do
  UNO_KKT_LIB=${A_LIB} timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} ${A_ARGS} > $R/a$i.json 2> $R/a$i.err
  UNO_KKT_LIB=${B_LIB} timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} ${B_ARGS} > $R/b$i.json 2> $R/b$i.err
done
OUT=${OUT:-ab} python - <<'PY'
import json, os
R = os.environ["OUT"]
for tag in ("a1", "b1", "a2", "b2"):
    d = json.loads(open(f"gpurun_out/r06/{R}/{tag}.json").read().strip().splitlines()[-1])
    k = d["roofline"]["kernel_ms_per_step"]
    sp = d.get("shipped_plugin_mode") or {}
    print(tag, d["value"], d["ms_per_step"], "scale", k["scale"], "factor", k["factor_lds"], "fwd", k["solve_fwd"], "bwd", k["solve_bwd"],
          "shipped", sp.get("value"), (sp.get("backward_error_unrefined") or [None, None])[1])
PY
