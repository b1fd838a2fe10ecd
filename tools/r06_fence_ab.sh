set -e
export TMPDIR=/tmp
R=gpurun_out/r06/fence
mkdir -p $R
K="test_kat_5x5 or test_scaling_bit_identical or test_c3_full_size"
UNO_KKT_LIB=ab/fixvar/libuno_kkt.so timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "$K" > $R/var_tests.log 2>&1
tail -3 $R/var_tests.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "$K" > $R/fix_tests.log 2>&1
tail -3 $R/fix_tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/fix$i.json 2> $R/fix$i.err
  UNO_KKT_LIB=ab/fixvar/libuno_kkt.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/var$i.json 2> $R/var$i.err
done
python - <<'PY'
import json
for tag in ("fix1","var1","fix2","var2"):
    d = json.loads(open(f"gpurun_out/r06/fence/{tag}.json").read().strip().splitlines()[-1])
    k = d["roofline"]["kernel_ms_per_step"]
    sp = d.get("shipped_plugin_mode") or {}
    print(tag, d["value"], d["ms_per_step"], "scale", k["scale"], "factor", k["factor_lds"], "fwd", k["solve_fwd"], "bwd", k["solve_bwd"], "shipped", sp.get("value"), sp.get("backward_error_unrefined"))
PY
