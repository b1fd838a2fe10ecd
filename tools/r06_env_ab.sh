# Bench the C3 line under several environment settings, alternated twice:
#   OUT=name bash tools/r06_env_ab.sh "UNO_KKT_CAPS=32,64,72,128" "UNO_KKT_CAPS=32,48,64,72,128" ...
set -e
export TMPDIR=/tmp
R=gpurun_out/r06/${OUT:-envab}
mkdir -p $R
for i in 1 2; do
  j=0
  for e in "$@"; do
    j=$((j+1))
    env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/v${j}_$i.json 2> $R/v${j}_$i.err
  done
done
OUT=${OUT:-envab} python - "$@" <<'PY'
import json, os, sys
R = os.environ["OUT"]
for i in (1, 2):
    for j, e in enumerate(sys.argv[1:], 1):
        d = json.loads(open(f"gpurun_out/r06/{R}/v{j}_{i}.json").read().strip().splitlines()[-1])
        k = d["roofline"]["kernel_ms_per_step"]
        sp = d.get("shipped_plugin_mode") or {}
        print(i, e, d["value"], "factor", k["factor_lds"], "scale", k["scale"], "fwd", k["solve_fwd"], "bwd", k["solve_bwd"],
              (sp.get("backward_error_unrefined") or [None, None])[1])
PY
