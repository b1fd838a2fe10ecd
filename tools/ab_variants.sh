set -e
R=gpurun_out/ab3
mkdir -p $R
for i in 1 2; do
  for v in A v1 v2; do
    if [ $v = A ]; then L=uno_amd/libuno_kkt_A.so; else L=uno_amd/libuno_kkt_$v.so; fi
    UNO_KKT_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/$v$i.json 2> $R/$v$i.err
  done
done
python - <<'PY'
import json
for i in (1,2):
    for v in ("A","v1","v2"):
        d = json.loads(open(f"gpurun_out/ab3/{v}{i}.json").read().strip().splitlines()[-1])
        k = d["roofline"]["kernel_ms_per_step"]
        print(v, i, d["value"], "factor", k["factor_lds"], "shipped", d["shipped_plugin_mode"]["value"], d["shipped_plugin_mode"]["backward_error_unrefined"][1])
PY
