#!/bin/bash
# timing probe: factorization with p = 0 in every front (assembly + contribution-block write only)
mkdir -p gpurun_out/nopiv
for v in 0 1 3 5 7 15; do
  UNO_KKT_DIAG_NOPIV=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-shipped > gpurun_out/nopiv/v$v.json 2> gpurun_out/nopiv/v$v.err
  python -c "import json; d=json.loads(open('gpurun_out/nopiv/v$v.json').read().strip().splitlines()[-1]); k=d['roofline']['kernel_ms_per_step']; print('nopiv=$v factor', k['factor_lds'], 'scale', k['scale'])" || tail -3 gpurun_out/nopiv/v$v.err
done
