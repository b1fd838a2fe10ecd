#!/bin/bash
# leaf-size / block-width sweep of the C3 bench (one GPU)
CFGS=("${@}"); [ ${#CFGS[@]} -eq 0 ] && CFGS=("32 64" "48 64" "64 64")
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  echo -n "leaf=$1 block=$2 "
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --leaf $1 --block $2 2>&1 | grep -o '"value": [0-9.]*\|"nnz_L": [0-9]*\|"levels": [0-9]*\|"factor_lds": [0-9.]*\|"solve_fwd": [0-9.]*' | tr '\n' ' '
  echo
done
