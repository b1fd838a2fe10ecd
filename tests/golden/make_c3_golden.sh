#!/bin/bash
# configs[2] golden trace: the reference Uno core (oracle/ref/Makefile, compiled from /root/reference) solving
# the synthetic arrowband NLP of KKT dimension 1e6 (nnz 2e7) under the ipopt preset with the CPU oracle
# (MUMPS semantics, oracle/kkt_oracle.c) as its linear solver.  Container CPU time only (about 1.5-2 h on one
# core); tests/test_uno_dropin.py::test_hipldl_plugin_arrowband_1e6 requires the GPU plugin to reproduce it.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
make -s -C "$ROOT/oracle" && make -s -j8 -C "$ROOT/oracle/ref"
"$ROOT/oracle/_ref/uno_kkt_driver" arrowband:1000000 linear_solver=ORACLE logger=SILENT | grep '^{' | tail -n 1 \
  > "$ROOT/tests/golden/arrowband1000000_uno_oracle.json"
# the same with the oracle's second ordering (Cuthill-McKee, not reversed): at this size the iterate sequence
# depends on the ordering's rounding; both runs are reference traces
UNO_ORACLE_ORDERING=1 "$ROOT/oracle/_ref/uno_kkt_driver" arrowband:1000000 linear_solver=ORACLE logger=SILENT | grep '^{' | tail -n 1 \
  | python3 -c "import json, sys; d = json.loads(sys.stdin.read()); d.pop('crosscheck', None); print(json.dumps(d))" \
  > "$ROOT/tests/golden/arrowband1000000_uno_oracle_cm.json"
