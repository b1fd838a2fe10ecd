#!/bin/bash
# Regenerates tests/golden/hs015_uno_oracle.json: the reference Uno core (built from /root/reference by
# oracle/ref/Makefile) solving hs015 with the ipopt preset and the CPU oracle as its linear solver.
# The trajectory matches SURVEY.md 8(c)'s independent probe (17 iterations, 24 factorizations,
# 18 solves, x = (0.500000009999, 1.99999994001), f = 306.499975495).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
make -s -C "$ROOT/oracle" && make -s -j8 -C "$ROOT/oracle/ref"
"$ROOT/oracle/_ref/uno_kkt_driver" hs015 linear_solver=ORACLE logger=SILENT > "$ROOT/tests/golden/hs015_uno_oracle.json"
cat "$ROOT/tests/golden/hs015_uno_oracle.json"
