#!/bin/bash
# Golden traces of the reference Uno core (libuno built from /root/reference by oracle/ref/Makefile)
# with the oracle plugin (linear_solver=ORACLE) on the reference's example .nl files, read by the
# ASL-free reader integration/models/NLModel.hpp.  hs015.nl / polak5.nl are copies of
# /root/reference/examples/*.nl (model data).  Run from the repository root after `make -C oracle/ref`.
set -e
for m in hs015 polak5; do
  oracle/_ref/uno_kkt_driver tests/golden/$m.nl linear_solver=ORACLE logger=SILENT | grep '^{' | tail -n 1 \
    | sed "s#\"model\": \"tests/golden/$m.nl\"#\"model\": \"$m.nl\"#" > tests/golden/${m}_nl_uno_oracle.json
done
# configs[1]: the synthetic arrowband NLP of KKT dimension 1e4 (integration/models/ArrowbandModel.hpp)
oracle/_ref/uno_kkt_driver arrowband:10000 linear_solver=ORACLE logger=SILENT | grep '^{' | tail -n 1 \
  > tests/golden/arrowband10000_uno_oracle.json
# the inequality-constrained variant (-1 <= A x - b <= 1: slacks in the ipopt preset), SURVEY 8(f) item 4
oracle/_ref/uno_kkt_driver arrowband_ineq:10000 linear_solver=ORACLE logger=SILENT | grep '^{' | tail -n 1 \
  > tests/golden/arrowband_ineq10000_uno_oracle.json
# n = 1e5 (4.5 min on one core; compared by the GPU test only) and its inequality-constrained variant
# (configs[3] fallback at the stated size); both in parallel
oracle/_ref/uno_kkt_driver arrowband:100000 linear_solver=ORACLE logger=SILENT | grep '^{' | tail -n 1 \
  > tests/golden/arrowband100000_uno_oracle.json &
oracle/_ref/uno_kkt_driver arrowband_ineq:100000 linear_solver=ORACLE logger=SILENT | grep '^{' | tail -n 1 \
  > tests/golden/arrowband_ineq100000_uno_oracle.json &
wait
[ "${1:-}" = "--no-convexify" ] && exit 0
# byrd-preset Hessian convexification (PrimalRegularization::regularize_hessian on the l1-relaxed problem's
# Hessian at a fixed sequence of points; driver mode convexify:<model>)
python3 - <<'PY'
import json, subprocess
out = {}
for m in ("tests/golden/hs015.nl", "tests/golden/polak5.nl", "arrowband:10000", "arrowband_ineq:10000", "arrowband:100000",
          "arrowband:1000000"):
    r = subprocess.run(["oracle/_ref/uno_kkt_driver", "convexify:" + m, "linear_solver=ORACLE", "logger=SILENT"],
                       capture_output=True, text=True, check=True)
    out[m.replace("tests/golden/", "")] = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
json.dump(out, open("tests/golden/convexify_uno_oracle.json", "w"), indent=0)
PY
