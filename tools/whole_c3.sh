#!/bin/bash
# configs[2] whole Uno solve (ipopt preset, arrowband:1000000) through the plugin, once per option set given
# as arguments (UNO_KKT_OPTIONS format; "" = the shipped plugin); JSON incl. host_profile_s per run in
# gpurun_out/${OUT:-whole}/.  Environment variables for the driver can be prefixed as VAR=value;... ahead of
# the option set, separated by '|': e.g. "UNO_HIPLDL_STAGE=0|"
mkdir -p gpurun_out/${OUT:-whole}
( while true; do date >> gpurun_out/${OUT:-whole}/heartbeat.log; sleep 30; done ) &
HB=$!; trap "kill $HB" EXIT
[ $# -eq 0 ] && set -- ""
for spec in "$@"; do
  envs=""; o="$spec"
  case "$spec" in *"|"*) envs="${spec%%|*}"; o="${spec#*|}";; esac
  t=$(echo "${envs}_${o}" | tr -c 'A-Za-z0-9=_.
' '_'); [ "$t" = "_" ] && t=shipped
  s=$(date +%s.%N)
  env $envs UNO_KKT_OPTIONS="$o" timeout -k 10 700 ./oracle/_ref/uno_kkt_driver arrowband:1000000 linear_solver=HIPLDL logger=SILENT > gpurun_out/${OUT:-whole}/$t.json 2> gpurun_out/${OUT:-whole}/$t.err || { echo "FAILED $t"; tail -5 gpurun_out/${OUT:-whole}/$t.err; exit 1; }
  e=$(date +%s.%N)
  echo "$t wall $(python -c "print(round($e - $s, 2))") s"
  python - gpurun_out/${OUT:-whole}/$t.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print({k: d.get(k) for k in ("status", "iterations", "factorizations", "solves", "host_profile_s", "kkt_stats") if k in d})
PY
done
