#!/bin/bash
# configs[2] whole Uno solve (ipopt preset, arrowband:1000000) through the plugin: shipped options, then
# delay_relaxed=1 (MUMPS delays); JSON incl. host_profile_s per run in gpurun_out/whole_r04/
mkdir -p gpurun_out/whole_r04
( while true; do date >> gpurun_out/whole_r04/heartbeat.log; sleep 30; done ) &
HB=$!; trap "kill $HB" EXIT
for o in "" "delay_relaxed=1"; do
  t=${o:-shipped}
  s=$(date +%s.%N)
  UNO_KKT_OPTIONS="$o" timeout -k 10 560 ./oracle/_ref/uno_kkt_driver arrowband:1000000 linear_solver=HIPLDL logger=SILENT > gpurun_out/whole_r04/$t.json 2> gpurun_out/whole_r04/$t.err || { echo "FAILED $t"; tail -5 gpurun_out/whole_r04/$t.err; exit 1; }
  e=$(date +%s.%N)
  echo "$t wall $(python -c "print(round($e - $s, 2))") s"
  python - gpurun_out/whole_r04/$t.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print({k: d.get(k) for k in ("status", "iterations", "factorizations", "solves", "host_profile_s", "kkt_stats") if k in d})
PY
done
