# per-level factor spans / tails: the headline (delay) mode vs the plugin's relaxed mode
set -e
R=gpurun_out/shipst
mkdir -p $R
timeout -k 10 200 python tools/stamps.py > $R/delay.txt 2>&1
OPTS=delay_relaxed=0 timeout -k 10 200 python tools/stamps.py > $R/relaxed.txt 2>&1
TAILS=1 OPTS=delay_relaxed=0 timeout -k 10 200 python tools/stamps.py > $R/relaxed_tails.txt 2>&1
