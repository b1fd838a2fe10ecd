"""Timeline of one steady-state factor+solve step from a rocprofv3 kernel-trace database: every kernel's start
and end relative to the step's first kernel, and the idle gaps (no kernel running) longer than 2 us.
usage: python tools/timeline.py <run_results.db> [step index from the end, default 2]"""
import sqlite3
import sys

db = sys.argv[1]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)").fetchall()]
s_col = "start" if "start" in cols else [x for x in cols if "start" in x][0]
e_col = "end" if "end" in cols else [x for x in cols if x.endswith("end")][0]
rows = c.execute(f"select name, {s_col}, {e_col} from kernels order by {s_col}").fetchall()
# a factorization's first kernel: k_reset_counters, or the first equilibration sweep that resets the counters
starts = [i for i, r in enumerate(rows) if "k_reset_counters" in r[0] or "k_sweep_front<true, false>" in r[0]]
i0 = starts[-back]
i1 = starts[-back + 1] if back > 1 else len(rows)
seg = rows[i0:i1]
t0 = seg[0][1]
busy_end = t0
print(f"{'start_us':>9} {'end_us':>9} {'dur_us':>8}  kernel")
for name, s, e in seg:
    if s - busy_end > 2000:
        print(f"{'':>9} {'':>9} {(s - busy_end) / 1e3:8.1f}  -- idle --")
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {name[:90]}")
    busy_end = max(busy_end, e)
print(f"step span {(busy_end - t0) / 1e3:.1f} us")
