"""Summaries of rocprofv3 result databases (rocpd SQLite) for profiles/.

usage: python tools/rocpd_summary.py stats <trace.db> <out.csv>
       python tools/rocpd_summary.py pmc <pmc.db> <out.json>

`stats` writes the per-kernel table of `rocprofv3 --kernel-trace --stats` (calls, total, average,
min, max in ns, share of GPU time).  `pmc` sums every counter per kernel class and divides by the
number of factorizations (k_pack dispatches) or solves (k_unscale dispatches), and records the
gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md (HBM section: FETCH_SIZE reports 1/2 of the bytes
of wide streaming reads; other access widths are uncalibrated) next to the raw number.
"""
import json
import sqlite3
import sys

GROUPS = {
    "factor": ("k_factor_lds", "k_factor_global", "k_factor_df", "k_factor_mf", "k_big_"),
    "solve": ("k_solve_fwd", "k_solve_bwd"),
    "pack": ("k_pack",),
    "scale": ("k_rowscan", "k_normmax", "k_scale_update"),
}


def group_of(name):
    for g, keys in GROUPS.items():
        if any(k in name for k in keys):
            return g
    return "other"


def stats(db, out):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows)
    with open(out, "w") as f:
        f.write("Name,Calls,TotalDurationNs,AverageNs,MinNs,MaxNs,Percentage\n")
        for n, cnt, s, a, mn, mx in rows:
            f.write(f"\"{n}\",{cnt},{s},{a:.1f},{mn},{mx},{100.0 * s / tot:.3f}\n")
    for g in GROUPS:
        s = sum(r[2] for r in rows if group_of(r[0]) == g)
        print(f"{g:8s} {s / 1e3:10.1f} us total")


def pmc(db, out):
    c = sqlite3.connect(db)
    # factorizations = k_pack dispatches, solves = k_unscale / k_xs_out dispatches (one per call)
    nfac = c.execute("select count(distinct dispatch_id) from counters_collection where kernel_name like '%k_pack%'").fetchone()[0]
    nsol = c.execute("select count(distinct dispatch_id) from counters_collection where kernel_name like '%k_unscale%' or kernel_name like '%k_xs_out%'").fetchone()[0]
    rows = c.execute("select kernel_name, counter_name, sum(value), count(*), sum(duration) "
                     "from counters_collection group by kernel_name, counter_name").fetchall()
    res = {"factorizations": nfac, "solves": nsol, "per_run": {}, "note": "KB per factorization (solve group: per solve); "
           "FETCH_SIZE_x2 applies the gfx950 1/2 correction for wide streaming reads (MI355X_MICROARCH.md, HBM)"}
    for name, cn, s, cnt, dur in rows:
        g = group_of(name)
        runs = max(1, nsol if g == "solve" else nfac)
        d = res["per_run"].setdefault(g, {})
        d[cn] = d.get(cn, 0.0) + s / runs
        if cn == "FETCH_SIZE":
            d["FETCH_SIZE_x2"] = d.get("FETCH_SIZE_x2", 0.0) + 2 * s / runs
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


def pmc_steady(db, out, skip=3):
    """As `pmc`, but per factorization / solve of the steady state only: dispatches are split into
    factorizations at every k_reset_counters dispatch (the first kernel of a factorization) and the first
    `skip` of them (warm-up, the first call's delayed-pivot merge rounds) are dropped."""
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection "
                     "order by dispatch_id").fetchall()
    starts = sorted({d for d, k, _, _ in rows if "k_reset_counters" in k or "k_sweep_front<true, false>" in k})
    import bisect
    res = {"per_run": {}, "factorizations": max(0, len(starts) - skip), "solves": 0,
           "note": f"steady state: factorizations after the first {skip} (k_reset_counters dispatches); KB per "
                   "factorization, solve group per solve; FETCH_SIZE_x2 applies the gfx950 1/2 correction"}
    solves = set()
    acc = {}
    for d, k, cn, v in rows:
        gi = bisect.bisect_right(starts, d) - 1
        if gi < skip:
            continue
        g = group_of(k)
        if g == "solve":
            solves.add(d if "k_solve_fwd" in k else None)
        acc.setdefault(g, {}).setdefault(cn, 0.0)
        acc[g][cn] += v
    nsol = len([x for x in solves if x is not None])
    res["solves"] = nsol
    nfac = max(1, res["factorizations"])
    for g, d in acc.items():
        runs = max(1, nsol if g == "solve" else nfac)
        res["per_run"][g] = {cn: v / runs for cn, v in d.items()}
        if "FETCH_SIZE" in d:
            res["per_run"][g]["FETCH_SIZE_x2"] = 2 * d["FETCH_SIZE"] / runs
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


def bykernel(db):
    """per kernel name: every counter summed over its dispatches, divided by the dispatch count"""
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, counter_name, sum(value), count(distinct dispatch_id) "
                     "from counters_collection group by kernel_name, counter_name order by kernel_name").fetchall()
    cur = None
    for name, cn, s, cnt in rows:
        if name != cur:
            cur = name
            print(f"{name[:70]}  ({cnt} dispatches)")
        print(f"    {cn:28s} {s / max(cnt, 1):16.0f} per dispatch")


if __name__ == "__main__":
    if sys.argv[1] == "pmc_steady":
        pmc_steady(sys.argv[2], sys.argv[3])
        sys.exit(0)
    if sys.argv[1] == "bykernel":
        bykernel(sys.argv[2])
    elif sys.argv[1] == "stats":
        stats(sys.argv[2], sys.argv[3])
    else:
        pmc(sys.argv[2], sys.argv[3])
