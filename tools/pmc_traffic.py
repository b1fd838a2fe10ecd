"""profiles/pmc_traffic.json from the FETCH_SIZE / WRITE_SIZE pass summaries of tools/profile_round.sh.

usage: python tools/pmc_traffic.py <pmc_fetch.json> <pmc_write.json> <out.json> [source script]
HBM bytes per factorization (factor kernel group) and per solve (solve group): FETCH_SIZE doubled
(gfx950 reports 1/2 of the bytes of wide streaming reads, MI355X_MICROARCH.md HBM section) + WRITE_SIZE,
KB = 1024 B.  bench.py reads the result as roofline.traffic / solve_roofline.traffic.
"""
import json
import sys

fe, wr, out = (json.load(open(sys.argv[1])), json.load(open(sys.argv[2])), sys.argv[3])
script = sys.argv[4] if len(sys.argv) > 4 else "tools/profile_r06.sh"
pf, pw = fe["per_run"], wr["per_run"]
kb = 1024.0
res = {
    "source": script + " (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, "
              "bench.py --steps 6 --warmup 1 --profile-only), summarised by tools/rocpd_summary.py pmc_steady "
              "and tools/pmc_traffic.py",
    "correction": "FETCH_SIZE doubled (gfx950: FETCH_SIZE tallies 1/2 of the bytes of wide streaming reads, "
                  "MI355X_MICROARCH.md HBM); WRITE_SIZE as reported; KB = 1024 B; the factor kernels' 8-byte gathers "
                  "are an uncalibrated access width, so the doubled figure is an upper bound",
    "factorizations_profiled": fe["factorizations"],
    "solves_profiled": fe["solves"],
    "factor_bytes_per_factorization": int(kb * (pf["factor"]["FETCH_SIZE_x2"] + pw["factor"]["WRITE_SIZE"])),
    "factor_bytes_raw_fetch_plus_write": int(kb * (pf["factor"]["FETCH_SIZE"] + pw["factor"]["WRITE_SIZE"])),
    "solve_bytes_per_solve": int(kb * (pf["solve"]["FETCH_SIZE_x2"] + pw["solve"]["WRITE_SIZE"])),
    "solve_bytes_raw_fetch_plus_write": int(kb * (pf["solve"]["FETCH_SIZE"] + pw["solve"]["WRITE_SIZE"])),
    "note": fe.get("note", ""),
    # bench.py uses the figures only for this workload (same n, nnz, default analysis options)
    "workload": {"n": 1000000, "nnz": 19999922, "note": "C3 (BASELINE.json configs[2]) at the library's default analysis options"},
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
