"""Large-front factorization throughput (the matrix-core path, DESIGN.md 4 'Large fronts'): one dense
symmetric indefinite front of order N (every column fully summed), factored repeatedly from values
resident in HBM; F = N^3/3 flops per factorization (LDL^T, 1x1 pivots).  Inertia checked against numpy's
eigenvalues once.  Prints one JSON line; run under rocprofv3 --pmc for the MFMA-busy counters.

usage (GPU box): python tools/bigfront_bench.py [N] [reps]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    import torch
    import uno_amd
    uno_amd.load_library()
    rng = np.random.default_rng(n)
    A = rng.standard_normal((n, n))
    S = (A + A.T) / 2 + np.diag(rng.uniform(-3, 3, n))
    r, c = np.tril_indices(n)
    v = S[r, c]
    g = uno_amd.HipKKT(0)
    g.analyze(n, r.astype(np.int64), c.astype(np.int64))
    vd = torch.from_numpy(np.ascontiguousarray(v)).to("cuda:0")
    g.factorize(device_ptr=vd.data_ptr())
    inertia = g.inertia()
    check = None
    if n <= 4096:
        ev = np.linalg.eigvalsh(S)
        check = (int((ev > 0).sum()), int((ev < 0).sum()), 0)
        assert inertia == check, (inertia, check)
    torch.cuda.synchronize()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        g.factorize(device_ptr=vd.data_ptr())
        g.inertia()
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    st = g.stats()
    med = float(np.median(t))
    flops = n ** 3 / 3.0
    print(json.dumps({"workload": f"dense symmetric indefinite front, order {n}", "n": n, "reps": reps,
                      "ms_per_factorization_median": round(1e3 * med, 4),
                      "fp64_TFs": round(flops / med / 1e12, 4), "fp64_peak_TFs": 78.6,
                      "frac": round(flops / med / 1e12 / 78.6, 5), "flops_per_factorization": flops,
                      "inertia": list(inertia), "inertia_eigvalsh": list(check) if check else None,
                      "pivots_2x2": st["pivots_2x2"], "max_front": st["max_front"]}))


if __name__ == "__main__":
    main()
