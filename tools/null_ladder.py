"""Rank-deficient large fronts (tests/test_big_fronts.py::test_rank_deficient_duplicated_rows matrices): the
inertia the GPU and the CPU oracle report at null-pivot thresholds null_tol_factor x MUMPS's default
(eps * 1e-5 * ||A_pre||_inf, ICNTL(24)=1), against numpy's; prints one JSON line per (n, k, factor).  Documents
the tightest threshold both solvers meet."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import uno_amd
    from oracle_ffi import OracleKKT
    uno_amd.load_library()
    for n, k in ((300, 6), (700, 10)):
        rng = np.random.default_rng(7 * n + k)
        A = rng.standard_normal((n, n))
        S = (A + A.T) / 2 + np.diag(rng.uniform(-3, 3, n))
        idx = rng.permutation(n)
        for s_, d_ in zip(idx[:k], idx[k:2 * k]):
            S[d_, :] = S[s_, :]
            S[:, d_] = S[:, s_]
        rr, cc = np.tril_indices(n)
        ev = np.linalg.eigvalsh(S)
        anorm = np.abs(S).sum(1).max()
        tol = 1e-10 * anorm
        expect = (int((ev > tol).sum()), int((ev < -tol).sum()), k)
        for fac in (1.0, 1e1, 1e2, 1e3, 1e4):
            g = uno_amd.HipKKT(0, null_tol_factor=fac)
            g.analyze(n, rr, cc)
            g.factorize(S[rr, cc])
            o = OracleKKT(null_tol_factor=fac)
            o.analyze(n, rr, cc)
            o.factorize(S[rr, cc])
            print(json.dumps({"n": n, "k": k, "null_tol_factor": fac, "numpy": expect, "gpu": g.inertia(),
                              "oracle": o.inertia(), "gpu_ok": g.inertia() == expect, "oracle_ok": o.inertia() == expect}),
                  flush=True)


if __name__ == "__main__":
    main()
