"""Diagnostics on the GPU: residuals / pivot statistics for the parity failure cases."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import uno_amd
from oracle_ffi import OracleKKT
from test_gpu_parity import random_sym

def run(n, r, c, v, b, S=None, **opt):
    g = uno_amd.HipKKT(0, **opt)
    g.analyze(n, r, c)
    g.factorize(v)
    try:
        ine = g.inertia()
    except Exception as e:
        print("  ERR", e); return
    x = g.solve(b)
    res = np.abs(uno_amd.coo_symv(n, r, c, v, x) - b).max()
    st = g.stats()
    print(f"  opt={opt} inertia={ine} res={res:.2e} 2x2={st['pivots_2x2']} relaxed={st['pivots_relaxed']} "
          f"merged={st['fronts_merged']} fronts={st['n_fronts']} maxfront={st['max_front']}")

for nmax, dens in [(40, 0.3), (150, 0.05), (300, 0.6)]:
    rng = np.random.default_rng(nmax)
    for trial in range(12):
        n = int(rng.integers(max(2, nmax // 3), nmax + 1))
        rr, cc, vv, S = random_sym(rng, n, dens, zero_diag_frac=0.5)
        ev = np.linalg.eigvalsh(S)
        if np.min(abs(ev)) < 1e-8 * max(1.0, abs(ev).max()):
            continue
        b = rng.standard_normal(n)
        o = OracleKKT(); o.analyze(n, rr, cc); o.factorize(vv)
        print(f"case nmax={nmax} n={n} expect={(int((ev>0).sum()), int((ev<0).sum()))} oracle={o.inertia()} {o.stats()}")
        run(n, rr, cc, vv, b)
        run(n, rr, cc, vv, b, delay_relaxed=1)
        run(n, rr, cc, vv, b, scale_iters=0)
        run(n, rr, cc, vv, b, max_block=1024, leaf_size=100000)
        break
n, nv, m, r, c, v, b = uno_amd.arrowband(10000, uno_amd.SEEDS["C2"])
print("C2")
run(n, r, c, v, b)
run(n, r, c, v, b, delay_relaxed=1)
run(n, r, c, v, b, scale_iters=0)
run(n, r, c, v, b, pivot_threshold=0.1)
