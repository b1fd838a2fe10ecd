"""Componentwise backward error of one C3 solve with the register solve kernels (solve_rg = 1) and the LDS-panel
kernels (solve_rg = 0), and the largest difference between the two solutions."""
import sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import uno_amd
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
N, nv, m, r, c, v, b = uno_amd.arrowband(n, uno_amd.SEEDS["C3"])
def omega(x):
    res = np.abs(uno_amd.coo_symv(N, r, c, v, x) - b)
    den = uno_amd.coo_symv(N, r, c, np.abs(v), np.abs(x)) + np.abs(b)
    w = np.where(den > 0, res / np.where(den > 0, den, 1.0), 0.0)
    i = int(np.argmax(w))
    return float(w[i]), i
xs = {}
for rg in (1, 0):
    g = uno_amd.HipKKT(0, solve_rg=rg)
    g.analyze(N, r, c)
    g.factorize(v)
    x = g.solve(b)
    xs[rg] = x
    print("solve_rg", rg, "inertia", g.inertia(), "omega", omega(x))
d = np.abs(xs[1] - xs[0])
print("max |x1 - x0|", d.max(), "at", int(np.argmax(d)), "rel", d.max() / np.abs(xs[0]).max())
