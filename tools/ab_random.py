import numpy as np, sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), 'tests'))
import uno_amd
uno_amd.load_library()
from test_gpu_parity import random_sym, both
rng = np.random.default_rng(300)
for trial in range(12):
    n = int(rng.integers(100, 301))
    rr, cc, vv, S = random_sym(rng, n, 0.6, zero_diag_frac=0.5)
    ev = np.linalg.eigvalsh(S)
    if np.min(abs(ev)) < 1e-8 * max(1.0, abs(ev).max()):
        continue
    g, o = both(n, rr, cc, vv)
    b = rng.standard_normal(n)
    xg = g.solve(b)
    print(os.environ.get("UNO_KKT_LIB", "default"), trial, n, g.inertia() == o.inertia(), float(np.abs(S @ xg - b).max()), g.stats()["pivots_2x2"])
