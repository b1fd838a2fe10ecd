"""Front shapes after the delay-merge rounds of the first C3 factorization (delay_relaxed = 1): how many fronts
leave the one-wave register solve class (p <= 32, m <= 72), at which levels."""
import ctypes, sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import uno_amd
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
N, nv, m, r, c, v, b = uno_amd.arrowband(n, uno_amd.SEEDS["C3"])
g = uno_amd.HipKKT(0)
g.analyze(N, r, c)
g.factorize(v); g.inertia()
st = g.stats()
nf = st["n_fronts"]
fo = np.zeros(nf, np.int32); fp = np.zeros(nf, np.int32); fl = np.zeros(nf, np.int32)
P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
g.lib.uno_kkt_debug_front_info.restype = ctypes.c_int64
assert g.lib.uno_kkt_debug_front_info(g.h, P(fo), P(fp), P(fl), ctypes.c_int64(nf)) == nf
print("fronts", nf, "merged", st["fronts_merged"], "max m", fo.max(), "max p", fp.max())
big = (fo > 72) | (fp > 32)
print("outside p<=32,m<=72:", big.sum())
for L in np.unique(fl[big]):
    q = big & (fl == L)
    print(f"  level {L}: {q.sum()} fronts, m {fo[q].min()}..{fo[q].max()}, p {fp[q].min()}..{fp[q].max()}")
print("m>64:", (fo > 64).sum(), " p hist (>32):", np.bincount(fp[fp > 32])[33:].tolist() if (fp > 32).any() else [])
