"""Phase times of the register panel's exact steps inside the a-posteriori large-front path (option
stamps=6): dense symmetric indefinite front of order N, one factorization."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import uno_amd
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
rng = np.random.default_rng(n)
A = rng.standard_normal((n, n))
S = (A + A.T) / 2 + np.diag(rng.uniform(-3, 3, n))
r, c = np.tril_indices(n)
g = uno_amd.HipKKT(0)
g.analyze(n, r.astype(np.int64), c.astype(np.int64))
v = np.ascontiguousarray(S[r, c])
g.factorize(v); g.inertia()
g.set_option("stamps", 6)
g.factorize(v); print("inertia", g.inertia())
nf = g.stats()["n_fronts"]
out = np.zeros(8 * nf, dtype=np.uint64)
fm = np.zeros(nf, dtype=np.int32); fp = np.zeros(nf, dtype=np.int32); fl = np.zeros(nf, dtype=np.int32)
g.lib.uno_kkt_debug_stamps.restype = ctypes.c_int64
P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
g.lib.uno_kkt_debug_stamps(g.h, P(out), ctypes.c_int64(len(out)), P(fm), P(fp), P(fl))
st = out.reshape(nf, 8).astype(np.int64)
f = int(np.argmax(fm))
calls = st[f, 4]
names = ["quick test + exact search + swaps", "register panel load + exact terms", "quick steps", "write-back"]
print(f"front {f} (m = {fm[f]}): {calls} exact steps")
for ph in range(4):
    print(f"  {names[ph]:36s} {st[f, ph] * 1e-2 / 1e3:8.3f} ms total  {st[f, ph] * 1e-2 / max(calls, 1):8.2f} us per step")
