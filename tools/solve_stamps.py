"""Per-level phase timings (start -> dependency met + values staged -> compute issued -> published) of one C3 dataflow solve (option solve_stamps=1): time from a front's
start to its dependency being met, to its values being staged, to its publication; plus the
per-level span (first start to last publication) in each direction."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import uno_amd
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
N, nv, m, r, c, v, b = uno_amd.arrowband(n, uno_amd.SEEDS["C3"])
g = uno_amd.HipKKT(0)
g.analyze(N, r, c)
g.factorize(v); g.inertia()
g.solve(b)
g.set_option("solve_stamps", 1)
g.solve(b); g.solve(b)
lib = g.lib
nf = g.stats()["n_fronts"]
out = np.zeros(8 * nf, dtype=np.uint64)
lib.uno_kkt_debug_solve_stamps.restype = ctypes.c_int64
k = lib.uno_kkt_debug_solve_stamps(g.h, out.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(len(out)))
assert k == nf, k
st = out.reshape(nf, 8).astype(np.int64)
fo = np.zeros(nf, np.int32); fp = np.zeros(nf, np.int32); fl = np.zeros(nf, np.int32)
P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
lib.uno_kkt_debug_front_info.restype = ctypes.c_int64
nf2 = lib.uno_kkt_debug_front_info(g.h, P(fo), P(fp), P(fl), ctypes.c_int64(nf))
assert nf2 == nf, (nf2, nf)
levels = fl
for d, name in ((0, "forward"), (4, "backward")):
    s = st[:, d:d + 4]
    t0 = s[:, 0].min()
    print(f"{name}: total {(s[:, 3].max() - t0) * 1e-2:8.1f} us")
    for L in range(levels.max() + 1):
        q = levels == L
        if not q.any():
            continue
        w = (s[q, 1] - s[q, 0]) * 1e-2; stg = (s[q, 2] - s[q, 1]) * 1e-2; cmp_ = (s[q, 3] - s[q, 2]) * 1e-2
        print(f"  level {L:2d} fronts {q.sum():6d} wait+stage {w.mean():6.2f} prefetch-issue {stg.mean():6.2f} compute {cmp_.mean():6.2f} us"
              f" | start {(s[q, 0].min() - t0) * 1e-2:7.1f} .. end {(s[q, 3].max() - t0) * 1e-2:7.1f} us")
