import sys; sys.path.insert(0, "/root/repo")
import uno_amd
n, nv, m, r, c, v, b = uno_amd.arrowband(10000, uno_amd.SEEDS["C2"])
g = uno_amd.HipKKT(0, verbose=1)
g.analyze(n, r, c); g.factorize(v)
print(g.stats())
