"""Factor timing with and without the dataflow upper-tree factorization (C3 by default)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import uno_amd
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
N, nv, m, r, c, v, b = uno_amd.arrowband(n, uno_amd.SEEDS["C3"])
for dff in (2, 1, 0):
    g = uno_amd.HipKKT(0, verbose=1, dataflow_factor=dff)
    g.analyze(N, r, c)
    g.factorize(v); g.inertia()
    g.set_option("timing", 1)
    g.reset_kernel_times()
    for _ in range(5):
        g.factorize(v); g.inertia()
    kt = g.kernel_times()
    st = g.stats()
    print(f"dataflow_factor={dff} df_fronts={st['factor_df_fronts']} aborts={st['factor_df_aborts']} inertia={g.inertia()}",
          {k: round(v[0] / max(1, 5), 4) for k, v in kt.items() if v[0] > 0})
    g.close()
