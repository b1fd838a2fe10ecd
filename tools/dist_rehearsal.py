"""Rehearsal of the distributed (subtree-partitioned) factorization at bench sizes on ONE GPU: K ranks
as host threads in one process (in-process transport, same orchestration code as RCCL), one system of
K x n rows.  Checks inertia against the single-rank path and the residual of rank 0's gathered
solution, and prints per-step times (ranks share the GPU, so this is not a scaling measurement).
usage: python tools/dist_rehearsal.py [K] [n_per_rank] [steps]"""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import uno_amd
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    n_per = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    n, nv, m, r, c, v, b = uno_amd.arrowband(n_per * K, uno_amd.SEEDS["C3"])
    group = uno_amd.LocalGroup(K)
    out, errs = [None] * K, []
    barrier = threading.Barrier(K)

    def rank_main(q):
        try:
            g = uno_amd.HipKKT(0)
            g.attach_local(group, q)
            t0 = time.perf_counter()
            g.analyze(n, r, c)
            ta = time.perf_counter() - t0
            g.factorize(v)
            g.inertia()
            x = g.solve(b)
            barrier.wait()
            t0 = time.perf_counter()
            for _ in range(steps):
                g.factorize(v)
                ine = g.inertia()
                x = g.solve(b)
            barrier.wait()
            dt = (time.perf_counter() - t0) / steps
            out[q] = (ine, x, dt, ta, g.dist_info())
            g.close()
        except Exception as e:
            errs.append((q, repr(e)))

    th = [threading.Thread(target=rank_main, args=(q,)) for q in range(K)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    group.close()
    assert not errs, errs
    s = uno_amd.HipKKT(0)
    s.analyze(n, r, c)
    s.factorize(v)
    ine_s = s.inertia()
    xs = s.solve(b)
    t0 = time.perf_counter()
    for _ in range(steps):
        s.factorize(v)
        s.inertia()
        s.solve(b)
    ts = (time.perf_counter() - t0) / steps
    ine, x, dt, ta, info = out[0]
    res = np.abs(uno_amd.coo_symv(n, r, c, v, x) - b).max()
    absk = uno_amd.coo_symv(n, r, c, np.abs(v), np.ones(n)).max()
    rel = res / (absk * np.abs(x).max() + np.abs(b).max())
    print(f"K={K} n={n} inertia dist={ine} single={ine_s} rel_res={rel:.2e} max|x-xs|/|xs|="
          f"{np.abs(x - xs).max() / np.abs(xs).max():.2e} step dist={dt * 1e3:.2f} ms single={ts * 1e3:.2f} ms "
          f"analysis={ta:.2f} s info={info}", flush=True)
    assert ine == ine_s and rel < 1e-10


if __name__ == "__main__":
    main()
