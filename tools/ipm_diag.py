"""Diagnostics of the device-resident IPM-like sequence (bench.py --mode ipm, second leg): per-kernel-class
times per factorization and the library's verbose log (UNO_KKT_VERBOSE=2: per-factorization wall time,
exact refactors).  usage: UNO_KKT_VERBOSE=2 python tools/ipm_diag.py [iters]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import uno_amd
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    uno_amd.load_library()
    n, nv, m, rows, cols, vals, rhs = uno_amd.arrowband(1_000_000, uno_amd.SEEDS["C3"])
    nh = sum(min(j, 12) + 1 for j in range(nv))
    sig0 = n + nh
    dev = torch.device("cuda", 0)
    kd = uno_amd.HipKKT(0, delay_relaxed=0)
    kd.analyze(n, rows, cols)
    lbv, ubv = np.full(nv, -10.0), np.full(nv, 10.0)
    assert kd.barrier_setup(lbv, ubv) == nv
    vd = torch.from_numpy(np.array(vals)).to(dev)
    bd = torch.from_numpy(np.array(rhs)).to(dev)
    xd = torch.empty_like(bd)
    xs = torch.empty(nv, dtype=torch.float64, device=dev)
    zl, zu = torch.empty_like(xs), torch.empty_like(xs)
    gen = torch.Generator(device=dev)
    gen.manual_seed(11)
    kd.set_option("timing", 1)
    for it in range(iters + 1):
        if it == 1:
            kd.reset_kernel_times()
            t0 = time.perf_counter()
            nfac = 0
        xs.uniform_(-9.0, 9.0, generator=gen)
        zl.copy_(10.0 ** (torch.rand(nv, dtype=torch.float64, device=dev, generator=gen) * 16 - 8))
        zu.copy_(-(10.0 ** (torch.rand(nv, dtype=torch.float64, device=dev, generator=gen) * 16 - 8)))
        torch.cuda.synchronize()
        kd.assemble_barrier(xs.data_ptr(), zl.data_ptr(), zu.data_ptr(), vd.data_ptr() + 8 * sig0)
        kd.fill_values(0, n, 0.0) if it else None
        t1 = time.perf_counter()
        kd.factorize(device_ptr=vd.data_ptr())
        inertia = kd.inertia()
        print(f"it {it} fac 0: {1e3 * (time.perf_counter() - t1):.2f} ms inertia {inertia} relaxed {kd.stats()['pivots_relaxed']}", flush=True)
        nf, dw = 1, 0.0
        while inertia != (nv, m, 0) and nf < 12:
            dw = 1e-4 if dw == 0.0 else dw * (100.0 if nf > 8 else 8.0)
            kd.fill_values(0, nv, dw)
            kd.fill_values(nv, m, -1e-8)
            t1 = time.perf_counter()
            kd.factorize()
            inertia = kd.inertia()
            print(f"it {it} fac {nf}: {1e3 * (time.perf_counter() - t1):.2f} ms dw {dw:.1e} inertia {inertia} relaxed {kd.stats()['pivots_relaxed']}", flush=True)
            nf += 1
        t1 = time.perf_counter()
        kd.solve_device(bd.data_ptr(), xd.data_ptr())
        torch.cuda.synchronize()
        print(f"it {it} solve {1e3 * (time.perf_counter() - t1):.2f} ms", flush=True)
        if it:
            nfac += nf
    dt = time.perf_counter() - t0
    kt = kd.kernel_times()
    print(f"{nfac} factorizations in {1e3 * dt:.1f} ms: {1e3 * dt / nfac:.2f} ms each")
    for k, v in kt.items():
        print(f"  {k:14s} {v[0] / nfac:8.3f} ms per factorization ({v[1]} launches)")


if __name__ == "__main__":
    main()
