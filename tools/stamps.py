"""Per-front phase timings of one C3 factorization (diagnostic build path, option stamps=1)."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import uno_amd
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
N, nv, m, r, c, v, b = uno_amd.arrowband(n, uno_amd.SEEDS["C3"])
g = uno_amd.HipKKT(0)
if os.environ.get("LEAF"):
    g.set_option("leaf_size", int(os.environ["LEAF"]))
for kv in filter(None, os.environ.get("OPTS", "").split(",")):  # e.g. OPTS=delay_relaxed=0 (the plugin's mode)
    k_, v_ = kv.split("=")
    g.set_option(k_, float(v_))
g.analyze(N, r, c)
g.factorize(v); g.inertia()
g.set_option("stamps", int(os.environ.get("MODE", "1")))
g.factorize(v); g.inertia()
lib = g.lib
nf = g.stats()["n_fronts"]
out = np.zeros(8 * nf, dtype=np.uint64)
fm = np.zeros(nf, dtype=np.int32); fp = np.zeros(nf, dtype=np.int32); fl = np.zeros(nf, dtype=np.int32)
lib.uno_kkt_debug_stamps.restype = ctypes.c_int64
P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
k = lib.uno_kkt_debug_stamps(g.h, P(out), ctypes.c_int64(len(out)), P(fm), P(fp), P(fl))
st = out.reshape(nf, 8).astype(np.int64)
asm = (st[:, 1] - st[:, 0]) * 10e-3   # us
loop = (st[:, 2] - st[:, 1]) * 10e-3
wout = (st[:, 3] - st[:, 2]) * 10e-3
cs = st[:, 4]; cu = st[:, 5]; cr = st[:, 6]; steps = np.maximum(st[:, 7], 1)
print("fronts", nf, "levels", fl.max() + 1)
if os.environ.get("MODE") == "2":
    w = (st[:, 4:8] - st[:, [2, 4, 5, 6]]) * 10e-3
    for lev in range(fl.max() + 1):
        s = fl == lev
        print(f"level {lev:2d} fronts {s.sum():6d} m {fm[s].mean():6.1f} | write: coef {w[s,0].mean():6.2f} L {w[s,1].mean():6.2f} "
              f"rows {w[s,2].mean():6.2f} cb {w[s,3].mean():6.2f} tail {((st[s,3]-st[s,7])*10e-3).mean():6.2f} us")
    sys.exit(0)
if os.environ.get("MODE") == "4":
    for lev in range(fl.max() + 1):
        s = fl == lev
        a0 = (st[s, 4] - st[s, 0]) * 10e-3
        a1 = (st[s, 5] - st[s, 4]) * 10e-3
        a2 = (st[s, 6] - st[s, 5]) * 10e-3
        print(f"level {lev:2d} m {fm[s].mean():5.1f} | assembly: rows+zero {a0.mean():6.2f} entries {a1.mean():6.2f} "
              f"children {a2.mean():6.2f} us (total {asm[s].mean():6.2f})")
    sys.exit(0)
if os.environ.get("MODE") == "5":  # tile kernels: shader cycles per front of each phase
    for lev in range(fl.max() + 1):
        s = fl == lev
        c = st[s, 4:8].astype(np.float64)
        print(f"level {lev:2d} m {fm[s].mean():5.1f} p {fp[s].mean():5.1f} | cycles/front: extract {c[:,0].mean():7.0f} "
              f"pivots {c[:,1].mean():7.0f} stage+mfma {c[:,2].mean():7.0f} lds-steps {c[:,3].mean():7.0f} | "
              f"assemble {asm[s].mean():6.2f} loop {loop[s].mean():6.2f} write {wout[s].mean():5.2f} us")
    sys.exit(0)
if os.environ.get("MODE") == "8":  # LDS-path pivot steps by phase (a UKKT_STEP_STAMPS build)
    n_l = st[:, 7] >> 40
    for lev in range(fl.max() + 1):
        s = fl == lev
        nl = n_l[s].astype(np.float64)
        tot = nl.sum()
        per = lambda col: (st[s, col].sum() / max(tot, 1))
        rel = ((st[s, 7] & 0xffffffffff).sum() / max(tot, 1))
        print(f"level {lev:2d} m {fm[s].mean():5.1f} p {fp[s].mean():5.1f} | LDS steps/front {nl.mean():5.2f} | cycles per LDS step: "
              f"spill {per(4):6.0f} search {per(5):6.0f} swap+update {per(6):6.0f} reload {rel:6.0f} | loop {loop[s].mean():6.2f} us")
    if os.environ.get("TAILS"):  # the slowest loops per level: LDS steps and their cycles (totals per front)
        for lev in range(fl.max() + 1):
            s = np.nonzero(fl == lev)[0]
            o = s[np.argsort(-loop[s])[:3]]
            print(f"level {lev:2d} slowest loops: " + ", ".join(
                f"f{f} m{fm[f]} p{fp[f]} loop {loop[f]:.1f} us LDS steps {n_l[f]} spill {st[f,4]} search {st[f,5]} "
                f"upd {st[f,6]} reload {st[f,7] & 0xffffffffff}" for f in o))
    sys.exit(0)
if os.environ.get("MODE") == "9":  # a UKKT_STEP_STAMPS build: shader cycles (2.4 GHz, tools/clk) of the loop phase
    for lev in range(fl.max() + 1):
        s = fl == lev
        c = st[s, 4:8].astype(np.float64) / 2400.0  # us
        print(f"level {lev:2d} m {fm[s].mean():5.1f} p {fp[s].mean():5.1f} | reg_load {c[:,0].mean():6.2f} pivot loop {c[:,1].mean():6.2f} "
              f"early CB+drain {c[:,2].mean():6.2f} bookkeeping+L {c[:,3].mean():6.2f} us | loop phase {loop[s].mean():6.2f} us")
    sys.exit(0)
if os.environ.get("MODE") == "11":  # dataflow hand-off: child signalled -> parent sees it -> children assembled
    par = np.full(nf, -1, dtype=np.int64)
    lib.uno_kkt_debug_front_parent = getattr(lib, "uno_kkt_debug_front_parent", None)
    # parents from the level structure: a front's parent is the unique front of the next level whose rows...
    # (not exported) -- use the timeline instead: per level, the latest child signal vs the level's arrivals
    for lev in range(1, fl.max() + 1):
        s = fl == lev
        c = fl == lev - 1
        seen = st[s, 4]; sig_prev = st[c, 5]; done_asm = st[s, 6]
        if (seen == 0).all() or (sig_prev == 0).all():
            continue
        print(f"level {lev:2d} fronts {s.sum():5d} | children assembled - arrival seen {((done_asm - seen) * 10e-3).mean():6.2f} us | "
              f"arrival seen - last signal of level {lev - 1} {((seen.max() - sig_prev[sig_prev > 0].max()) * 10e-3):7.2f} us (max - max) | "
              f"loop start - children assembled {((st[s, 1] - done_asm) * 10e-3).mean():5.2f} us")
    sys.exit(0)
if os.environ.get("MODE") == "10":  # any build: real-time phase boundaries inside the loop phase
    for lev in range(fl.max() + 1):
        s = fl == lev
        rl = (st[s, 4] - st[s, 1]) * 10e-3; pv = (st[s, 5] - st[s, 4]) * 10e-3
        cb = (st[s, 6] - st[s, 5]) * 10e-3; rest = (st[s, 2] - st[s, 6]) * 10e-3
        print(f"level {lev:2d} m {fm[s].mean():5.1f} p {fp[s].mean():5.1f} | reg_load {rl.mean():6.2f} pivot loop {pv.mean():6.2f} "
              f"({pv.mean() * 1e3 / max(fp[s].mean(), 1):5.0f} ns/step) early CB+drain {cb.mean():6.2f} bookkeeping+L {rest.mean():6.2f} us | "
              f"loop phase {loop[s].mean():6.2f} us")
    sys.exit(0)
if os.environ.get("MODE") == "3":
    w4, w5 = st[:, 4], st[:, 5]
    parts = np.stack([w4 & 0xffffffff, w4 >> 32, w5 & 0xffffffff, w5 >> 32, st[:, 6]], 1).astype(np.float64)
    for lev in range(fl.max() + 1):
        s = fl == lev
        per = parts[s] / steps[s][:, None]
        print(f"level {lev:2d} m {fm[s].mean():5.1f} p {fp[s].mean():5.1f} | per step: akk {per[:,0].mean():6.0f} test {per[:,1].mean():6.0f} "
              f"ballot {per[:,2].mean():6.0f} reads {per[:,3].mean():6.0f} fma {per[:,4].mean():6.0f} | loop {loop[s].mean():6.2f} us")
    sys.exit(0)
if os.environ.get("ENDS"):  # per level: end-time percentiles and the latest-ending fronts (start / assembled / end)
    t0 = st[:, 0].min()
    for lev in range(fl.max() + 1):
        s = np.nonzero(fl == lev)[0]
        e = (st[s, 3] - t0) * 10e-3
        q = np.percentile(e, [50, 90, 99, 100])
        o = s[np.argsort(-e)[:4]]
        print(f"level {lev:2d} end p50 {q[0]:7.1f} p90 {q[1]:7.1f} p99 {q[2]:7.1f} max {q[3]:7.1f} | latest: " + ", ".join(
            f"f{f} m{fm[f]} p{fp[f]} [{(st[f,0]-t0)*10e-3:.1f} {(st[f,1]-t0)*10e-3:.1f} {(st[f,3]-t0)*10e-3:.1f}]" for f in o))
    sys.exit(0)
if os.environ.get("TAILS"):  # per level: the slowest fronts (the level's tail) -- loop / write maxima and who
    for lev in range(fl.max() + 1):
        s = np.nonzero(fl == lev)[0]
        tot = (st[s, 3] - st[s, 0]) * 10e-3
        o = s[np.argsort(-tot)[:3]]
        print(f"level {lev:2d} mean total {tot.mean():6.2f} us, slowest: " + ", ".join(
            f"f{f} m{fm[f]} p{fp[f]} asm {asm[f]:.1f} loop {loop[f]:.1f} write {wout[f]:.1f}" for f in o))
for lev in range(fl.max() + 1):
    s = fl == lev
    print(f"level {lev:2d} fronts {s.sum():6d} m {fm[s].mean():6.1f} p {fp[s].mean():5.1f} | assemble {asm[s].mean():7.2f} us "
          f"loop {loop[s].mean():7.2f} us write {wout[s].mean():6.2f} us | cycles/step search {(cs[s]/steps[s]).mean():7.0f} "
          f"update {(cu[s]/steps[s]).mean():7.0f} rest {(cr[s]/steps[s]).mean():6.0f} | span {(st[s,3].max()-st[s,0].min())*10e-3:8.1f} us")
tot = sum((st[fl == l, 3].max() - st[fl == l, 0].min()) * 10e-3 for l in range(fl.max() + 1))
print(f"sum of level spans {tot:.1f} us")
t0 = st[:, 0].min()
print("timeline (us from the first front start): level first start .. last end")
for lev in range(fl.max() + 1):
    s = fl == lev
    print(f"  level {lev:2d} {(st[s, 0].min() - t0) * 10e-3:8.1f} .. {(st[s, 3].max() - t0) * 10e-3:8.1f}")
