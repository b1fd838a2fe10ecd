"""bench.py -- KKT factor+solve throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2], SURVEY.md 8(d) "C3"): the arrowband interior-point KKT of
dimension N = 1e6 (nv = 750k variables, m = 250k equality constraints, nnz ~ 2.0e7 COO entries in
Uno's ipopt-preset layout, uno_amd/csrc/arrowband.c).  A step is one numerical LDL^T factorization
+ one inertia query + one nrhs=1 solve, after an untimed symbolic analysis; values and right-hand
side are already resident in HBM when the timed region starts.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N), default
--mode dist: ONE arrowband KKT of the C5 family (seed 0x5EED0005) of dimension
N x 5e5 (weak scaling: 5e5 rows per GPU, so N = 8 is exactly BASELINE.json configs[4], n = 4e6,
nnz = 8e7) is factored and solved across the N GPUs -- independent elimination subtrees per rank, the
subtree roots' contribution blocks / update vectors sent to rank 0 over RCCL (xGMI) for the top of
the assembly tree, the top rows of the solution broadcast back, inertia all-reduced, the solution
gathered on rank 0.  value = (N x 1e6 / 1e6) factor+solves per second, i.e. n=1e6-equivalent
factor+solves/s of the whole job (factor flops, L bytes and solve bytes of the arrowband family all
grow linearly in n).  --mode replicas: an independent C3 system per GPU (no data-path collective).

Prints ONE JSON line on rank 0 (contract in the task statement), with `roofline` for the dominant
kernel class (HIP events on the solver's stream, second timed pass) and `cpu_baseline` from the CPU
oracle (oracle/kkt_oracle.c, a restatement of MUMPS -- MUMPS itself is not available here).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0    # MI355X HBM3E spec (MI355X_MICROARCH.md)
PEAK_FP64_TFS = 78.6     # MI355X FP64 vector/matrix spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=0,
                    help="KKT dimension per GPU (default: 1e6 = C3 on one GPU / in replicas; 5e5 per GPU in dist mode, "
                         "C5 = 4e6 at 8 GPUs)")
    ap.add_argument("--mode", choices=["dist", "replicas", "ipm"], default=None,
                    help="default: dist for N>1, the C3 system for N=1.  dist: one C5-family system of N x 5e5 rows "
                         "partitioned over the GPUs (also at N=1: the same-size N=1 point of the scaling curve); "
                         "replicas: one C3 system per GPU; ipm: an interior-point-like sequence through the "
                         "drop-in's host-value path (1 GPU)")
    ap.add_argument("--no-shipped", action="store_true",
                    help="skip the second line measured in the Uno plugin's configuration (delay_relaxed=0 + refinement)")
    ap.add_argument("--ipm-iters", type=int, default=12)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-n", type=int, default=1_000_000)
    ap.add_argument("--profile-only", action="store_true", help="skip event pass and CPU baseline")
    ap.add_argument("--leaf", type=int, default=0, help="nested-dissection leaf size (0 = library default)")
    ap.add_argument("--block", type=int, default=0, help="max supernode width (0 = library default)")
    ap.add_argument("--dataflow", type=int, default=1, help="1: one-launch dataflow solve, 0: level-scheduled solve")
    ap.add_argument("--opt", action="append", default=[], help="library option name=value (A/B experiments)")
    return ap.parse_args()


def run_ipm(args):
    """An interior-point-like sequence at C3 through the path the Uno plugin takes (integration/HIPLDLSolver.cpp):
    values on the HOST (page-locked once), every iteration a new barrier diagonal Sigma (log-uniform in
    [1e-8, 1e8], the late-IPM spread) uploaded in full, then the inertia-correction loop of
    PrimalDualRegularization.hpp:133-219 (delta_w = 1e-4, then x8 / x100) whose retries upload only the
    regularization diagonal (uno_kkt_factorize_update), then one solve with host rhs / solution.  Threshold
    relaxation instead of delayed pivots (the plugin's setting), so no re-analysis happens inside the loop.
    Reports the end-to-end wall time per iteration and per factorization, PCIe included."""
    import torch
    import uno_amd
    uno_amd.load_library()
    torch.cuda.init()
    n, nv, m, rows, cols, vals, rhs = uno_amd.arrowband(args.n or 1_000_000, uno_amd.SEEDS["C3"])
    nh = sum(min(j, 12) + 1 for j in range(nv))
    sig0 = n + nh  # Sigma positions [sig0, sig0 + nv) (uno_amd/csrc/arrowband.c layout)
    kkt = uno_amd.HipKKT(0, delay_relaxed=0, pin_host_values=1)
    kkt.analyze(n, rows, cols)
    v = np.array(vals)
    rng = np.random.default_rng(7)
    kkt.factorize(v)
    kkt.inertia()
    kkt.solve(rhs)
    torch.cuda.synchronize()
    its, facs, retries, t_it = [], 0, 0, []
    for it in range(args.ipm_iters):
        v[sig0:sig0 + nv] = 10.0 ** rng.uniform(-8, 8, nv)
        v[:n] = 0.0
        t0 = time.perf_counter()
        kkt.factorize(v)
        inertia = kkt.inertia()
        nf, dw = 1, 0.0
        while inertia != (nv, m, 0) and nf < 12:
            dw = 1e-4 if dw == 0.0 else dw * (100.0 if nf > 8 else 8.0)
            v[:nv] = dw
            v[nv:n] = -1e-8
            kkt.factorize_update(v, 0, n)
            inertia = kkt.inertia()
            nf += 1
        x = kkt.solve(rhs)
        t_it.append(time.perf_counter() - t0)
        facs += nf
        retries += nf - 1
        its.append(list(inertia))
    st = kkt.stats()
    # the same sequence device-resident: the iterate (x, zl, zu, y) lives in HBM and every
    # value of every iteration is produced on the device -- the model's gradient and constraints (torch on the
    # resident band / Jacobian terms: the model's part), the augmented KKT values by uno_kkt_assemble_augmented
    # (regularization zeros, sigma * H, Sigma from x / zl / zu, J: Subproblem::assemble_augmented_matrix), the
    # inertia-correction retries by uno_kkt_fill_values, the right-hand side by uno_kkt_assemble_rhs
    # (Subproblem.cpp:80-99), the solve on device vectors, then the primal-dual direction and the
    # fraction-to-boundary step lengths by uno_kkt_assemble_direction (PrimalDualInteriorPointProblem.cpp:173-325).
    # Nothing crosses PCIe but the inertia (3 integers) and the two step lengths.
    dev = torch.device("cuda", 0)
    kd = uno_amd.HipKKT(0, delay_relaxed=0)
    kd.analyze(n, rows, cols)
    lbv, ubv = np.full(nv, -10.0), np.full(nv, 10.0)
    assert kd.barrier_setup(lbv, ubv) == nv
    nj = len(vals) - (n + nh + nv)
    kd.augmented_setup(n, nh, nj)
    jrow = np.asarray(rows[n + nh + nv:], dtype=np.int64)            # J^T entries (var, nv + j), constraint-major
    jcol = np.asarray(cols[n + nh + nv:], dtype=np.int64) - nv
    kd.rhs_setup(nv, m, jcol, jrow)
    T = lambda a, dt=torch.float64: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)
    hess_d = T(np.asarray(vals[n:n + nh]))                           # the model's Hessian terms (H of the QP)
    jac_d = T(np.asarray(vals[n + nh + nv:]))
    hr, hc = T(np.asarray(rows[n:n + nh]), torch.int64), T(np.asarray(cols[n:n + nh]), torch.int64)
    hoff = torch.nonzero(hr != hc).flatten()            # off-diagonal Hessian terms (gathered once)
    hr_off, hc_off = hr[hoff].contiguous(), hc[hoff].contiguous()
    jr_d, jc_d = T(jrow, torch.int64), T(jcol, torch.int64)
    lb_d, ub_d = T(lbv), T(ubv)
    vd = torch.empty(len(vals), dtype=torch.float64, device=dev)
    gvec = torch.empty(nv, dtype=torch.float64, device=dev)
    grad, cons = torch.empty_like(gvec), torch.empty(m, dtype=torch.float64, device=dev)
    rhs_d = torch.empty(n, dtype=torch.float64, device=dev)
    sol_d = torch.empty_like(rhs_d)
    xs = torch.empty(nv, dtype=torch.float64, device=dev)
    zl, zu = torch.empty_like(xs), torch.empty_like(xs)
    yv = torch.empty(m, dtype=torch.float64, device=dev)
    dx, dzl, dzu = torch.empty_like(xs), torch.empty_like(xs), torch.empty_like(xs)
    dy = torch.empty_like(yv)
    # the synthetic model's Hessian (symmetric) and Jacobian as device CSR matrices, built once (the values are
    # fixed): its gradient and constraints are two sparse matrix-vector products per iteration
    try:
        hrow = torch.cat([hr, hc_off])
        hcol = torch.cat([hc, hr_off])
        hval = torch.cat([hess_d, hess_d[hoff]])
        H_csr = torch.sparse_coo_tensor(torch.stack([hrow, hcol]), hval, (nv, nv)).coalesce().to_sparse_csr()
        J_csr = torch.sparse_coo_tensor(torch.stack([jc_d, jr_d]), jac_d, (m, nv)).coalesce().to_sparse_csr()
        _ = H_csr @ gvec
    except Exception:  # no sparse kernels: the scatter form
        H_csr = J_csr = None
    gen = torch.Generator(device=dev)
    gen.manual_seed(11)
    gvec.uniform_(-1.0, 1.0, generator=gen)
    torch.cuda.synchronize()
    t_dev, facs_d, steps_d = [], 0, []
    t_asm, t_model = [], []
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    stream = torch.cuda.ExternalStream(kd.stream())
    for it in range(args.ipm_iters + 1):
        # a new interior point: x inside the box, bound multipliers of the late-IPM spread
        xs.uniform_(-9.0, 9.0, generator=gen)
        zl.copy_(10.0 ** (torch.rand(nv, dtype=torch.float64, device=dev, generator=gen) * 16 - 8))
        zu.copy_(-(10.0 ** (torch.rand(nv, dtype=torch.float64, device=dev, generator=gen) * 16 - 8)))
        yv.uniform_(-1.0, 1.0, generator=gen)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        # model evaluation on the device (ArrowbandModel: gradient H x + g, constraints A x - b with b = 0 here)
        if H_csr is not None:
            torch.add(gvec, H_csr @ xs, out=grad)
            cons.copy_(J_csr @ xs)
        else:
            grad.copy_(gvec)
            grad.index_add_(0, hr, hess_d * xs[hc])
            grad.index_add_(0, hc_off, hess_d[hoff] * xs[hr_off])
            cons.zero_()
            cons.index_add_(0, jc_d, jac_d * xs[jr_d])
        torch.cuda.current_stream().synchronize()
        t_model.append(time.perf_counter() - t0)
        with torch.cuda.stream(stream):
            ev[0].record(stream)
        kd.assemble_augmented(1.0, hess_d.data_ptr(), jac_d.data_ptr(), xs.data_ptr(), zl.data_ptr(), zu.data_ptr(),
                              vd.data_ptr())
        with torch.cuda.stream(stream):
            ev[1].record(stream)
        kd.factorize(device_ptr=vd.data_ptr())
        inertia = kd.inertia()
        nf, dw = 1, 0.0
        while inertia != (nv, m, 0) and nf < 12:
            dw = 1e-4 if dw == 0.0 else dw * (100.0 if nf > 8 else 8.0)
            kd.fill_values(0, nv, dw)
            kd.fill_values(nv, m, -1e-8)
            kd.factorize()
            inertia = kd.inertia()
            nf += 1
        kd.assemble_rhs(grad.data_ptr(), cons.data_ptr(), yv.data_ptr(), jac_d.data_ptr(), rhs_d.data_ptr())
        kd.solve_device(rhs_d.data_ptr(), sol_d.data_ptr())
        ap, ad = kd.assemble_direction(nv, m, sol_d.data_ptr(), xs.data_ptr(), lb_d.data_ptr(), ub_d.data_ptr(),
                                       zl.data_ptr(), zu.data_ptr(), 1e-6, 0.99, dx.data_ptr(), dy.data_ptr(),
                                       dzl.data_ptr(), dzu.data_ptr())
        torch.cuda.synchronize()
        if it:  # the first pass warms up
            t_dev.append(time.perf_counter() - t0)
            t_asm.append(ev[0].elapsed_time(ev[1]))
            facs_d += nf
            steps_d.append([ap, ad])
    # the device-assembled values of the last iteration against the host restatement of the same assembly
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    asm_check = None
    if os.path.exists(os.path.join(ROOT, "oracle", "ipm_oracle.py")):
        import ipm_oracle
        # the last iteration's values after its retries: the regularization prefix holds delta_w / -delta_c
        # (uno_kkt_fill_values), every other position the assembly's value
        ref = ipm_oracle.assemble_augmented(n, 1.0, np.asarray(vals[n:n + nh]), np.asarray(vals[n + nh + nv:]),
                                            xs.cpu().numpy(), lbv, ubv, zl.cpu().numpy(), zu.cpu().numpy())
        got = vd.cpu().numpy()
        asm_check = bool(np.array_equal(got[n:].view(np.uint64), ref[n:].view(np.uint64)))
    res = np.abs(uno_amd.coo_symv(n, rows, cols, v, x) - rhs).max()
    absk = uno_amd.coo_symv(n, rows, cols, np.abs(v), np.ones(n)).max()
    total = sum(t_it)
    print(json.dumps({
        "metric": "KKT factorizations/s, IPM-like sequence through the drop-in host-value path (C3, PCIe included)",
        "value": round(facs / total, 3), "unit": "factorizations/s", "n_gpus": 1, "higher_is_better": True,
        "iterations": args.ipm_iters, "factorizations": facs, "inertia_correction_retries": retries,
        "ms_per_iteration_median": round(1e3 * float(np.median(t_it)), 3), "ms_per_factorization": round(1e3 * total / facs, 3),
        "fronts_merged": st["fronts_merged"], "pivots_relaxed_last": st["pivots_relaxed"],
        "device_resident": {"factorizations_per_s": round(facs_d / sum(t_dev), 3), "factorizations": facs_d,
                            # the same without the model evaluation (torch index_add_ on the synthetic model: the
                            # caller's code, outside the solver)
                            "solver_factorizations_per_s": round(facs_d / (sum(t_dev) - sum(t_model[1:])), 3),
                            "ms_per_iteration_median": round(1e3 * float(np.median(t_dev)), 3),
                            "ms_per_factorization": round(1e3 * sum(t_dev) / facs_d, 3),
                            "model_eval_ms_median": round(1e3 * float(np.median(t_model)), 3),
                            "assemble_augmented_ms_median": round(float(np.median(t_asm)), 4),
                            "assemble_augmented_GBs": round((8.0 * (len(vals) + nh + nj) + 45.0 * nv) / (float(np.median(t_asm)) * 1e-3) / 1e9, 1),
                            "assembly_bit_identical_to_oracle": asm_check,
                            "step_lengths_last": steps_d[-1] if steps_d else None,
                            "note": "per iteration on the device: model gradient / constraints (torch), augmented KKT "
                                    "values (uno_kkt_assemble_augmented: zeros, sigma*H, Sigma, J), delta_w retries "
                                    "(uno_kkt_fill_values), rhs (uno_kkt_assemble_rhs), solve, direction + "
                                    "fraction-to-boundary (uno_kkt_assemble_direction): no value crosses PCIe"},
        "rel_residual_last": float(res / (absk * np.abs(x).max() + np.abs(rhs).max())),
        "config": {"workload": "C3 arrowband KKT, Sigma redrawn per iteration, delta_w retries, host values + rhs",
                   "n": n, "nnz": len(vals), "full_upload_bytes": 8 * len(vals), "retry_upload_bytes": 8 * n},
    }))


def main():
    args = parse()
    if args.mode == "ipm":
        return run_ipm(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
    dev = torch.device("cuda", local)

    import uno_amd
    uno_amd.load_library()
    def build(dist_mode):
        if dist_mode:  # one C5-family system of dimension world * n, the same on every rank
            seed, n_total = uno_amd.SEEDS["C5"], (args.n or 500_000) * world
        else:          # independent system per rank
            seed, n_total = uno_amd.SEEDS["C3"] + rank, args.n or 1_000_000
        n, nv, m, rows, cols, vals, rhs = uno_amd.arrowband(n_total, seed)
        kkt = uno_amd.HipKKT(local)
        if dist_mode and world > 1:
            from uno_amd.replicas import share_bytes
            uid = share_bytes(uno_amd.rccl_unique_id() if rank == 0 else None, world)
            kkt.attach_rccl(uid, rank, world)
        if args.leaf:
            kkt.set_option("leaf_size", args.leaf)
        if args.block:
            kkt.set_option("max_block", args.block)
        kkt.set_option("dataflow_solve", args.dataflow)
        for kv in args.opt:
            k_, v_ = kv.split("=", 1)
            kkt.set_option(k_, float(v_))
        t0 = time.perf_counter()
        kkt.analyze(n, rows, cols)
        t_analysis = time.perf_counter() - t0
        vals_d = torch.from_numpy(vals).to(dev)
        rhs_d = torch.from_numpy(rhs).to(dev)
        x_d = torch.empty_like(rhs_d)
        torch.cuda.synchronize()
        return n_total, (n, nv, m, rows, cols, vals, rhs), kkt, t_analysis, vals_d, rhs_d, x_d

    mode = args.mode or ("dist" if world > 1 else "single")
    dist_mode = mode == "dist"
    dist_fallback = None
    if dist_mode:
        # the partitioned path is checked once before timing; a rank that fails (RCCL or device error)
        # makes every rank fall back to independent replicas, reported in the JSON line
        ok, err = 1, ""
        try:
            n_total, gen, kkt, t_analysis, vals_d, rhs_d, x_d = build(True)
            kkt.factorize(device_ptr=vals_d.data_ptr())
            kkt.inertia()
            kkt.solve_device(rhs_d.data_ptr(), x_d.data_ptr())
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001 -- reported, then the replicas mode runs
            ok, err = 0, repr(e)[:300]
        flag = torch.tensor([ok], dtype=torch.int32, device=dev)
        if world > 1:
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if int(flag.item()) == 0:
            dist_fallback = err or "another rank failed"
            dist_mode = False
    if not dist_mode:
        n_total, gen, kkt, t_analysis, vals_d, rhs_d, x_d = build(False)
    n, nv, m, rows, cols, vals, rhs = gen

    def first_factorization():
        """The first factorization of a pattern, timed alone: with MUMPS-style delays it includes the merge
        rounds (a delayed column moves into the parent front: host structure rebuild + refactorization)."""
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        kkt_ = kkt
        kkt_.factorize(device_ptr=vals_d.data_ptr())
        kkt_.inertia()
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t1)

    first_ms = first_factorization()
    first_merges = kkt.stats()["fronts_merged"]

    def step():
        kkt.factorize(device_ptr=vals_d.data_ptr())
        inertia = kkt.inertia()
        kkt.solve_device(rhs_d.data_ptr(), x_d.data_ptr())
        return inertia

    from uno_amd.replicas import aggregate, timed_steps
    elapsed, inertia = timed_steps(step, args.steps, args.warmup, torch.cuda.synchronize, world, dev)
    # also the median of >= 20 individually synchronised steps (reported beside the
    # contract's K-step wall time)
    per_step = []
    for _ in range(max(20, args.steps) if not args.profile_only else 0):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        per_step.append(time.perf_counter() - t1)
    if world > 1 and per_step:
        tt = torch.tensor(per_step, dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        per_step = tt.cpu().tolist()
    median_ms = round(1e3 * float(np.median(per_step)), 4) if per_step else None

    # parity sanity on the measured system: relative residual of the last solve (rank 0 holds the
    # complete solution in dist mode)
    rel_res = None
    if rank == 0 or not dist_mode:
        x = x_d.cpu().numpy()
        res = np.abs(uno_amd.coo_symv(n, rows, cols, vals, x) - rhs).max()
        absk = uno_amd.coo_symv(n, rows, cols, np.abs(vals), np.ones(n)).max()
        rel_res = float(res / (absk * np.abs(x).max() + np.abs(rhs).max()))
    st = kkt.stats()
    dinfo = kkt.dist_info() if dist_mode and world > 1 else None
    assert st["solve_aborts"] == 0, f"dataflow solve aborted {st['solve_aborts']} times (level-scheduled redo)"

    # second timed pass with per-kernel HIP events on the solver stream (roofline)
    ktimes = {}
    if not args.profile_only:
        kkt.set_option("timing", 1)
        kkt.reset_kernel_times()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        ktimes = kkt.kernel_times()
        kkt.set_option("timing", 0)

    # ---- the same step in the Uno plugin's configuration (integration/HIPLDLSolver.cpp:15-27): threshold
    # relaxation instead of delayed pivots (delay_relaxed=0) and one refinement step per solve after a
    # factorization that relaxed a pivot.  Single-GPU lines only (the plugin drives one GPU).
    shipped = None
    if world == 1 and not args.no_shipped and not args.profile_only:
        ks = uno_amd.HipKKT(local, delay_relaxed=0)
        ks.set_option("dataflow_solve", args.dataflow)
        for kv in args.opt:  # A/B options apply to this handle too (its delay_relaxed stays the plugin's)
            k_, v_ = kv.split("=", 1)
            if k_ != "delay_relaxed":
                ks.set_option(k_, float(v_))
        ks.analyze(n, rows, cols)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ks.factorize(device_ptr=vals_d.data_ptr())
        s_inertia = ks.inertia()
        torch.cuda.synchronize()
        s_first = 1e3 * (time.perf_counter() - t1)
        xs_d = torch.empty_like(rhs_d)

        def sstep():
            ks.factorize(device_ptr=vals_d.data_ptr())
            i_ = ks.inertia()
            ks.solve_device(rhs_d.data_ptr(), xs_d.data_ptr())
            return i_
        s_elapsed, s_inertia = timed_steps(sstep, args.steps, args.warmup, torch.cuda.synchronize, 1, dev)
        sst = ks.stats()
        xsv = xs_d.cpu().numpy()
        # normwise backward error eta = |b - A x|_inf / (|A|_inf |x|_inf + |b|_inf) with and without the refinement step
        anorm_inf = float(uno_amd.coo_symv(n, rows, cols, np.abs(vals), np.ones(n)).max())
        def eta(xv):
            """normwise and componentwise backward errors of xv"""
            r = np.abs(uno_amd.coo_symv(n, rows, cols, vals, xv) - rhs)
            den = uno_amd.coo_symv(n, rows, cols, np.abs(vals), np.abs(xv)) + np.abs(rhs)
            comp = float(np.max(np.where(den > 0, r / np.where(den > 0, den, 1.0), 0.0)))
            return [float(r.max() / (anorm_inf * np.abs(xv).max() + np.abs(rhs).max())), comp]
        eta_refined = eta(xsv)
        ks.set_option("refine", 0)
        ks.solve_device(rhs_d.data_ptr(), xs_d.data_ptr())
        torch.cuda.synchronize()
        eta_unrefined = eta(xs_d.cpu().numpy())
        ks.set_option("refine", 1)
        sres = np.abs(uno_amd.coo_symv(n, rows, cols, vals, xsv) - rhs).max()
        sabs = uno_amd.coo_symv(n, rows, cols, np.abs(vals), np.ones(n)).max()
        shipped = {"value": round(args.steps / s_elapsed, 4), "unit": "factor+solve/s",
                   "ms_per_step": round(1e3 * s_elapsed / args.steps, 4),
                   "first_factorization_ms": round(s_first, 3),
                   "options": "delay_relaxed=0, refine=1 (HIPLDLSolver.cpp)",
                   "pivots_relaxed": sst["pivots_relaxed"], "fronts_merged": sst["fronts_merged"],
                   "refinement_steps_per_solve": 1 if sst["pivots_relaxed"] > 0 else 0,
                   "inertia": list(s_inertia), "inertia_equal_to_headline": tuple(s_inertia) == tuple(inertia),
                   "backward_error_unrefined": eta_unrefined, "backward_error_refined": eta_refined,
                   "rel_residual": float(sres / (sabs * np.abs(xsv).max() + np.abs(rhs).max()))}
        del ks

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    # whole-job throughput in n=1e6-equivalent factor+solves (dist: one system of world * n rows)
    value, ms_per_step = aggregate(args.steps, world, elapsed)
    if dist_mode:
        value = args.steps * (n_total / 1_000_000) / elapsed

    # ---- roofline of the dominant kernel class (rank 0's kernels) ----
    K = args.steps
    n2 = st["pivots_2x2"]
    bytes_solve = 8.0 * (2 * st["nnz_L"] + n + n2) + 24.0 * n      # SURVEY 8(d) B_solve, per solve
    flops_fac = st["flops"]                                         # per factorization
    if dinfo:  # rank 0's share: its subtrees + the top of the tree
        flops_fac = dinfo["my_flops"] + dinfo["top_flops"]
    bytes_fac = 8.0 * (st["nnz_unique"] + st["nnz_L"] + n)          # B_min per factorization
    roof = None
    if ktimes:
        fac_ms = (ktimes["factor_lds"][0] + ktimes["factor_global"][0]) / K
        sol_ms = (ktimes["solve_fwd"][0] + ktimes["solve_bwd"][0]) / K
        others = {k: v[0] / K for k, v in ktimes.items()}
        if fac_ms >= sol_ms:
            # bound = max(F / P_FP64, B_min / BW).  At C3 F / B_min ~ 4.8 flop/B, below the
            # FP64 ridge (78.6 TF / 8 TB/s ~ 9.8 flop/B), so the roofline of the factorization is HBM
            ach_f = flops_fac / (fac_ms * 1e-3) / 1e12
            t_flop, t_hbm = flops_fac / (PEAK_FP64_TFS * 1e12), bytes_fac / (PEAK_HBM_GBS * 1e9)
            bound = "hbm" if t_hbm >= t_flop else "mfma"
            ach_b = bytes_fac / (fac_ms * 1e-3) / 1e9
            roof = {"kernel": "factor (k_factor_lds level launches of the lower tree + one k_factor_df dataflow launch "
                              "of the upper tree, one factorization)",
                    "bound": bound,
                    "achieved": round(ach_b, 2) if bound == "hbm" else round(ach_f, 4),
                    "peak": PEAK_HBM_GBS if bound == "hbm" else PEAK_FP64_TFS,
                    "unit": "GB/s" if bound == "hbm" else "TFLOP/s",
                    "frac": round(ach_b / PEAK_HBM_GBS if bound == "hbm" else ach_f / PEAK_FP64_TFS, 5),
                    "traffic": None,
                    "algorithmic": f"B_min {bytes_fac:.4e} B and F {flops_fac:.4e} FP64 flop per factorization "
                                   f"(intensity {flops_fac / bytes_fac:.2f} flop/B)",
                    "ms_per_launch_group": round(fac_ms, 4),
                    "fp64_TFs": round(ach_f, 4), "fp64_frac": round(ach_f / PEAK_FP64_TFS, 5)}
        else:
            ach = bytes_solve / (sol_ms * 1e-3) / 1e9
            roof = {"kernel": "solve (k_solve_fwd_df + k_solve_bwd_df dataflow launches of one solve)",
                    "bound": "hbm", "achieved": round(ach, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(ach / PEAK_HBM_GBS, 5), "traffic": None,
                    "algorithmic": f"{bytes_solve:.4e} B per solve", "ms_per_launch_group": round(sol_ms, 4)}
        roof["kernel_ms_per_step"] = {k: round(v, 4) for k, v in others.items()}
        roof["solve_GBs"] = round(bytes_solve / (sol_ms * 1e-3) / 1e9, 2) if sol_ms > 0 else None
        # PMC-measured HBM bytes (profiles/pmc_traffic.json, rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this
        # bench): used only when the profile was taken on this workload (same n, nnz, default analysis options)
        pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        pmcd = {}
        if os.path.exists(pmc):
            try:
                cand = json.load(open(pmc))
                wl = cand.get("workload", {})
                if (wl.get("n") == n and wl.get("nnz") == len(vals) and not args.leaf and not args.block
                        and not args.opt and world == 1):
                    pmcd = cand
            except Exception:
                pmcd = {}
        roof["traffic"] = pmcd.get("factor_bytes_per_factorization")
        roof["traffic_source"] = (pmcd.get("source") if pmcd else
                                  "null: profiles/pmc_traffic.json was not measured on this workload / options")
        # the triangular solve against the HBM roofline (north_star target: >= 60 %)
        if sol_ms > 0:
            sach = bytes_solve / (sol_ms * 1e-3) / 1e9
            roof["solve_roofline"] = {"bound": "hbm", "achieved": round(sach, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                      "frac": round(sach / PEAK_HBM_GBS, 5),
                                      "traffic": pmcd.get("solve_bytes_per_solve"),
                                      "algorithmic": f"{bytes_solve:.4e} B per solve (fwd + bwd)",
                                      "ms_per_solve": round(sol_ms, 4)}

    # ---- CPU baseline (BASELINE.md 4 "Fallback": MUMPS unavailable offline) ----
    # oracle/cpu_mf.cpp: multifrontal LDL^T on the product's nested-dissection analysis, OpenMP over the
    # fronts of each tree level, timed on the host cores this job may use (OMP_NUM_THREADS, 16 on the GPU
    # box); the one-thread oracle (oracle/kkt_oracle.c) factors the same matrix once more as the checker
    cpu = None
    if not args.no_cpu_baseline and not args.profile_only and world == 1:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from cpu_baseline_ffi import CpuMF, threads
        from oracle_ffi import OracleKKT
        cn, _, _, cr, cc, cv, cb = uno_amd.arrowband(args.cpu_baseline_n, uno_amd.SEEDS["C3"])
        c = CpuMF()
        c.analyze(cn, cr, cc)
        c.factorize(cv)  # warm-up (first touch of the arenas)
        c.solve(cb)
        reps, t_cpu, per = 0, 0.0, []
        while reps < 60 and t_cpu < 12.0:
            t1 = time.perf_counter()
            c.factorize(cv)
            c_inertia = c.inertia()
            c.solve(cb)
            per.append(time.perf_counter() - t1)
            t_cpu += per[-1]
            reps += 1
        o = OracleKKT()
        o.analyze(cn, cr, cc)
        o.factorize(cv)
        o_inertia = o.inertia()
        # parity on the measured system: GPU, CPU baseline and oracle give the same inertia
        assert tuple(c_inertia) == tuple(o_inertia), f"CPU baseline inertia {c_inertia} != oracle {o_inertia}"
        if cn == n:
            assert tuple(o_inertia) == tuple(inertia), f"GPU inertia {inertia} != oracle {o_inertia}"
        model = ""
        try:
            model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
        except Exception:  # noqa: BLE001 -- informational
            pass
        try:
            affinity = len(os.sched_getaffinity(0))
        except Exception:  # noqa: BLE001 -- informational
            affinity = None
        cpu = {"value": round(1.0 / float(np.median(per)), 4), "unit": "factor+solve/s", "cores": threads(),
               "reps_min_max_per_s": [round(1.0 / max(per), 4), round(1.0 / min(per), 4)],
               "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
               "kind": "port",
               "sample": f"oracle/cpu_mf.cpp (multi-threaded multifrontal restatement on the product's ND analysis; "
                         f"MUMPS unavailable) on arrowband n={cn} nnz={len(cv)}: median of {reps} "
                         f"factor+inertia+solve reps ({t_cpu:.1f} s), {threads()} OpenMP threads",
               "nproc": os.cpu_count(), "affinity_cpus": affinity,
               "cores_note": "OpenMP threads = OMP_NUM_THREADS, the host-core share the GPU pool leases per GPU: the "
                             "harness exports OMP_NUM_THREADS=16 on every 1-GPU box and caps worker pools at 16; nproc / "
                             "sched_getaffinity show the whole shared host (other leases run on the same cores), so "
                             "running at affinity_cpus threads would time contention, not MUMPS-class host throughput",
               "cpu_model": model,
               "inertia": list(o_inertia), "inertia_checked_against_gpu": cn == n,
               "gpu_over_cpu": round(value / (1.0 / float(np.median(per))), 1) if per else None}

    out = {
        "metric": "KKT factor+solve/sec & HBM GB/s, n=1e6 nnz=2e7 ipopt preset, 1/2/4/8 GPU",
        "value": round(value, 4),
        "unit": "factor+solve/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "ms_per_step_median": median_ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic (arrowband KKT generator, SURVEY 8(d), C5 family seed 0x5EED0005, one system over all ranks)"
                 if dist_mode else "synthetic (arrowband KKT generator, SURVEY 8(d), seed 0x5EED0003+rank)"),
        "config": {"workload": ("C5-family arrowband KKT (n = %d over %d GPUs), ipopt-preset COO layout, factor+inertia+solve"
                                % (n_total, world)) if dist_mode else "C3 arrowband KKT, ipopt-preset COO layout, factor+inertia+solve",
                   "n": n, "nv": nv, "m": m, "nnz": int(len(vals)), "nnz_unique": st["nnz_unique"],
                   "nnz_L": st["nnz_L"], "fronts": st["n_fronts"], "levels": st["n_levels"],
                   "max_front": st["max_front"], "ordering": "nested dissection (BFS level sets), 6 dense nodes last",
                   "analysis_s": round(t_analysis, 3), "inertia": list(inertia),
                   "pivots_2x2": st["pivots_2x2"], "pivots_relaxed": st["pivots_relaxed"],
                   "solve_schedule": f"dataflow grid {st['solve_grid']}" if st["solve_grid"] else "level-synchronous",
                   "fronts_merged": st["fronts_merged"], "rel_residual": rel_res,
                   "first_factorization_ms": round(first_ms, 3),
                   "first_factorization_note": "timed alone after the warm-up-free analysis: MUMPS-style delays "
                                               "(delay_relaxed=1) are resolved here by merge rounds "
                                               f"({first_merges} fronts merged); the timed steps refactor the merged structure",
                   "solve_aborts": st["solve_aborts"],
                   "parallelism": (f"subtree-partitioned x{world} (RCCL root exchange to rank 0)" if dist_mode
                                   else f"replicas x{world} (independent KKT per GPU)"),
                   "value_unit_note": "n=1e6-equivalent factor+solves per second of the whole job",
                   "dist": dinfo, "dist_fallback": dist_fallback},
        "roofline": roof,
        "cpu_baseline": cpu,
        "shipped_plugin_mode": shipped,
    }
    print(json.dumps(out))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
