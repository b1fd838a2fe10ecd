"""Multi-GPU path: one factorization partitioned into independent elimination
subtrees per rank, subtree roots' contribution blocks sent to rank 0 for the top of the tree.

CPU tests check the partition (host-only analysis, no device).  GPU tests run the whole distributed
algorithm on ONE GPU with the in-process transport (one host thread per rank, device-to-device
copies instead of RCCL, same orchestration code) and compare it with the single-GPU path and the
oracle: inertia exact, solution within the north_star 1e-10 relative residual (the factorization
arithmetic per front is the same, so the two solutions agree to rounding)."""
import threading

import numpy as np
import pytest

from oracle_ffi import OracleKKT

RES_TOL = 1e-10


@pytest.fixture(scope="module")
def ua():
    import uno_amd
    uno_amd.load_library()
    return uno_amd


def _check_partition(owner, parent, world):
    nf = len(owner)
    assert ((owner >= -1) & (owner < world)).all()
    for f in range(nf):
        p = parent[f]
        if p < 0:
            continue
        assert p > f  # children numbered before parents
        if owner[f] == -1:
            assert owner[p] == -1, "top set must be closed towards the root"
        elif owner[p] != -1:
            assert owner[p] == owner[f], "a subtree belongs to one rank"


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_partition_arrowband(ua, world):
    n, _, _, r, c, _, _ = ua.arrowband(60000, ua.SEEDS["C3"])
    owner, parent, nsub = ua.debug_partition(n, r, c, world)
    _check_partition(owner, parent, world)
    assert nsub >= world
    counts = np.array([(owner == q).sum() for q in range(world)])
    assert (counts > 0).all()
    assert counts.max() <= 1.25 * counts.mean()  # balanced subtrees (fronts as a proxy)
    assert (owner == -1).sum() < 0.01 * len(owner)


def test_partition_random(ua):
    from test_gpu_parity import random_sym
    rng = np.random.default_rng(7)
    for world in (2, 5):
        for n, dens in ((40, 0.3), (400, 0.01)):
            rr, cc, _, _ = random_sym(rng, n, dens, 0.3)
            owner, parent, _ = ua.debug_partition(n, rr, cc, world)
            _check_partition(owner, parent, world)


def run_group(ua, world, n, r, c, batches, rhs, **opt):
    """Every rank (thread) analyses, then for each value batch factorizes + inertia + solve."""
    group = ua.LocalGroup(world)
    out = [None] * world
    errs = []

    def rank_main(q):
        try:
            g = ua.HipKKT(0, **opt)
            g.attach_local(group, q)
            g.analyze(n, r, c)
            res = []
            for v in batches:
                g.factorize(v)
                ine = g.inertia()
                res.append((ine, g.solve(rhs)))
            out[q] = (res, g.dist_info(), g.stats())
            g.close()
        except Exception as e:  # surfaced below
            errs.append((q, repr(e)))

    th = [threading.Thread(target=rank_main, args=(q,)) for q in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    group.close()
    assert not errs, errs
    return out


def rel_residual(ua, n, r, c, v, x, b):
    res = ua.coo_symv(n, r, c, v, x) - b
    absv = ua.coo_symv(n, r, c, np.abs(v), np.ones(n))
    return np.abs(res).max() / (absv.max() * np.abs(x).max() + np.abs(b).max())


@pytest.mark.gpu
@pytest.mark.parametrize("world,dfs", [(2, 1), (3, 1), (4, 1), (2, 0), (3, 0)])
def test_distributed_arrowband(ua, world, dfs):
    """dfs = 1: each rank solves its own subtrees with the dataflow solve (one launch per direction), the
    top of the tree level-scheduled on rank 0; dfs = 0: level-scheduled subtree solves."""
    n, nv, m, r, c, v, b = ua.arrowband(40000, ua.SEEDS["C2"])
    v2 = v.copy()
    v2[:nv] = 1e-2       # inertia-correction retry: primal regularization on the diagonal
    v2[nv:n] = -1e-9
    single = ua.HipKKT(0)
    single.analyze(n, r, c)
    ref = []
    for vv in (v, v2):
        single.factorize(vv)
        ref.append((single.inertia(), single.solve(b)))
    out = run_group(ua, world, n, r, c, (v, v2), b, dist_dataflow_solve=dfs)
    info0 = out[0][1]
    assert info0["world"] == world and info0["subtrees"] >= world
    assert all((o[2]["solve_grid"] > 0) == bool(dfs) for o in out)
    assert all(o[2]["solve_aborts"] == 0 for o in out)
    assert sum(o[1]["my_fronts"] for o in out) + info0["top_fronts"] == single.stats()["n_fronts"]
    # the ranks' own subtrees use the dataflow factorization of their upper levels too
    assert sum(o[2]["factor_df_fronts"] for o in out) > 0 and all(o[2]["factor_df_aborts"] == 0 for o in out)
    for k, vv in enumerate((v, v2)):
        for q in range(world):
            assert out[q][0][k][0] == ref[k][0], (q, k)      # inertia all-reduced to every rank
        x0 = out[0][0][k][1]                                 # rank 0: gathered solution
        assert rel_residual(ua, n, r, c, vv, x0, b) < RES_TOL
        np.testing.assert_allclose(x0, ref[k][1], rtol=1e-12, atol=1e-14 * np.abs(ref[k][1]).max())


@pytest.mark.gpu
def test_distributed_delayed_pivots(ua):
    """Indefinite matrices with zero diagonals: fronts delay pivots; every rank must apply the union of
    all ranks' delayed columns and still agree with the oracle's inertia."""
    from test_gpu_parity import random_sym
    rng = np.random.default_rng(11)
    checked = merged = 0
    for trial in range(10):
        nn = int(rng.integers(150, 300))
        rr, cc, vv, S = random_sym(rng, nn, 0.03, zero_diag_frac=0.5)
        ev = np.linalg.eigvalsh(S)
        if np.min(abs(ev)) < 1e-8 * max(1.0, abs(ev).max()):
            continue
        o = OracleKKT()
        o.analyze(nn, rr, cc)
        o.factorize(vv)
        b = rng.standard_normal(nn)
        out = run_group(ua, 2, nn, rr, cc, (vv,), b, dist_force=1)  # small: split although the gate would decline
        expect = (int((ev > 0).sum()), int((ev < 0).sum()), 0)
        assert out[0][0][0][0] == out[1][0][0][0] == o.inertia() == expect
        x = out[0][0][0][1]
        np.testing.assert_allclose(S @ x, b, atol=1e-8 * np.linalg.cond(S) * np.abs(b).max())
        merged += out[0][2]["fronts_merged"]
        checked += 1
    assert checked >= 5
    assert merged > 0  # the delayed-pivot rounds were exercised


@pytest.mark.gpu
@pytest.mark.slow
def test_c5_eight_ranks(ua):
    """BASELINE.json configs[4] exactly: the C5 arrowband KKT (n = 4e6, nnz = 8e7, seed 0x5EED0005) split
    into subtrees over 8 ranks (here 8 in-process ranks on one GPU: the same orchestration as RCCL, with
    device-to-device copies) must give the single-GPU inertia on every rank and, on rank 0, a solution
    bit-identical to the single-GPU one (per-front arithmetic is shared; scaling maxima are exact)."""
    n, nv, m, r, c, v, b = ua.arrowband(4_000_000, ua.SEEDS["C5"])
    assert len(v) > 7.9e7
    single = ua.HipKKT(0)
    single.analyze(n, r, c)
    single.factorize(v)
    ine = single.inertia()
    xs = single.solve(b)
    assert rel_residual(ua, n, r, c, v, xs, b) < RES_TOL
    single.close()
    out = run_group(ua, 8, n, r, c, (v,), b)
    assert out[0][1]["world"] == 8 and out[0][1]["subtrees"] >= 8
    for q in range(8):
        assert out[q][0][0][0] == ine, q
    np.testing.assert_array_equal(out[0][0][0][1], xs)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_multiprocess_host_transport(world):
    """The partitioned factorization across real processes (one rank each, all on one GPU): the library's
    exchange goes through uno_kkt_attach_host with torch.distributed over gloo carrying the staged host
    buffers (RCCL refuses several ranks on one device).  Every rank reports the inertia of the whole
    matrix, equal to the single-GPU path's; rank 0's gathered solution agrees with the single-GPU one
    and meets the residual bar -- before and after an inertia-correction change of the diagonal."""
    import json
    import os
    import socket
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = [subprocess.Popen([sys.executable, os.path.join(here, "dist_host_worker.py"), str(q), str(world), str(port),
                               "60000"], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for q in range(world)]
    outs = []
    for p in procs:
        try:
            so, se = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for pp in procs:
                pp.kill()
            raise
        assert p.returncode == 0, se[-3000:]
        outs.append(json.loads([l for l in so.splitlines() if l.startswith("{")][-1]))
    r0 = outs[0]
    assert r0["dist"]["world"] == world and r0["dist"]["subtrees"] >= world
    for run_i, run in enumerate(r0["runs"]):
        assert run["inertia"] == run["ref_inertia"]
        assert all(o["runs"][run_i]["inertia"] == run["inertia"] for o in outs)
        assert run["rel_residual"] < RES_TOL
        assert run["max_rel_diff"] < 1e-9
    assert r0["stats"]["factorizations"] == 2 and r0["stats"]["solves"] == 2


def check_comm_traces(traces):
    """The transport calls of every rank (option comm_trace) form a consistent RCCL program: the k-th send from
    rank a to rank b has the size of the k-th receive on b from a, every send / receive sits inside a
    group_begin / group_end bracket (ncclGroupStart / End), and the collectives (all-reduce count and
    operation, broadcast size and root) are issued in the same order with the same arguments on every rank."""
    world = len(traces)
    coll = []
    # stream ordering: every send / recv / collective is enqueued on the handle's main stream
    # with no side-stream factor launch left un-joined into it, i.e. after every launch that produced its buffer
    for q, tr in enumerate(traces):
        for i, t in enumerate(tr):
            if t[0] in ("send", "recv", "allreduce", "broadcast"):
                assert i > 0 and tr[i - 1][0] == "order", f"rank {q}: {t[0]} #{i} without an order record"
                assert tr[i - 1][1] == 1, f"rank {q}: {t[0]} #{i} not on the main stream"
                assert tr[i - 1][2] == 0, f"rank {q}: {t[0]} #{i} enqueued before side-stream launches were joined"
    traces = [[t for t in tr if t[0] != "order"] for tr in traces]
    for q, tr in enumerate(traces):
        depth = 0
        for op, peer, nbytes, red in tr:
            if op == "group_begin":
                depth += 1
            elif op == "group_end":
                assert depth > 0, f"rank {q}: group_end without group_begin"
                depth -= 1
            elif op in ("send", "recv"):
                assert depth > 0, f"rank {q}: {op} outside a group"
                assert 0 <= peer < world and peer != q
        assert depth == 0
        coll.append([t for t in tr if t[0] in ("allreduce", "broadcast")])
    for q in range(1, world):
        assert coll[q] == coll[0], f"rank {q} collectives differ from rank 0's"
    for a in range(world):
        for b in range(world):
            if a == b:
                continue
            sends = [t[2] for t in traces[a] if t[0] == "send" and t[1] == b]
            recvs = [t[2] for t in traces[b] if t[0] == "recv" and t[1] == a]
            assert sends == recvs, f"sends {a}->{b} {sends[:8]} vs receives {recvs[:8]}"
    return sum(len(c) for c in coll[:1]), sum(1 for tr in traces for t in tr if t[0] == "send")


@pytest.mark.gpu
def test_multiprocess_rccl_call_sequence():
    """VERDICT r4 (multi-GPU): the exact call sequence of the RCCL path -- the options the RCCL transport runs
    with (one-launch dataflow subtree solves on) and the library's group send / recv and collective calls --
    driven across two real processes through the host transport over gloo, every call recorded (option
    comm_trace).  The traces are a consistent RCCL program (matched sizes and order, sends inside groups,
    identical collectives on both ranks) and the results equal the single-GPU path's."""
    import json
    import os
    import socket
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    world = 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = [subprocess.Popen([sys.executable, os.path.join(here, "dist_host_worker.py"), str(q), str(world), str(port),
                               "60000", "rccl_sequence"], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for q in range(world)]
    outs = []
    for p in procs:
        try:
            so, se = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for pp in procs:
                pp.kill()
            raise
        assert p.returncode == 0, se[-3000:]
        outs.append(json.loads([l for l in so.splitlines() if l.startswith("{")][-1]))
    r0 = outs[0]
    assert r0["dist"]["world"] == world and r0["dist"]["partitioned"] == 1
    for run_i, run in enumerate(r0["runs"]):
        assert run["inertia"] == run["ref_inertia"]
        assert all(o["runs"][run_i]["inertia"] == run["inertia"] for o in outs)
        assert run["rel_residual"] < RES_TOL
        assert run["max_rel_diff"] < 1e-9
    assert all(o["stats"]["solve_grid"] > 0 for o in outs)  # the dataflow subtree solve was armed
    n_coll, n_send = check_comm_traces([[tuple(t) for t in o["comm_trace"]] for o in outs])
    assert n_coll > 0 and n_send > 0


@pytest.mark.gpu
@pytest.mark.parametrize("aborting_rank", [0, 1])
def test_distributed_abort_on_one_rank(ua, aborting_rank):
    """a dataflow-solve abort on ONE rank only.  The abort flag is all-reduced before any rank
    writes x, so no rank writes x from a peer's invalid top values, and every rank redoes the solve level by
    level; with x aliasing the rhs (in-place device solve) the redo still starts from b.  Rank 0's gathered
    solution equals the single-GPU one."""
    import torch
    n, nv, m, r, c, v, b = ua.arrowband(40000, ua.SEEDS["C2"])
    single = ua.HipKKT(0)
    single.analyze(n, r, c)
    single.factorize(v)
    ref = single.solve(b)
    world = 2
    group = ua.LocalGroup(world)
    out, errs = [None] * world, []

    def rank_main(q):
        try:
            g = ua.HipKKT(0, dist_dataflow_solve=1)
            g.attach_local(group, q)
            g.analyze(n, r, c)
            g.factorize(v)
            g.inertia()
            if q == aborting_rank:
                g.set_option("debug_abort_solves", 1)
            bd = torch.from_numpy(b.copy()).to("cuda")
            g.solve_device(bd.data_ptr(), bd.data_ptr())
            torch.cuda.synchronize()
            out[q] = (bd.cpu().numpy(), g.stats())
            g.close()
        except Exception as e:  # surfaced below
            errs.append((q, repr(e)))

    th = [threading.Thread(target=rank_main, args=(q,)) for q in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    group.close()
    assert not errs, errs
    assert all(o[1]["solve_aborts"] == 1 for o in out)  # every rank saw the all-reduced verdict
    np.testing.assert_allclose(out[0][0], ref, rtol=1e-12, atol=1e-14 * np.abs(ref).max())


def test_partition_gate_cpu(ua):
    """SURVEY.md 8(e) / north_star gate, host only: the arrowband family exposes enough balanced subtrees, so
    world ranks partition it (estimated efficiency >= 0.5); a dense system (one front) and a tiny chain
    expose too little, so the group declines and runs replicas."""
    n, _, _, r, c, _, _ = ua.arrowband(60000, ua.SEEDS["C3"])
    for world in (2, 4, 8):
        ok, eff, nsub = ua.debug_partition_gate(n, r, c, world)
        assert ok and eff >= 0.5 and nsub >= world, (world, eff, nsub)
    k = 120  # dense: one front, no independent subtrees
    rr, cc = np.tril_indices(k)
    ok, eff, nsub = ua.debug_partition_gate(k, rr, cc, 4)
    assert not ok and nsub < 4
    rr = np.arange(1, 200)  # a path of 200 nodes: separators of 1 node, but little work to split
    ok8, eff8, _ = ua.debug_partition_gate(200, np.concatenate([np.arange(200), rr]),
                                           np.concatenate([np.arange(200), rr - 1]), 8, min_efficiency=0.99)
    assert not ok8 and eff8 < 0.99


@pytest.mark.gpu
def test_declined_partition_runs_replicas(ua):
    """The declined outcome on the GPU: a dense indefinite system in a 2-rank in-process group is not split
    (dist_info partitioned == 0); every rank factors and solves the whole matrix itself, so every rank's
    inertia and solution equal the single-GPU ones, with no collective on the data path."""
    rng = np.random.default_rng(3)
    k = 150
    M = rng.standard_normal((k, k))
    S = M + M.T
    rr, cc = np.tril_indices(k)
    vv = S[rr, cc]
    b = rng.standard_normal(k)
    single = ua.HipKKT(0)
    single.analyze(k, rr, cc)
    single.factorize(vv)
    ine, x = single.inertia(), single.solve(b)
    out = run_group(ua, 2, k, rr, cc, (vv,), b)
    for q in range(2):
        assert out[q][1]["partitioned"] == 0
        assert out[q][0][0][0] == ine
        np.testing.assert_array_equal(out[q][0][0][1], x)


@pytest.mark.gpu
def test_gate_agrees_across_ranks(ua):
    """The partition gate is all-reduced: rank 0 would partition (dist_min_efficiency 0), rank 1 declines
    (dist_min_efficiency 2, unreachable); every rank must take the declined outcome (no rank left waiting in
    a collective the replicas never join), with the single-GPU inertia and solution on each rank."""
    n, nv, m, r, c, v, b = ua.arrowband(40000, ua.SEEDS["C2"])
    single = ua.HipKKT(0)
    single.analyze(n, r, c)
    single.factorize(v)
    ine, x = single.inertia(), single.solve(b)
    group = ua.LocalGroup(2)
    out, errs = [None, None], []

    def rank_main(q):
        try:
            g = ua.HipKKT(0, dist_min_efficiency=0.0 if q == 0 else 2.0)
            g.attach_local(group, q)
            g.analyze(n, r, c)
            g.factorize(v)
            out[q] = (g.inertia(), g.solve(b), g.dist_info())
            g.close()
        except Exception as e:  # surfaced below
            errs.append((q, repr(e)))

    th = [threading.Thread(target=rank_main, args=(q,)) for q in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    group.close()
    assert not errs, errs
    for q in range(2):
        assert out[q][2]["partitioned"] == 0
        assert out[q][0] == ine
        np.testing.assert_array_equal(out[q][1], x)


def test_comm_trace_checker_catches_mismatches():
    """The RCCL-program checker of test_multiprocess_rccl_call_sequence rejects a size mismatch, a send outside
    a group, diverging collectives, and an exchange enqueued off the main stream or before a side stream's factor
    launches were joined (CPU only: synthetic traces)."""
    O = ("order", 1, 0, -1)
    good = [[("group_begin", -1, 0, -1), O, ("send", 1, 64, -1), ("group_end", -1, 0, -1), O, ("allreduce", -1, 24, 0)],
            [("group_begin", -1, 0, -1), O, ("recv", 0, 64, -1), ("group_end", -1, 0, -1), O, ("allreduce", -1, 24, 0)]]
    assert check_comm_traces(good) == (1, 1)
    bad_size = [good[0], [t if t[0] != "recv" else ("recv", 0, 56, -1) for t in good[1]]]
    bad_group = [[t for t in good[0] if t[0] != "group_begin" and t[0] != "group_end"], good[1]]
    bad_coll = [good[0], good[1][:-1] + [("allreduce", -1, 24, 1)]]
    bad_stream = [[("order", 0, 0, -1) if i == 1 else t for i, t in enumerate(good[0])], good[1]]
    bad_join = [good[0], [("order", 1, 1, -1) if i == 4 else t for i, t in enumerate(good[1])]]
    bad_missing = [[t for i, t in enumerate(good[0]) if i != 1], good[1]]
    for bad in (bad_size, bad_group, bad_coll, bad_stream, bad_join, bad_missing):
        with pytest.raises(AssertionError):
            check_comm_traces(bad)
