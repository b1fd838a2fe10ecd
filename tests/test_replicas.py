"""N>1 bench path on the CPU: world_size-2 gloo run of the replica harness (uno_amd/replicas.py).

Each rank factors and solves its OWN small arrowband KKT (seed + rank, as bench.py does) with the CPU
oracle standing in for the device step; the test checks the contract the driver relies on: both
ranks see the same max-over-ranks time, value = steps * world / max, each rank's solve is correct,
and no rank's system is another's."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import uno_amd
    from oracle_ffi import OracleKKT
    from uno_amd.replicas import aggregate, timed_steps
    n, _, _, r, c, v, b = uno_amd.arrowband(3000, uno_amd.SEEDS["C3"] + rank)
    o = OracleKKT()
    o.analyze(n, r, c)
    state = {}

    def step():
        o.factorize(v)
        state["x"] = o.solve(b)
        return o.inertia()

    steps = 3 + 2 * rank  # ranks do different amounts of local work; the max must win
    elapsed, inertia = timed_steps(step, steps, 1, lambda: None, world)
    value, ms = aggregate(3, world, elapsed)
    x = state["x"]
    res = np.abs(uno_amd.coo_symv(n, r, c, v, x) - b).max() / (np.abs(b).max() + 1e-300)
    out[rank] = (elapsed, value, float(res), tuple(inertia), float(np.abs(v).sum() + b.sum()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_replicas_gloo():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    (e0, v0, r0, i0, s0), (e1, v1, r1, i1, s1) = out[0], out[1]
    assert e0 == e1 > 0                        # max over ranks, identical everywhere
    assert v0 == pytest.approx(3 * world / e0)
    assert r0 < 1e-8 and r1 < 1e-8
    assert sum(i0) == sum(i1) == 3000
    assert s0 != s1                            # independent systems per rank
