"""CPU test of the host-staged exchange's Python half (uno_amd.GlooComm): two processes over gloo call the
uno_kkt_host_comm_t callbacks through their C function pointers exactly as the library's HostTransport does
(uno_amd/csrc/comm.cpp): a batch of send / recv completed by group_end, the four all-reduce ops on 8-byte
elements, broadcast.  The GPU side (staging, the partitioned factorization) is
tests/test_distributed.py::test_multiprocess_host_transport."""
import ctypes
import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import uno_amd
    c = uno_amd.GlooComm()
    s = c.struct
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    res = {}
    # a group: every rank sends 3 doubles to every other rank, receives theirs
    outs = {p: np.arange(3, dtype=np.float64) + 10 * rank + p for p in range(world) if p != rank}
    ins = {p: np.zeros(3) for p in range(world) if p != rank}
    for p in outs:
        assert s.send(None, ptr(outs[p]), 24, p) == 0
    for p in ins:
        assert s.recv(None, ptr(ins[p]), 24, p) == 0
    assert s.group_end(None) == 0
    res["recv"] = {p: ins[p].tolist() for p in ins}
    for op, arr in ((0, np.array([rank + 1, 5], dtype=np.uint64)), (1, np.array([rank, 7 - rank], dtype=np.uint64)),
                    (2, np.array([0.5 * rank, -1.0])), (3, np.array([0.25, rank * 1.0]))):
        assert s.allreduce(None, ptr(arr), 2, op) == 0
        res[f"op{op}"] = arr.tolist()
    b = np.full(4, float(rank))
    assert s.broadcast(None, ptr(b), 32, 1) == 0
    res["bcast"] = b.tolist()
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_host_comm_callbacks():
    world = 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        o = 1 - r
        assert got[r]["recv"][o] == [10 * o + r + k for k in range(3)]
        assert got[r]["op0"] == [3, 10]
        assert got[r]["op1"] == [1, 7]
        assert got[r]["op2"] == [0.5, -1.0]
        assert got[r]["op3"] == [0.5, 1.0]
        assert got[r]["bcast"] == [1.0] * 4
