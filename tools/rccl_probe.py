"""Two-process RCCL rehearsal of the distributed factorization on the GPUs that are visible (one or
more ranks per GPU).  Unique-id exchange over gloo, then the library's own RCCL communicator.
usage: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/rccl_probe.py [n]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    dev = rank % max(1, torch.cuda.device_count())
    import uno_amd
    from uno_amd.replicas import share_bytes
    n_per = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    n, nv, m, r, c, v, b = uno_amd.arrowband(n_per * world, uno_amd.SEEDS["C2"])
    g = uno_amd.HipKKT(dev)
    uid = share_bytes(uno_amd.rccl_unique_id() if rank == 0 else None, world)
    g.attach_rccl(uid, rank, world)
    g.analyze(n, r, c)
    g.factorize(v)
    ine = g.inertia()
    x = g.solve(b)
    if rank == 0:
        s = uno_amd.HipKKT(dev)
        s.analyze(n, r, c)
        s.factorize(v)
        xs = s.solve(b)
        print(f"rccl probe world={world} n={n} inertia={ine} single={s.inertia()} "
              f"max|dx|={np.abs(x - xs).max():.3e} info={g.dist_info()}", flush=True)
        assert ine == s.inertia()
        assert np.abs(x - xs).max() <= 1e-12 * np.abs(xs).max()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
