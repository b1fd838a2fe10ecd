"""One rank of the multi-process distributed factorization on ONE GPU (tests/test_distributed.py):
torch.distributed over gloo carries the library's exchange through the host-staged transport
(uno_kkt_attach_host), so the partitioned factorization and solve run across real processes.
usage: python tests/dist_host_worker.py RANK WORLD PORT N"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    rank, world, port, n = (int(a) for a in sys.argv[1:5])
    # optional 5th argument "rccl_sequence": the options the RCCL transport runs with by default (the dataflow
    # subtree solve on, dist_dataflow_solve = 1) and the transport calls recorded (comm_trace) for the test to
    # match sends with receives and collectives across ranks
    rccl_sequence = len(sys.argv) > 5 and sys.argv[5] == "rccl_sequence"
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import numpy as np
    import torch
    import torch.distributed as dist
    torch.cuda.is_available()  # torch's HIP runtime first (tests/conftest.py)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import uno_amd
    uno_amd.load_library()
    N, nv, m, r, c, v, b = uno_amd.arrowband(n, uno_amd.SEEDS["C5"])
    g = uno_amd.HipKKT(0, comm_trace=1, dist_dataflow_solve=1) if rccl_sequence else uno_amd.HipKKT(0)
    g.attach_host(uno_amd.GlooComm(), rank, world)
    g.analyze(N, r, c)
    out = {"rank": rank, "dist": g.dist_info(), "runs": []}
    v2 = v.copy()
    v2[:nv] = 1e-2  # an inertia-correction retry: new regularization diagonal, same pattern
    v2[nv:N] = -1e-9
    for vals in (v, v2):
        g.factorize(vals)
        ine = g.inertia()
        x = g.solve(b)
        run = {"inertia": list(ine)}
        if rank == 0:
            ref = uno_amd.HipKKT(0)  # the single-GPU path on the same system
            ref.analyze(N, r, c)
            ref.factorize(vals)
            xr = ref.solve(b)
            res = np.abs(uno_amd.coo_symv(N, r, c, vals, x) - b).max()
            absk = uno_amd.coo_symv(N, r, c, np.abs(vals), np.ones(N)).max()
            run.update(ref_inertia=list(ref.inertia()), max_rel_diff=float(np.abs(x - xr).max() / np.abs(xr).max()),
                       rel_residual=float(res / (absk * np.abs(x).max() + np.abs(b).max())))
            ref.close()
        out["runs"].append(run)
    out["stats"] = {k: g.stats()[k] for k in ("factorizations", "solves", "solve_grid", "solve_aborts")}
    if rccl_sequence:
        out["comm_trace"] = g.debug_comm_trace()
    g.close()
    dist.barrier()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
