"""Timing harness for the multi-GPU bench.

The only collectives are the barriers bracketing the timed region and one MAX all-reduce of the
per-rank elapsed time; `value` is then all ranks' factor+solves / that max.  Kept free of GPU calls
so the same code runs under gloo on the CPU in the tests (tests/test_replicas.py).
"""
import time


def timed_steps(step, steps, warmup, sync, world, device=None):
    """Run `warmup` untimed and `steps` timed calls of `step`, bracketed by barrier + `sync`.

    Returns (max-over-ranks elapsed seconds, last step result)."""
    import torch
    import torch.distributed as dist
    out = None
    for _ in range(warmup):
        out = step()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    sync()
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item()), out


def share_bytes(payload, world):
    """Broadcast a small bytes object from rank 0 (the RCCL unique id of the library's communicator)."""
    import torch.distributed as dist
    if world <= 1:
        return payload
    box = [payload]
    dist.broadcast_object_list(box, src=0)
    return box[0]


def aggregate(steps, world, elapsed):
    """Whole-job throughput (weak scaling: every rank does `steps` units) and ms per step."""
    return steps * world / elapsed, 1e3 * elapsed / steps
