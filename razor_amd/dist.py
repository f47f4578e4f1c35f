"""Multi-GPU batch split.

FEC groups are independent: flex_fec_sender_update never reads across groups
(sim_transport/fec/flex_fec_sender.c:146-245) and the receiver keys all state
by fec_id (sim_transport/sim_fec.c:152-166).  So N GPUs take contiguous slices
[d*G/N, (d+1)*G/N) of the batch, one process per GPU, with no data-path
collective; the only communication is the control-plane barrier and the
max-over-ranks reduction of the timed region.
"""
from __future__ import annotations

import time


def shard_groups(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous slice of `total` groups for `rank` of `world`: (first, count)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    lo = total * rank // world
    hi = total * (rank + 1) // world
    return lo, hi - lo


def timed_steps(step, steps: int, warmup: int, sync, dist=None, reduce_device=None) -> float:
    """Runs `warmup` untimed steps, then times exactly `steps` steps bracketed by
    barrier + sync on both sides; returns the max over ranks (seconds)."""
    for _ in range(warmup):
        step()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64, device=reduce_device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed
