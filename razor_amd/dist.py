"""Multi-GPU batch split and the bench's cross-rank clock.

FEC groups are independent: flex_fec_sender_update never reads across groups
(sim_transport/fec/flex_fec_sender.c:146-245) and the receiver keys all state
by fec_id (sim_transport/sim_fec.c:152-166).  So N GPUs take contiguous slices
[d*G/N, (d+1)*G/N) of the batch, one process per GPU, with no data-path
collective; the only communication is the control plane (a CPU gloo group):
the barriers around the timed region and the exchange of each rank's clock
readings.

Timing (StepWindow): every rank reads CLOCK_MONOTONIC after the opening
barrier + device synchronize (t0) and after its closing synchronize (t1),
before the closing barrier.  The ranks of one node share that clock, so the
whole job's time is max(t1) - min(t0): from the first rank starting to the
last rank finishing, with the barrier-exit skew between the ranks' starts
(start_skew_us) measured instead of folded into one rank's elapsed time.
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


def mono_ns() -> int:
    """CLOCK_MONOTONIC in ns: one clock for every process of the node."""
    return time.clock_gettime_ns(time.CLOCK_MONOTONIC)


class StepWindow:
    """The timed region of bench.py (and of timed_steps): start() = barrier,
    sync, t0; stop() = sync, t1, barrier; reduce() exchanges every rank's
    (t0, t1) over the control-plane group and returns the job's window."""

    def __init__(self, dist=None, sync=lambda: None):
        self.dist, self.sync = dist, sync
        self.t0 = self.t1 = None

    def start(self):
        if self.dist is not None:
            self.dist.barrier()
        self.sync()
        self.t0 = mono_ns()

    def stop(self):
        self.sync()
        self.t1 = mono_ns()
        if self.dist is not None:
            self.dist.barrier()

    def reduce(self) -> dict:
        """elapsed_s = max(t1) - min(t0) over the ranks; rank_elapsed_max_s =
        max(t1 - t0) (the old max-over-ranks rule, for comparison);
        start_skew_us / stop_skew_us = the spread of the ranks' t0 / t1;
        t0_us / t1_us = every rank's readings relative to min(t0)."""
        if self.t0 is None or self.t1 is None:
            raise RuntimeError("StepWindow.reduce before start/stop")
        pairs = [(self.t0, self.t1)]
        if self.dist is not None:
            import torch

            mine = torch.tensor([self.t0, self.t1], dtype=torch.int64)
            allp = [torch.zeros(2, dtype=torch.int64) for _ in range(self.dist.get_world_size())]
            self.dist.all_gather(allp, mine)
            pairs = [(int(p[0]), int(p[1])) for p in allp]
        t0s, t1s = [p[0] for p in pairs], [p[1] for p in pairs]
        base = min(t0s)
        return {"elapsed_s": (max(t1s) - base) / 1e9,
                "rank_elapsed_max_s": max(b - a for a, b in pairs) / 1e9,
                "start_skew_us": round((max(t0s) - base) / 1e3, 2),
                "stop_skew_us": round((max(t1s) - min(t1s)) / 1e3, 2),
                "t0_us": [round((a - base) / 1e3, 2) for a in t0s],
                "t1_us": [round((b - base) / 1e3, 2) for b in t1s],
                "clock": "CLOCK_MONOTONIC (one node: comparable across ranks)"}


def timed_steps(step, steps: int, warmup: int, sync, dist=None) -> dict:
    """Runs `warmup` untimed steps, then times exactly `steps` steps in a
    StepWindow; returns its reduce() (elapsed_s = the job's window)."""
    for _ in range(warmup):
        step()
    w = StepWindow(dist, sync)
    w.start()
    for _ in range(steps):
        step()
    w.stop()
    return w.reduce()


def device_identity(device) -> dict:
    """The physical GPU a rank ran on: index, PCI domain:bus:device, name and
    UUID (so a scaling line shows N distinct devices)."""
    import torch

    p = torch.cuda.get_device_properties(device)
    return {"device": int(torch.device(device).index or 0),
            "pci_bus_id": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0",
            "name": p.name, "uuid": str(getattr(p, "uuid", ""))}


def gather_objects(dist, obj) -> list:
    """Every rank's `obj` (rank order) over the control-plane group; [obj] alone."""
    if dist is None:
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out
