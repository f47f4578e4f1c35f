"""CPU, world_size 2 over gloo: the batch split used by bench.py --gpus N
(razor_amd/dist.py) covers every group exactly once, needs no data-path
collective, and reproduces the single-process result.  The oracle stands in
for the GPU engine here (this test runs without a GPU)."""
import hashlib
import json
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _digest(parity, meta, fsize):
    h = hashlib.sha256()
    for a in (parity, meta, fsize):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def _worker(rank, world, port, total, outdir):
    sys.path[:0] = [str(ROOT), str(ROOT / "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    from pyoracle import Oracle
    from razor_amd.dist import shard_groups, timed_steps

    dist.init_process_group("gloo", rank=rank, world_size=world)
    o = Oracle(1200)
    shards, hdr = o.fill_groups(42, total, 10, 1200, ragged=True)
    lo, n = shard_groups(total, world, rank)
    plan = o.plan_from_fraction(10, 80, 1)
    out = {}

    def step():
        out["r"] = o.encode_batch(plan, shards[lo:lo + n], hdr[lo:lo + n], 1200)

    win = timed_steps(step, steps=3, warmup=1, sync=lambda: None, dist=dist)
    parity, meta, fsize, status = out["r"]
    digs = [None] * world
    dist.all_gather_object(digs, {"lo": lo, "n": n, "digest": [_digest(parity[g], meta[g], fsize[g])
                                                               for g in range(n)]})
    if rank == 0:
        Path(outdir, "result.json").write_text(json.dumps({"shards": digs, "window": win}))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("total", [64, 7])
def test_batch_split_world2(tmp_path, total):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), total, str(tmp_path)), nprocs=world, join=True)
    res = json.loads((tmp_path / "result.json").read_text())
    sys.path[:0] = [str(ROOT / "oracle")]
    from pyoracle import Oracle

    o = Oracle(1200)
    shards, hdr = o.fill_groups(42, total, 10, 1200, ragged=True)
    parity, meta, fsize, _ = o.encode_batch(o.plan_from_fraction(10, 80, 1), shards, hdr, 1200)
    whole = [_digest(parity[g], meta[g], fsize[g]) for g in range(total)]
    got = []
    expect_lo = 0
    for s in res["shards"]:
        assert s["lo"] == expect_lo  # contiguous, no overlap, no gap
        expect_lo += s["n"]
        got += s["digest"]
    assert expect_lo == total
    assert got == whole
    # the window bench.py's time_steps uses (razor_amd/dist.StepWindow): every rank's CLOCK_MONOTONIC t0 / t1,
    # the job's time from the first start to the last stop, skews >= 0
    w = res["window"]
    assert len(w["t0_us"]) == len(w["t1_us"]) == world
    assert min(w["t0_us"]) == 0 and w["start_skew_us"] == max(w["t0_us"]) >= 0 and w["stop_skew_us"] >= 0
    assert all(b >= a for a, b in zip(w["t0_us"], w["t1_us"]))
    assert w["elapsed_s"] >= w["rank_elapsed_max_s"] > 0
    assert abs(w["elapsed_s"] * 1e6 - max(w["t1_us"])) < 1.0


def test_shard_groups_cover():
    from razor_amd.dist import shard_groups

    for total in (0, 1, 7, 65536, 1 << 20):
        for world in (1, 2, 3, 4, 8):
            spans = [shard_groups(total, world, r) for r in range(world)]
            assert sum(n for _, n in spans) == total
            assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            assert max(n for _, n in spans) - min(n for _, n in spans) <= 1


def test_bench_digest_rules():
    """bench.py's reference digest per rank: the whole case at N = 1, the
    strong-scaling slices of config 4, the weak-scaling chunks of the config 3
    stream (chunk 0 is config 3's own digest)."""
    sys.path[:0] = [str(ROOT)]
    import bench

    cases = {c["name"]: c for c in json.loads(bench.GOLDEN.read_text())["cases"]}
    c2, weak, c4 = (cases["c2_k10_rows_S1200_G65536"], cases["c3_weak_k10_rows_S1200_G524288"],
                    cases["c4_k10_rows_S1200_G1048576"])
    assert bench.golden_digest("c2_k10_rows_S1200_G65536", 1, 0) == c2["sha256"]
    assert weak["chunk"] == 65536 and len(weak["chunks"]) == 8 and weak["chunks"][0] == c2["sha256"]
    for r in range(8):
        assert bench.golden_digest(bench.CONFIGS["c3"]["weak_golden"], 8, r, chunk=65536) == weak["chunks"][r]
    assert bench.golden_digest(bench.CONFIGS["c3"]["weak_golden"], 2, 1, chunk=4096) is None
    for n in (2, 4, 8):
        assert [bench.golden_digest("c4_k10_rows_S1200_G1048576", n, r) for r in range(n)] == c4["slices"][str(n)]
