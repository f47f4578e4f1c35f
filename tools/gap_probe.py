"""Measurement only (GPU box): what the default bench step (c3: encode one
buffer set, decode the other) spends between its two kernels.  Times K steps
three ways, interleaved: no events at all, the kernels' own events
(hipExtLaunchKernel, the bench's default), stream events around each call;
prints ms per step for each and the kernels' own durations.

    python tools/gap_probe.py [--steps 100] [--rounds 3]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT)]

import bench  # noqa: E402
from razor_amd.fec import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = native(1000)
    cfg = bench.CONFIGS["c3"]
    sets = [bench.Workload(lib, cfg["groups"], cfg["k"], cfg["S"], 80, dev, 0, seed=1000, config_id=cfg["config_id"])
            for _ in range(2)]
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    for w in sets:
        w.encode(sp)
    for i in range(10):
        sets[i % 2].encode(sp)
        sets[(i - 1) % 2].decode(sp)
    torch.cuda.synchronize(dev)
    K = args.steps
    kev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(4)) for _ in range(K)]
    sev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(4)) for _ in range(K)]
    for q in kev + sev:
        for e in q:
            e.record(stream)
    torch.cuda.synchronize(dev)

    def run(mode):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(K):
            if mode == "own":
                lib.timing_events(kev[i][0].cuda_event, kev[i][1].cuda_event)
            elif mode == "bracket":
                sev[i][0].record(stream)
            sets[i % 2].encode(sp)
            if mode == "bracket":
                sev[i][1].record(stream)
            if mode == "own":
                lib.timing_events(kev[i][2].cuda_event, kev[i][3].cuda_event)
            elif mode == "bracket":
                sev[i][2].record(stream)
            sets[(i - 1) % 2].decode(sp)
            if mode == "bracket":
                sev[i][3].record(stream)
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) * 1e3 / K
        out = {"ms_per_step": round(ms, 4)}
        if mode == "own":
            out["encode_us"] = round(float(np.mean([a.elapsed_time(b) for a, b, _, _ in kev])) * 1e3, 1)
            out["decode_us"] = round(float(np.mean([c.elapsed_time(d) for _, _, c, d in kev])) * 1e3, 1)
        if mode == "bracket":
            out["encode_us"] = round(float(np.mean([a.elapsed_time(b) for a, b, _, _ in sev])) * 1e3, 1)
            out["decode_us"] = round(float(np.mean([c.elapsed_time(d) for _, _, c, d in sev])) * 1e3, 1)
        return out

    res = {m: [] for m in ("none", "own", "bracket")}
    for _ in range(args.rounds):
        for m in res:
            res[m].append(run(m))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
