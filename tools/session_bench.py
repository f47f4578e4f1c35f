"""Receiver-session push cost by batch size, without sockets: the lossy,
reordered k = 10 / 1,200-B stream of tools/rx_bench.py pushed through
rfec_rx_session_push_datagrams in fixed batches from pinned slots, with the
session's eviction called every --evict-every pushes.  Reports per-push time
and the report's host / device / D2H split; the recovered count must not depend
on the batch size.  --lib loads another build of the library (A/B).

Usage (GPU box): python tools/session_bench.py [--batches 256,1024,4096] [--pipelined] [--lib path] [--out file.json]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tools")]

from razor_amd.fec import RX_SEG_DTYPE, Native, rfec_rx_report  # noqa: E402
from rx_bench import DSTRIDE, S, STRIDE, stream  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16384)
    ap.add_argument("--batches", default="256,1024,4096")
    ap.add_argument("--evict-every", type=int, default=8)
    ap.add_argument("--lib", default="")
    ap.add_argument("--pageable-out", action="store_true", help="payload output in pageable memory")
    ap.add_argument("--pipelined", action="store_true",
                    help="rfec_rx_session_push_datagrams_async: each call ingests the previous batch")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    lib = Native(1200, args.lib or None)
    dgram, dlen, ns, nf = stream(lib, args.frames, 0.05, 32)
    n = len(dlen)
    pin = lib.lib.rfec_pinned_alloc(n * DSTRIDE + n * 2 + 256)
    slots = np.ctypeslib.as_array((C.c_uint8 * (n * DSTRIDE)).from_address(pin)).reshape(n, DSTRIDE)
    lens = np.ctypeslib.as_array((C.c_uint16 * n).from_address(pin + n * DSTRIDE))
    slots[:] = dgram
    lens[:] = dlen
    res = {"datagrams": n, "lib": args.lib or "in-tree", "evict_every": args.evict_every,
           "output": "pageable" if args.pageable_out else "pinned",
           "push": "pipelined" if args.pipelined else "synchronous", "batches": {}}
    for B in [int(x) for x in args.batches.split(",")]:
        cap = B + 256
        out = np.zeros(cap, RX_SEG_DTYPE)
        if args.pageable_out:
            outp = np.zeros((cap, STRIDE), np.uint8)
        else:  # pinned, as a receive loop would keep its output rows
            outp, keep = lib.pinned_array((cap, STRIDE), np.uint8)
        h = lib.lib.rfec_rx_session_create(STRIDE, S)
        nout, rep = C.c_uint32(), rfec_rx_report()
        tot = {"host_us": 0.0, "kernel_us": 0.0, "d2h_us": 0.0}
        recovered, pushes = 0, 0
        t0 = time.perf_counter()
        push = (lib.lib.rfec_rx_session_push_datagrams_async if args.pipelined else
                lib.lib.rfec_rx_session_push_datagrams)
        for a in list(range(0, n, B)) + ([n] if args.pipelined else []):
            m = min(B, n - a)  # pipelined: a last call with m = 0 flushes
            rc = push(h, m, DSTRIDE, slots[a:].ctypes.data if m else None, lens[a:].ctypes.data if m else None,
                      None, out.ctypes.data, outp.ctypes.data, cap, C.byref(nout), C.byref(rep))
            if rc:
                raise SystemExit(f"push failed: {lib.last_error()}")
            recovered += nout.value
            for f in tot:
                tot[f] += getattr(rep, f)
            pushes += m > 0
            if m and args.evict_every and pushes % args.evict_every == 0:
                lib.lib.rfec_rx_session_evict(h, None)
        dt = time.perf_counter() - t0
        lib.lib.rfec_rx_session_destroy(h)
        res["batches"][str(B)] = {"pushes": pushes, "us_per_push": dt / pushes * 1e6, "datagrams_per_s": n / dt,
                                  "recovered": recovered,
                                  **{f + "_per_push": v / pushes for f, v in tot.items()}}
        print(B, json.dumps(res["batches"][str(B)]), flush=True)
    lib.lib.rfec_pinned_free(pin)
    rec = {v["recovered"] for v in res["batches"].values()}
    res["consistent"] = len(rec) == 1
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1))
    if not res["consistent"]:
        raise SystemExit(f"recovered counts differ across batch sizes: {rec}")


if __name__ == "__main__":
    main()
