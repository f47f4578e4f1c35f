"""Measurement only (GPU box): host -> device bandwidth of the ways the
host-memory paths (rfec_host_encode_groups / rfec_host_recover_groups) could
move a chunk: one hipMemcpyAsync from pinned memory, the same split over two
or four streams (more DMA engines), and the GPU reading the pinned memory
itself (rfec_probe_copy over the host-mapped pointer: every CU's loads cross
PCIe).  Also device -> host, one copy and two.

    python tools/h2d_probe.py [--mib 512] [--reps 5]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT)]

from razor_amd.fec import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=512)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = native(1000)
    n = args.mib << 20
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h.fill_(7)
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    torch.cuda.synchronize()

    def timed(fn):
        best = 1e30
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return round(n / best / 1e9, 1)

    def split(k, h2d=True):
        def f():
            part = n // k
            for i in range(k):
                with torch.cuda.stream(streams[i]):
                    if h2d:
                        d[i * part:(i + 1) * part].copy_(h[i * part:(i + 1) * part], non_blocking=True)
                    else:
                        h[i * part:(i + 1) * part].copy_(d[i * part:(i + 1) * part], non_blocking=True)
        return f

    def zero_copy():
        rc = lib.lib.rfec_probe_copy(C.c_void_p(h.data_ptr()), C.c_void_p(d.data_ptr()), C.c_size_t(n), C.c_uint(1),
                                     C.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
        assert rc == 0, rc

    out = {"bytes": n, "GBps": {
        "h2d_1_stream": timed(split(1)), "h2d_2_streams": timed(split(2)), "h2d_4_streams": timed(split(4)),
        "h2d_gpu_reads_pinned": timed(zero_copy),
        "d2h_1_stream": timed(split(1, False)), "d2h_2_streams": timed(split(2, False))}}
    ok = bool(torch.equal(d[:1 << 20].cpu(), h[:1 << 20]))
    out["verified"] = ok
    print(json.dumps(out))


if __name__ == "__main__":
    main()
