"""Measurement only (GPU box): the PCIe link as the zero-copy host paths use
it.  The struct gather kernel (rfec_launch_host_gather over 8 chunks of
sim_segment_t in an rfec_pinned_alloc block) vs contiguous device reads of
pinned memory (rfec_probe_copy) and one DMA; then device reads beside device
writes to host memory (kernel or DMA, whole or per chunk); then 16-B lanes at
a 4-byte offset from 16-B alignment (the structs' data) vs aligned.

    python tools/zc_probe.py [groups_per_chunk=8192]

Prints three JSON lines (GB/s, then ms)."""
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent  # the repo root
sys.path[:0] = [str(ROOT)]
from razor_amd.fec import native, seg_dtype  # noqa: E402

lib = native(1200)
L = lib.lib
hip = C.CDLL("libamdhip64.so")
G, k = int(sys.argv[1]) if len(sys.argv) > 1 else 8192, 10
n = G * k
segs, keep = lib.pinned_array((n * 8,), seg_dtype(1200))  # 8 chunks worth
segs["data_size"] = 1200
segs["data"] = 7
dp = C.c_void_p()
assert hip.hipHostGetDevicePointer(C.byref(dp), C.c_void_p(segs.ctypes.data), 0) == 0
delta = dp.value - segs.ctypes.data
isz = segs.dtype.itemsize
ptr = torch.tensor((segs.ctypes.data + delta + np.arange(n * 8, dtype=np.uint64) * isz).view(np.int64), device="cuda")
dst = torch.empty((2, n, 1216), dtype=torch.uint8, device="cuda")
hdr = torch.empty((2, n, 20), dtype=torch.uint8, device="cuda")
ss = [torch.cuda.Stream(), torch.cuda.Stream()]
out = {}


def timed(fn, nbytes, reps=5):
    best = 1e30
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return round(nbytes / best / 1e9, 2)


def gather(c, s):
    with torch.cuda.stream(ss[s]):
        rc = L.rfec_launch_host_gather(C.c_void_p(ptr.data_ptr() + c * n * 8), n, C.c_void_p(dst[s].data_ptr()),
                                       C.c_void_p(hdr[s].data_ptr()), None, 0, None, None, None, None, 1216, 1200,
                                       None, None, 0, C.c_void_p(ss[s].cuda_stream))
        assert rc == 0


def g1():
    for c in range(8):
        gather(c, 0)


def g2():
    for c in range(8):
        gather(c, c & 1)


total = 8 * n * isz
out["gather_1stream_GBps"] = timed(g1, total)
out["gather_2streams_GBps"] = timed(g2, total)
torch.cuda.synchronize()
ok = bool((dst[0, :, :1200] == 7).all()) and not bool(dst[0, :, 1200:].any())
raw = C.c_void_p(segs.ctypes.data + delta)
flat = torch.empty(total, dtype=torch.uint8, device="cuda")
for fl in (0, 1, 2, 3):
    out[f"probe_copy_flags{fl}_GBps"] = timed(lambda: L.rfec_probe_copy(raw, C.c_void_p(flat.data_ptr()),
                                                                      C.c_size_t(total), fl, None), total)
hsrc = torch.from_numpy(segs.view(np.uint8).reshape(-1))
out["memcpy_h2d_GBps"] = timed(lambda: flat.copy_(hsrc, non_blocking=True), total)
out["verified"] = ok
out["bytes"] = total
print(json.dumps(out))

# --- duplex: device reads of host memory beside device writes to host memory
wbytes = 245 * (1 << 20)
hw, kw = lib.pinned_array((wbytes,), np.uint8)
assert hip.hipHostGetDevicePointer(C.byref(dp), C.c_void_p(hw.ctypes.data), 0) == 0
hwd = C.c_void_p(dp.value)
dsrc = torch.zeros(wbytes, dtype=torch.uint8, device="cuda")
hwt = torch.from_numpy(hw)
res = {}


def wr_kernel(s):
    with torch.cuda.stream(ss[s]):
        assert L.rfec_probe_write(hwd, C.c_size_t(wbytes), 1, C.c_void_p(ss[s].cuda_stream)) == 0


def wr_dma(s):
    with torch.cuda.stream(ss[s]):
        hwt.copy_(dsrc, non_blocking=True)


def gath_all(s):
    for c in range(8):
        gather(c, s)


def timed_ms(fn, reps=5):
    best = 1e30
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return round(best * 1e3, 2)


res["gather_ms"] = timed_ms(lambda: gath_all(0))
res["write_kernel_ms"] = timed_ms(lambda: wr_kernel(1))
res["write_dma_ms"] = timed_ms(lambda: wr_dma(1))
res["gather+write_kernel_ms"] = timed_ms(lambda: (wr_kernel(1), gath_all(0)))
res["gather+write_dma_ms"] = timed_ms(lambda: (wr_dma(1), gath_all(0)))


def interleaved():  # per chunk: write a 1/8 slice between gathers, both streams
    for c in range(8):
        gather(c, 0)
        with torch.cuda.stream(ss[1]):
            L.rfec_probe_write(C.c_void_p(hwd.value + c * (wbytes // 8)), C.c_size_t(wbytes // 8), 1,
                               C.c_void_p(ss[1].cuda_stream))


res["gather+write_kernel_sliced_ms"] = timed_ms(interleaved)
res["read_bytes"] = total
res["write_bytes"] = wbytes
print(json.dumps(res))

# --- alignment: 16-B lanes at a 4-B offset from 16-B alignment
al = {}
al["write_aligned_ms"] = timed_ms(lambda: L.rfec_probe_write(hwd, C.c_size_t(wbytes - 64), 0, None))
al["write_off4_ms"] = timed_ms(lambda: L.rfec_probe_write(C.c_void_p(hwd.value + 4), C.c_size_t(wbytes - 64), 0, None))
al["write_off4_nt_ms"] = timed_ms(lambda: L.rfec_probe_write(C.c_void_p(hwd.value + 4), C.c_size_t(wbytes - 64), 1, None))
al["read_aligned_ms"] = timed_ms(lambda: L.rfec_probe_copy(raw, C.c_void_p(flat.data_ptr()), C.c_size_t(total - 64), 0, None))
al["read_off4_ms"] = timed_ms(lambda: L.rfec_probe_copy(C.c_void_p(raw.value + 4), C.c_void_p(flat.data_ptr()), C.c_size_t(total - 64), 0, None))
al["read_off4_nt_ms"] = timed_ms(lambda: L.rfec_probe_copy(C.c_void_p(raw.value + 4), C.c_void_p(flat.data_ptr()), C.c_size_t(total - 64), 1, None))
print(json.dumps(al))
