"""The receiver session's host control plane alone, on the CPU (no GPU): the C
host layer built with tests/host_stub/stub_hip.c (a host-memory stand-in for
the HIP runtime; it computes no payload), driven with the parsed records of a
c3 stream (k = 10, the sender's 3 x 4 plan, `--loss` loss, reordering within
`--window` arrivals, 2 % duplicates) in batches of `--batch` arrivals through
rfec_rx_session_push.  Reports the library's own host_us per arrival (the
arrival-order control plane + building the device tables) and checks the
delivered headers against the oracle's event-by-event receiver.

A development tool for the control plane's cost (the GPU box measures the real
path: tools/rx_session_bench.py).

Usage: python tools/rx_host_bench.py [--groups 65536] [--batch 4096] [--threads N]
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "oracle")]

sys.path.insert(0, str(ROOT / "tests"))
from razor_amd.build import HOST_SRC  # noqa: E402
from razor_amd.fec import RX_SEG_DTYPE, Native, rfec_rx_report  # noqa: E402
from rx_cases import c3_records  # noqa: E402

ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
CAP = 16  # payload capacity / row stride: the control plane reads sizes only


def build_stub(out: Path, opt="-O2") -> Path:
    inc = [f"-I{ROCM / 'include'}", f"-I{ROOT / 'include'}", f"-I{ROOT / 'razor_amd' / 'csrc'}"]
    cmd = ["gcc", "-std=c99", opt, "-g", "-fPIC", "-shared", "-DSIM_VIDEO_SIZE=1200", "-D__HIP_PLATFORM_AMD__", *inc,
           *(str(ROOT / "razor_amd" / "csrc" / f) for f in HOST_SRC), str(ROOT / "razor_amd" / "csrc" / "rfec_net.c"),
           str(ROOT / "tests" / "host_stub" / "stub_hip.c"), "-o", str(out), "-lpthread", "-lm"]
    subprocess.run(cmd, check=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=65536)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--loss", type=float, default=0.05)
    ap.add_argument("--window", type=int, default=32)
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--lib", default="")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--evict", type=int, default=1,
                    help="rfec_rx_session_evict after every push (the heartbeat's sim_fec_evict); 0: never")
    args = ap.parse_args()
    so = Path(args.lib) if args.lib else build_stub(Path("/tmp/librazor_fec_rxhost.so"))
    lib = Native(1200, path=str(so))
    recs = c3_records(args.groups, args.loss, args.window, cap=CAP)
    n = len(recs)
    pay = np.zeros((n, CAP), np.uint8)
    sess = lib.rx_session(CAP, CAP, args.threads)
    max_out = 4 * args.batch
    out = np.zeros(max_out, RX_SEG_DTYPE)
    outp = np.zeros((max_out, CAP), np.uint8)
    nout, rep = C.c_uint32(), rfec_rx_report()
    got = []
    host = dev = tot = 0.0
    t0 = time.perf_counter()
    for a0 in range(0, n, args.batch):
        m = min(args.batch, n - a0)
        lib._check(lib.lib.rfec_rx_session_push(sess.h, m, recs.ctypes.data + a0 * 64, pay.ctypes.data + a0 * CAP,
                                                out.ctypes.data, outp.ctypes.data, max_out, C.byref(nout),
                                                C.byref(rep), None), "push")
        got.append(out[:nout.value].copy())
        if args.evict and m == args.batch:
            lib._check(lib.lib.rfec_rx_session_evict(sess.h, None), "evict")
        host += rep.host_us
        dev += rep.kernel_us + rep.h2d_us + rep.d2h_us
        tot += rep.total_us
    wall = time.perf_counter() - t0
    info = sess.info()
    print("session:", info)
    print("split ms:", {k: round(v / 1e3, 2) for k, v in info.items() if k.endswith("_us")})
    got = np.concatenate(got)
    print(f"arrivals {n}  recovered {len(got)}  wall {wall * 1e3:.1f} ms  host_us {host:.0f} "
          f"({host * 1e3 / n:.1f} ns/arrival)  stub-device {dev:.0f} us  total {tot:.0f} us  "
          f"-> {n / (host * 1e-6) / 1e6:.2f} M arrivals/s of host plane")
    if not args.no_verify:
        import pyoracle as po

        o = po.Oracle(1200)
        eo, _, emts, edrop = o.rx_recover(recs, np.zeros((n, CAP), np.uint8), CAP, max_out=1 << 22,
                                    evict_every=args.batch if args.evict else 0)
        i, j = np.argsort(got["hdr"]["seq"], kind="stable"), np.argsort(eo["hdr"]["seq"], kind="stable")
        ok = len(got) == len(eo) and np.array_equal(got["hdr"][i], eo["hdr"][j]) and np.array_equal(
            got["fec_id"][i], eo["fec_id"][j]) and sess.info()["max_ts"] == emts
        print("verified vs oracle:", ok)
        if not ok:
            raise SystemExit(1)


if __name__ == "__main__":
    main()
