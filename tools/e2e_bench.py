"""End-to-end (host memory in, host memory out) encode rate, stage by stage,
through rfec_host_encode_groups: gather from sim_segment_t (AoS, payload at
offset 34) into pinned SoA -> H2D -> encode kernel -> D2H -> scatter into
sim_fec_t.  The path starts and ends in host memory like the reference's
(UDP socket buffers, sim_session.c); the device-resident rate is bench.py's.

Usage (GPU box): python tools/e2e_bench.py [--groups 65536] [--reps 5] [--out file.json]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "oracle")]

from razor_amd.fec import HDR_DTYPE, fec_dtype, native, seg_dtype  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    G, k, S = args.groups, 10, 1200
    lib = native(1200)
    plan = lib.plan_from_fraction(k, 80, 1)
    n = plan.n_lines
    rng = np.random.default_rng(11)
    segs = np.zeros(G * k, seg_dtype(1200))
    segs["data"] = rng.integers(0, 256, (G * k, S), dtype=np.uint8)
    gi = np.repeat(np.arange(G, dtype=np.uint64), k)
    ii = np.tile(np.arange(k, dtype=np.uint64), G)
    segs["packet_id"] = (1 + gi * k + ii).astype(np.uint32)
    segs["fid"] = (1 + gi).astype(np.uint32)
    segs["timestamp"] = (33 * gi).astype(np.uint32)
    segs["index"] = ii
    segs["total"] = k
    segs["ftype"] = (gi % 60 == 0)
    segs["data_size"] = S
    fecs = np.zeros(G * n, fec_dtype(1200))
    sp = segs.ctypes.data + np.arange(G * k, dtype=np.uint64) * segs.dtype.itemsize
    fp = fecs.ctypes.data + np.arange(G * n, dtype=np.uint64) * fecs.dtype.itemsize
    lib.host_encode_groups(plan, G, sp, fp)  # warm: staging allocation
    runs = [lib.host_encode_groups(plan, G, sp, fp) for _ in range(args.reps)]
    med = {key: float(np.median([r[key] for r in runs])) for key in runs[0]}
    # verify a sample against the oracle
    from pyoracle import Oracle

    o = Oracle(1200)
    idx = np.r_[0:4, G // 2:G // 2 + 4, G - 4:G]
    sh = segs["data"].reshape(G, k, S)[idx]
    hdr = np.zeros((len(idx), k), HDR_DTYPE)
    sg = segs.reshape(G, k)[idx]
    for a, b in (("seq", "packet_id"), ("fid", "fid"), ("ts", "timestamp"), ("index", "index"), ("total", "total"),
                 ("ftype", "ftype"), ("payload_type", "payload_type"), ("size", "data_size")):
        hdr[a] = sg[b]
    par, meta, fs, _ = o.encode_batch(o.plan_from_fraction(k, 80, 1), sh, hdr, S)
    f = fecs.reshape(G, n)[idx]
    ok = bool(np.array_equal(f["fec_data"], par) and np.array_equal(f["meta"], meta)
              and np.array_equal(f["fec_data_size"], fs)
              # fec_id runs 1, 2, ... and wraps past 65535 to 1 (flex_fec_sender.c:241-243)
              and np.all(f["fec_id"] == (idx[:, None] % 65535 + 1)) and np.all(f["base_id"] == hdr["seq"][:, :1]))
    enc_bytes = G * (k + n) * S
    res = {"groups": G, "k": k, "r": n, "payload": S, "reps": args.reps, "median_us": med,
           "enc_algorithmic_bytes": enc_bytes,
           "e2e_GiBps": enc_bytes / (med["total_us"] * 1e-6) / 2**30,
           "pcie_inclusive_GiBps": enc_bytes / ((med["h2d_us"] + med["kernel_us"] + med["d2h_us"]) * 1e-6) / 2**30,
           "device_resident_GiBps": enc_bytes / (med["kernel_us"] * 1e-6) / 2**30,
           "h2d_GBps": (G * k * (1216 - 16 + 20)) / (med["h2d_us"] * 1e-6) / 1e9,
           "verified_sample": ok}
    print(json.dumps(res, indent=1))
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1))
    if not ok:
        raise SystemExit("e2e verification failed")


if __name__ == "__main__":
    main()
