"""Receiver ingestion end to end: a lossy, reordered SIM_SEG + SIM_FEC datagram
stream (from the product sender) -> rfec_wire_parse -> rfec_rx_recover, per
stage, verified against the oracle's event-by-event receiver on the whole
stream.  The oracle's time on the same records is reported beside it (one
host core: the reference's receiver is a per-session serial loop).

Workload: F frames of k = 10 x 1,200 bytes at protect_fraction 80 (3 row + 4
column parities per group), `--loss` independent loss, reordering within
`--window` datagrams, 2 % duplicates.

Usage (GPU box): python tools/rx_bench.py [--frames 32768] [--out file.json]
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
sys.path[:0] = [str(ROOT), str(ROOT / "oracle")]

from razor_amd.fec import FRAME_DTYPE, WIRE_REC_DTYPE, native  # noqa: E402

S, K, DSTRIDE, STRIDE = 1200, 10, 1280, 1200


def stream(lib, F, loss, window, seed=1):
    rng = np.random.default_rng(seed)
    blob = rng.integers(0, 256, F * K * S, dtype=np.uint8)
    frames = np.zeros(F, FRAME_DTYPE)
    frames["data"] = blob.ctypes.data + np.arange(F, dtype=np.uint64) * (K * S)
    frames["size"] = K * S
    frames["ftype"] = np.arange(F) % 60 == 0
    frames["payload_type"] = 96
    frames["protect_fraction"] = 80
    frames["now_ms"] = 1_700_000_000_000 + np.arange(F) * 33
    st = lib.sender_init()
    segs, groups, sdg, sdl, fdg, fdl, _ = lib.send_frames(st, frames, 0x5EED, DSTRIDE, max_segs=F * K + 64,
                                                          max_groups=F + 8, max_parities=F * 8 + 64)
    # send order: a group's parities after the segment that closes it
    ns, nf = len(segs), len(fdl)
    pos_seg = np.arange(ns, dtype=np.float64)
    pos_fec = np.empty(nf)
    p = 0
    for g in groups:
        nl = int(g["n_lines"])
        last = int(g["first_seg"]) + int(g["count"]) - 1
        pos_fec[p:p + nl] = last + (np.arange(nl) + 1) / (nl + 1)
        p += nl
    kind = np.concatenate([np.zeros(ns, np.int8), np.ones(nf, np.int8)])
    idx = np.concatenate([np.arange(ns), np.arange(nf)])
    pos = np.concatenate([pos_seg, pos_fec])
    keep = rng.random(len(pos)) >= loss
    kind, idx, pos = kind[keep], idx[keep], pos[keep]
    dup = rng.random(len(pos)) < 0.02
    kind = np.concatenate([kind, kind[dup]])
    idx = np.concatenate([idx, idx[dup]])
    key = np.concatenate([pos + rng.integers(0, window, len(pos)), pos[dup] + rng.integers(window, 3 * window, dup.sum())])
    o = np.argsort(key, kind="stable")
    kind, idx = kind[o], idx[o]
    n = len(kind)
    dgram = np.empty((n, DSTRIDE), np.uint8)
    dlen = np.empty(n, np.uint16)
    s_m, f_m = kind == 0, kind == 1
    dgram[s_m], dlen[s_m] = sdg[idx[s_m]], sdl[idx[s_m]]
    dgram[f_m], dlen[f_m] = fdg[idx[f_m]], fdl[idx[f_m]]
    return dgram, dlen, ns, nf


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=32768)
    ap.add_argument("--loss", type=float, default=0.05)
    ap.add_argument("--window", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    lib = native(1200)
    dgram, dlen, ns, nf = stream(lib, args.frames, args.loss, args.window)
    n = len(dlen)
    d_dg = torch.from_numpy(dgram.reshape(-1)).cuda()
    d_dl = torch.from_numpy(dlen.view(np.uint8)).cuda()
    recs = torch.empty(n * WIRE_REC_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    pay = torch.empty(n * STRIDE, dtype=torch.uint8, device="cuda")
    best = None
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lib.wire_parse(n, DSTRIDE, d_dg.data_ptr(), d_dl.data_ptr(), STRIDE, S, recs.data_ptr(), pay.data_ptr())
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        out, outp, mts, rep = lib.rx_recover(n, recs.data_ptr(), pay.data_ptr(), STRIDE, S, 0, 1 << 20)
        t2 = time.perf_counter()
        if best is None or t2 - t0 < best[0]:
            best = (t2 - t0, t1 - t0, t2 - t1, {f: getattr(rep, f) for f, _ in rep._fields_}, out, outp, mts)
    wall, t_parse, t_rx, rep, out, outp, mts = best
    res = {"frames": args.frames, "segments_sent": ns, "parities_sent": nf, "arrivals": n, "loss": args.loss,
           "window": args.window, "recovered": len(out), "max_ts": mts, "parse_s": t_parse, "rx_s": t_rx,
           "wall_s": wall, "rx_report": rep, "arrivals_per_s": n / wall, "rx_arrivals_per_s": n / t_rx,
           "arrival_GBps": float(dlen.astype(np.int64).sum()) / wall / 1e9}
    if not args.no_verify:
        from pyoracle import Oracle
        o = Oracle(1200)
        h_recs = recs.cpu().numpy().view(WIRE_REC_DTYPE)
        h_pay = pay.cpu().numpy().reshape(-1, STRIDE)
        t0 = time.perf_counter()
        eo, eop, emts, edrop = o.rx_recover(h_recs, h_pay, S, max_out=1 << 20)
        t_or = time.perf_counter() - t0
        i = np.argsort(eo["hdr"]["seq"], kind="stable")
        ok = (len(eo) == len(out) and np.array_equal(eo["hdr"][i], out["hdr"]) and
              np.array_equal(eop[i], outp) and emts == mts and edrop == rep["n_fec_dropped"])
        res.update({"verified": bool(ok), "oracle_s": t_or, "oracle_arrivals_per_s": n / t_or, "oracle_cores": 1})
    print(json.dumps(res, indent=1))
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1))
    if not res.get("verified", True):
        raise SystemExit("rx verification failed")


if __name__ == "__main__":
    main()
