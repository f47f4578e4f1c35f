"""Sender end to end: video frames in host memory -> SIM_SEG + SIM_FEC
datagrams in host memory (rfec_host_send_frames: plan, staging into pinned SoA
slots, H2D, encode, framing + CRC32, D2H), per stage.

Workload: F frames of 10 x 1,200 bytes (one k = 10 group per frame at
protect_fraction 80 -> 3 row + 4 column parities... the rows-only bench plan is
not what the sender emits: sim_sender_fec uses the full plan), in calls of
`--chunk` frames.  Verified: every SIM_FEC datagram of a sample of groups is
re-derived by the oracle (encode + frame) and compared byte for byte.

Usage (GPU box): python tools/send_bench.py [--frames 65536] [--chunk 8192] [--out file.json]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "oracle")]

from razor_amd.fec import FRAME_DTYPE, native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=65536)
    ap.add_argument("--chunk", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--pageable", action="store_true", help="datagrams into fresh pageable numpy arrays per call")
    ap.add_argument("--frames-mem", default="pinned", choices=("pinned", "pageable"),
                    help="frame bytes in an rfec_pinned_alloc block (the device gathers the segments itself) or not")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    lib = native(1200)
    S, k = 1200, 10
    F, CH = args.frames, args.chunk
    rng = np.random.default_rng(1)
    blob = rng.integers(0, 256, F * k * S, dtype=np.uint8)
    frames = np.zeros(F, FRAME_DTYPE)
    frames["data"] = blob.ctypes.data + np.arange(F, dtype=np.uint64) * (k * S)
    frames["size"] = k * S
    frames["ftype"] = (np.arange(F) % 60 == 0)
    frames["payload_type"] = 96
    frames["protect_fraction"] = 80
    frames["now_ms"] = 1_700_000_000_000 + np.arange(F) * 33
    keep_frames = None
    if args.frames_mem == "pinned":  # what a capture / encoder hands over: frames in pinned, device-mapped memory
        pb, keep_frames = lib.pinned_array(blob.shape, np.uint8)
        pb[...] = blob
        frames["data"] = pb.ctypes.data + np.arange(F, dtype=np.uint64) * (k * S)
        blob = pb
    dstride = 1280  # 10 x 128 B: whole-line datagram stores
    bufs, keep_alive = None, []
    if not args.pageable:  # datagram slots in pinned memory, reused across calls (what a sender hands to sendmmsg)
        ms, mp = CH * k + 128, CH * 8 + 64
        sdg, a = lib.pinned_array((ms, dstride), np.uint8)
        sdl, b = lib.pinned_array((ms,), np.uint16)
        fdg, c = lib.pinned_array((mp, dstride), np.uint8)
        fdl, d = lib.pinned_array((mp,), np.uint16)
        bufs, keep_alive = (sdg, sdl, fdg, fdl), [a, b, c, d]
    best = None
    for rep in range(args.reps):
        st = lib.sender_init()
        tot = {"plan_us": 0.0, "stage_us": 0.0, "h2d_us": 0.0, "kernel_us": 0.0, "d2h_us": 0.0, "total_us": 0.0}
        nseg = npar = 0
        keep = None
        t0 = time.perf_counter()
        for c0 in range(0, F, CH):
            segs, groups, sdg, sdl, fdg, fdl, r = lib.send_frames(st, frames[c0:c0 + CH], 77, dstride,
                                                                  max_segs=CH * k + 128, max_groups=CH + 8,
                                                                  max_parities=CH * 8 + 64, bufs=bufs)
            for key in tot:
                tot[key] += getattr(r, key)
            nseg += r.n_segs
            npar += r.n_parities
            zc = r.zero_copy
            if c0 == 0:
                keep = (segs.copy(), groups.copy(), fdg[:64].copy(), fdl[:64].copy(), sdg[:256].copy(), sdl[:256].copy())
        wall = time.perf_counter() - t0
        if best is None or wall < best[0]:
            best = (wall, tot, nseg, npar, keep)
    wall, tot, nseg, npar, keep = best
    # verify: the first groups' SIM_FEC datagrams against the oracle
    from pyoracle import FEC_STAMP, HDR_DTYPE, Oracle
    o = Oracle(1200)
    segs, groups, fdg0, fdl0, sdg0, sdl0 = keep
    ok = True
    # the first SIM_SEG datagrams: parsed back, payload = the frame bytes
    recs, pay = o.parse_batch(sdg0, sdl0, 1216, S)
    for i in range(len(sdl0)):
        off = int(frames["data"][segs["frame"][i]]) - blob.ctypes.data + int(segs["offset"][i])
        ds = int(segs["data_size"][i])
        ok = ok and int(recs["status"][i]) == 0 and int(recs["hdr"]["seq"][i]) == int(segs["packet_id"][i]) and \
            bool(np.array_equal(pay[i, :ds], blob[off:off + ds]))
    p = 0
    for g in groups[:8]:
        plan = o.plan_from_fraction(int(g["count"]), int(g["protect_fraction"]), 3)
        sel = segs[int(g["first_seg"]):int(g["first_seg"]) + int(g["count"])]
        sh = np.zeros((1, len(sel), S), np.uint8)
        hd = np.zeros((1, len(sel)), HDR_DTYPE)
        for i, s in enumerate(sel):
            off = int(frames["data"][s["frame"]]) - blob.ctypes.data + int(s["offset"])
            ds = int(s["data_size"])
            sh[0, i, :ds] = blob[off:off + ds]
            hd[0, i] = (s["packet_id"], s["fid"], s["timestamp"], s["index"], s["total"], s["ftype"],
                        s["payload_type"], s["data_size"])
        par, meta, fs, stt = o.encode_batch(plan, sh, hd, S)
        n = plan.n_lines
        stamps = np.zeros(n, FEC_STAMP)
        stamps["uid"], stamps["base_id"], stamps["fec_id"], stamps["count"] = 77, g["base_id"], g["fec_id"], g["count"]
        stamps["send_ts"] = g["fec_ts"]
        stamps["row"], stamps["col"] = plan.row, plan.col
        stamps["index"] = [plan.line[l].index for l in range(n)]
        stamps["transport_seq"] = fdg0[p:p + n, 17].astype(np.uint16) << 8 | fdg0[p:p + n, 18]  # taken from the wire
        od, ol = o.frame_fec_batch(par.reshape(n, S), meta.reshape(n), fs.reshape(n), None, stamps, S, dstride)
        ok = ok and bool(np.array_equal(ol, fdl0[p:p + n]) and np.array_equal(od, fdg0[p:p + n]))
        p += n
    frame_bytes = F * k * S
    dgram_bytes = nseg * (S + 32) + npar * (S + 49)
    res = {"frames": F, "chunk": CH, "output_memory": "pageable" if args.pageable else "pinned",
           "frames_memory": args.frames_mem, "zero_copy": {"in": bool(zc & 1), "out": bool(zc & 2)},
           "segments": nseg, "parities": npar, "frame_bytes": frame_bytes,
           "pcie_GBps": (frame_bytes + dgram_bytes) / wall / 1e9,
           "datagram_bytes": dgram_bytes, "wall_s": wall, "stage_us": tot, "frames_GiBps": frame_bytes / wall / 2**30,
           "datagrams_per_s": (nseg + npar) / wall, "gpu_only_GiBps": frame_bytes / (tot["kernel_us"] * 1e-6) / 2**30,
           "verified_sample": ok}
    print(json.dumps(res, indent=1))
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1))
    if not ok:
        raise SystemExit("send verification failed")


if __name__ == "__main__":
    main()
