"""Device-resident wire-codec throughput on the bench workload (BASELINE.json
config 3 shape: 65,536 groups, k = 10, r = 3, 1,200-byte payloads):

  frame_fec  196,608 SIM_FEC datagrams (1,249 B each) from the parity slots
  frame_seg  655,360 SIM_SEG datagrams (1,232 B each) from the source slots
  parse      all 851,968 datagrams back into records + payload slots

Each kernel is timed with HIP events on its own stream; results are checked
(parse(frame(x)) == x on every datagram; a sample against the oracle's bytes).

Algorithmic bytes per datagram:
  frame_fec  read L + 46 (payload, meta 20, stamp 24, size 2), write L + 49 + 2 (datagram, length)
  frame_seg  read L + 32 (payload, header 20, stamp 12),        write L + 36 + 2
  parse      read len + 2,                                     write 64 + stride (record, zero-tailed slot)

Usage: python tools/wire_bench.py [--groups 65536] [--reps 20] [--out file.json]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "oracle")]

from razor_amd.fec import FEC_STAMP_DTYPE, SEG_STAMP_DTYPE, HDR_DTYPE, Native, native  # noqa: E402

HBM_PEAK = 8000.0


def timed(fn, reps, stream, lib=None):
    """Median / mean kernel time: the kernel's own start / stop (rfec_timing_events, as bench.py)
    when the library has it, else stream events around each call."""
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    own = lib is not None and hasattr(lib.lib, "rfec_timing_events")
    if own:
        for a, b in ev:  # torch creates an event at its first record
            a.record(stream)
            b.record(stream)
        torch.cuda.synchronize()
    for a, b in ev:
        if own:
            lib.timing_events(a.cuda_event, b.cuda_event)
            fn()
        else:
            a.record(stream)
            fn()
            b.record(stream)
    torch.cuda.synchronize()
    t = np.array([a.elapsed_time(b) * 1e-3 for a, b in ev])
    return float(np.median(t)), float(t.mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--lib", default="", help="another build of the library (A/B)")
    ap.add_argument("--dstride", type=int, default=0, help="datagram slot width for both kinds (e.g. 1504: 1500-B receive slots, 32-byte lanes)")
    ap.add_argument("--stride", type=int, default=0, help="payload slot stride (framing input, parse output; default 1216)")
    ap.add_argument("--out", default="")
    ap.add_argument("--tuning", type=int, default=0, help="rfec_set_tuning bits")
    ap.add_argument("--only", default="", help="comma list of kernels to time (frame_fec,frame_seg,parse_fec,parse_seg)")
    args = ap.parse_args()
    G, k, n, S = args.groups, 10, 3, 1200
    P = args.stride or 1216  # payload slot stride: the engine's 16-B-aligned FEC slots
    lib = Native(1200, args.lib) if args.lib else native(1200)
    lib.set_tuning(args.tuning)
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    sp = st.cuda_stream
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    NF, NS = G * n, G * k
    parity = torch.randint(0, 256, (NF, P), dtype=torch.uint8, device=dev, generator=gen)
    shards = torch.randint(0, 256, (NS, P), dtype=torch.uint8, device=dev, generator=gen)
    rng = np.random.default_rng(3)
    meta = np.zeros(NF, HDR_DTYPE)
    meta["seq"] = rng.integers(0, 2**31, NF)
    meta["size"] = S
    fstamp = np.zeros(NF, FEC_STAMP_DTYPE)
    fstamp["uid"] = 77
    fstamp["fec_id"] = np.arange(NF) // n + 1
    fstamp["index"] = np.arange(NF) % n
    fstamp["row"], fstamp["col"], fstamp["count"] = 3, 4, k
    fstamp["transport_seq"] = np.arange(NF)
    hdr = np.zeros(NS, HDR_DTYPE)
    hdr["seq"] = 1 + np.arange(NS)  # contiguous ids (sim_sender.c:338): widths vary across 65535
    hdr["fid"] = 1 + np.arange(NS) // k
    hdr["index"] = np.arange(NS) % k
    hdr["total"] = k
    hdr["size"] = S
    sstamp = np.zeros(NS, SEG_STAMP_DTYPE)
    sstamp["uid"] = 77
    sstamp["fec_id"] = np.arange(NS) // k + 1
    sstamp["transport_seq"] = np.arange(NS)
    to = lambda a: torch.from_numpy(a.view(np.uint8).reshape(-1).copy()).to(dev)  # noqa: E731
    d_meta, d_fs, d_fst, d_hdr, d_sst = to(meta), to(np.full(NF, S, np.uint16)), to(fstamp), to(hdr), to(sstamp)
    # datagram slots: 1,280 B (10 x 128: whole-line stores; the minimal 16-B multiples, 1,264 / 1,248, leave
    # slot edges inside 128-B lines and frame at 0.52-0.53 of peak against 0.60-0.61)
    DF, DS = (args.dstride, args.dstride) if args.dstride else (1280, 1280)
    dg_f = torch.empty((NF, DF), dtype=torch.uint8, device=dev)
    dl_f = torch.empty((NF,), dtype=torch.int16, device=dev)
    dg_s = torch.empty((NS, DS), dtype=torch.uint8, device=dev)
    dl_s = torch.empty((NS,), dtype=torch.int16, device=dev)
    rec_f = torch.empty((NF, 64), dtype=torch.uint8, device=dev)
    pay_f = torch.empty((NF, P), dtype=torch.uint8, device=dev)
    rec_s = torch.empty((NS, 64), dtype=torch.uint8, device=dev)
    pay_s = torch.empty((NS, P), dtype=torch.uint8, device=dev)

    def frame_fec():
        lib.wire_frame_fec(NF, P, S, parity.data_ptr(), d_meta.data_ptr(), d_fs.data_ptr(), None, d_fst.data_ptr(),
                           DF, dg_f.data_ptr(), dl_f.data_ptr(), sp)

    def frame_seg():
        lib.wire_frame_seg(NS, P, S, shards.data_ptr(), d_hdr.data_ptr(), d_sst.data_ptr(), DS, dg_s.data_ptr(),
                           dl_s.data_ptr(), sp)

    def parse_f():
        lib.wire_parse(NF, DF, dg_f.data_ptr(), dl_f.data_ptr(), P, S, rec_f.data_ptr(), pay_f.data_ptr(), sp)

    def parse_s():
        lib.wire_parse(NS, DS, dg_s.data_ptr(), dl_s.data_ptr(), P, S, rec_s.data_ptr(), pay_s.data_ptr(), sp)

    with torch.cuda.stream(st):
        for f in (frame_fec, frame_seg, parse_f, parse_s):
            f()
        torch.cuda.synchronize()
        res = {}
        lenf = S + 49
        lens = int(np.mean(np.where(hdr["seq"] > 65535, 2, 0) + 26 + 4)) + S
        alg = {"frame_fec": NF * ((S + 46) + (lenf + 2)),
               "frame_seg": NS * ((S + 32) + (lens + 2)),
               "parse_fec": NF * ((lenf + 2) + (64 + S)),
               "parse_seg": NS * ((lens + 2) + (64 + S))}
        for name, f in (("frame_fec", frame_fec), ("frame_seg", frame_seg), ("parse_fec", parse_f),
                        ("parse_seg", parse_s)):
            if args.only and name not in args.only.split(","):
                continue
            med, mean = timed(f, args.reps, st, lib)
            res[name] = {"median_us": round(med * 1e6, 2), "mean_us": round(mean * 1e6, 2),
                         "algorithmic_bytes": alg[name], "GBps": round(alg[name] / med / 1e9, 1),
                         "frac_of_hbm_peak": round(alg[name] / med / 1e9 / HBM_PEAK, 4)}
    # verification: parse(frame(x)) == x everywhere
    ok = bool(torch.equal(pay_f[:, :S], parity[:, :S]) and torch.equal(pay_s[:, :S], shards[:, :S]))
    ok = ok and not bool(pay_f[:, S:].any()) and not bool(pay_s[:, S:].any())  # slot tails zeroed
    rf = rec_f.cpu().numpy()
    rs = rec_s.cpu().numpy()
    ok = ok and bool((rf[:, 0] == 0).all() and (rs[:, 0] == 0).all())
    ok = ok and bool((dl_f.cpu().numpy().view(np.uint16) == lenf).all())
    # sample against the oracle's datagram bytes
    from pyoracle import Oracle
    o = Oracle(1200)
    idx = np.r_[0:64, NF // 2:NF // 2 + 64, NF - 64:NF]
    og, ol = o.frame_fec_batch(np.ascontiguousarray(parity[idx, :S].cpu().numpy()), meta[idx], np.full(len(idx), S, np.uint16), None,
                               fstamp[idx], S, DF)
    ok = ok and bool(np.array_equal(dg_f[idx].cpu().numpy(), og))
    idx = np.r_[0:64, 65530:65600, NS - 64:NS]
    og, ol = o.frame_seg_batch(np.ascontiguousarray(shards[idx, :S].cpu().numpy()), hdr[idx], sstamp[idx], S, DS)
    ok = ok and bool(np.array_equal(dg_s[idx].cpu().numpy(), og))
    out = {"groups": G, "k": k, "r": n, "payload": S, "payload_stride": P, "fec_datagrams": NF, "seg_datagrams": NS,
           "dstride": {"fec": DF, "seg": DS}, "kernels": res, "verified": ok,
           "timing": ("the kernel's own start / stop (rfec_timing_events)" if hasattr(lib.lib, "rfec_timing_events")
                      else "stream events around each call")}
    print(json.dumps(out, indent=1))
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1))
    if not ok:
        raise SystemExit("wire verification failed")


if __name__ == "__main__":
    main()
