"""The receive path from socket buffers: a lossy, reordered c3 datagram stream
(k = 10 x 1,200 B, the sender's 3 x 4 plan, 5 % loss, reordering within 32
datagrams, 2 % duplicates; tools/rx_bench.stream) in PINNED datagram slots --
what rfec_udp_recv_batch fills -- pushed through a receiver session in
batches of `--batch` datagrams:

  async  rfec_rx_session_push_datagrams_async (the pipelined push: the parse of
         batch i runs on the device while the host ingests batch i-1)
  sync   rfec_rx_session_push_datagrams

Per mode: wall time, datagrams/s, datagram GB/s, and the library's own stage
split summed over the batches (host control plane, device, copies).  Every
delivered segment (header, fec_id, payload row) is checked against the
oracle's event-by-event receiver over the whole stream (the reference's
sim_fec.c / flex_fec_receiver.c semantics, pinned by tests/golden/rx.json).

Usage (GPU box): python tools/rx_session_bench.py [--frames 32768] [--batch 4096] [--out f.json]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tools")]

from razor_amd.fec import RX_SEG_DTYPE, WIRE_REC_DTYPE, native, rfec_rx_report  # noqa: E402
from rx_bench import DSTRIDE, S, STRIDE, stream  # noqa: E402

REP_FIELDS = ("host_us", "h2d_us", "kernel_us", "d2h_us", "total_us")
OUT = OUTP = None  # pinned outputs, one row per datagram at most (main)


def run(lib, mode, n, dg, dl, batch, max_out, threads, evict):
    """One pass of the whole stream through a fresh session (`threads`
    control-plane shards); returns the delivered (segments, rows) in delivery
    order, the wall seconds and the summed report."""
    sess = lib.rx_session(STRIDE, S, threads)
    # the recovered segments go to consecutive slices of one pinned output (what a receiver hands on):
    # nothing is copied inside the timed loop
    out, ko = OUT
    outp, kp = OUTP
    cap = len(out)
    pos = [0]
    nout, rep = C.c_uint32(), rfec_rx_report()
    fn = (lib.lib.rfec_rx_session_push_datagrams_async if mode == "async" else
          lib.lib.rfec_rx_session_push_datagrams)
    tot = dict.fromkeys(REP_FIELDS, 0.0)
    tot.update(n_recovered=0, n_groups=0, n_fec_dropped=0, n_unmodelled=0, calls=0)

    def call(a0, m):
        p_dg = dg.ctypes.data + a0 * DSTRIDE if m else None
        p_dl = dl.ctypes.data + a0 * 2 if m else None
        o = pos[0]
        lib._check(fn(sess.h, m, DSTRIDE, p_dg, p_dl, None, out.ctypes.data + o * out.itemsize,
                      outp.ctypes.data + o * STRIDE, min(max_out, cap - o), C.byref(nout), C.byref(rep)), fn.__name__)
        pos[0] = o + nout.value
        for f in REP_FIELDS:
            tot[f] += getattr(rep, f)
        for f in ("n_recovered", "n_groups", "n_fec_dropped", "n_unmodelled"):
            tot[f] += getattr(rep, f)
        tot["calls"] += 1

    ev = lib.lib.rfec_rx_session_evict
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a0 in range(0, n, batch):
        call(a0, min(batch, n - a0))
        # the heartbeat's sim_fec_evict once per ingested full batch (the async call ingests the previous one)
        if evict and (mode == "sync" and a0 + batch <= n or mode == "async" and a0 > 0):
            lib._check(ev(sess.h, None), "evict")
    if mode == "async":
        call(0, 0)  # flush the last pending batch
        if evict and n % batch == 0:
            lib._check(ev(sess.h, None), "evict")
    wall = time.perf_counter() - t0
    info = sess.info()
    sess.close()
    return out[:pos[0]].copy(), outp[:pos[0]].copy(), wall, tot, info


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=32768)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--loss", type=float, default=0.05)
    ap.add_argument("--window", type=int, default=32)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--modes", default="async,sync")
    ap.add_argument("--threads", default="1,8", help="control-plane shards to measure (rfec_rx_session_set_threads)")
    ap.add_argument("--evict", type=int, default=1, help="rfec_rx_session_evict after every ingested batch "
                    "(the heartbeat's sim_fec_evict, sim_receiver.c:881; the oracle evicts at the same points); 0: never")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    lib = native(1200)
    dgram, dlen, ns, nf = stream(lib, args.frames, args.loss, args.window)
    n = len(dlen)
    # the UDP batch slots: pinned, device-mapped (rfec_pinned_alloc), as rfec_udp_recv_batch fills them
    dg, k1 = lib.pinned_array((n, DSTRIDE), np.uint8)
    dl, k2 = lib.pinned_array((n,), np.uint16)
    dg[...] = dgram
    dl[...] = dlen
    gb = float(dlen.astype(np.int64).sum()) / 1e9
    global OUT, OUTP
    OUT = lib.pinned_array((n,), RX_SEG_DTYPE)
    OUTP = lib.pinned_array((n, STRIDE), np.uint8)
    # the oracle over the whole stream (the records from the product parse, checked bit-exact elsewhere)
    d_dg = torch.from_numpy(dgram.reshape(-1)).cuda()
    d_dl = torch.from_numpy(dlen.view(np.uint8)).cuda()
    recs = torch.empty(n * WIRE_REC_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    pay = torch.empty(n * STRIDE, dtype=torch.uint8, device="cuda")
    lib.wire_parse(n, DSTRIDE, d_dg.data_ptr(), d_dl.data_ptr(), STRIDE, S, recs.data_ptr(), pay.data_ptr())
    torch.cuda.synchronize()
    from pyoracle import Oracle

    o = Oracle(1200)
    t0 = time.perf_counter()
    eo, eop, emts, edrop = o.rx_recover(recs.cpu().numpy().view(WIRE_REC_DTYPE), pay.cpu().numpy().reshape(-1, STRIDE),
                                        S, max_out=1 << 20, evict_every=args.batch if args.evict else 0)
    t_or = time.perf_counter() - t0
    del d_dg, d_dl, recs, pay
    res = {"stream": {"frames": args.frames, "segments_sent": ns, "parities_sent": nf, "datagrams": n,
                      "datagram_GB": round(gb, 4), "loss": args.loss, "window": args.window, "duplicates": 0.02,
                      "k": 10, "payload": S, "plan": "3 x 4 (3 rows + 4 columns)", "dstride": DSTRIDE},
           "batch": args.batch, "evict_every_batch": bool(args.evict), "oracle": {"recovered": int(len(eo)), "s": round(t_or, 3),
                                           "datagrams_per_s": round(n / t_or), "cores": 1},
           "pid_cpus": len(os.sched_getaffinity(0))}
    ok_all = True
    for mode, threads in [(m, int(t)) for m in args.modes.split(",") for t in args.threads.split(",")]:
        best = None
        for _ in range(args.reps):
            r = run(lib, mode, n, dg, dl, args.batch, max(2 * args.batch, 8192), threads, args.evict)
            if best is None or r[2] < best[2]:
                best = r
        seg, row, wall, tot, info = best
        # delivery order: per call, ascending packet_id (the reference drains lowest id first, per arrival);
        # compare as sets keyed by packet_id against the oracle
        i = np.argsort(seg["hdr"]["seq"], kind="stable")
        j = np.argsort(eo["hdr"]["seq"], kind="stable")
        ok = (len(seg) == len(eo) and np.array_equal(seg["hdr"][i], eo["hdr"][j]) and
              np.array_equal(seg["fec_id"][i], eo["fec_id"][j]) and
              np.array_equal(row[i][:, :S], eop[j][:, :S]) and tot["n_fec_dropped"] == edrop)
        ok_all &= ok
        res[f"{mode}_T{threads}"] = {"threads": threads, "wall_s": round(wall, 4), "datagrams_per_s": round(n / wall), "datagram_GBps": round(gb / wall, 3),
                     "recovered": int(len(seg)), "verified_vs_oracle": bool(ok),
                     "stage_us_sum": {f: round(tot[f], 1) for f in REP_FIELDS},
                     "host_us_per_batch": round(tot["host_us"] / max(1, tot["calls"]), 2),
                     "calls": tot["calls"], "groups_peeled": tot["n_groups"], "unmodelled": tot["n_unmodelled"],
                     "session_after": {k: (round(v, 1) if isinstance(v, float) else v) for k, v in info.items()},
                     "host_split_us_per_batch": {k: round(v / max(1, tot["calls"]), 1) for k, v in info.items()
                                                 if k.endswith("_us")}}
        print(mode, threads, json.dumps(res[f"{mode}_T{threads}"]), flush=True)
    res["verified"] = ok_all
    print(json.dumps(res, indent=1))
    if args.out:
        Path(args.out).parent.mkdir(parents=True, exist_ok=True)
        Path(args.out).write_text(json.dumps(res, indent=1))
    if not ok_all:
        raise SystemExit("rx session verification failed")


if __name__ == "__main__":
    main()
