"""Receive path from the socket: a lossy, reordered SIM_SEG + SIM_FEC datagram
stream of the product sender goes over loopback UDP (rfec_udp_send_batch /
rfec_udp_recv_batch, sendmmsg / recvmmsg) into a pinned slot block.  Two
receivers:
  * streaming: every recvmmsg batch goes straight into a receiver session
    (rfec_rx_session_push_datagrams: H2D, rfec_wire_parse, ingestion with
    the state kept across batches) while the sender is still sending;
  * block: the whole received block through rfec_host_recv_datagrams once.
Reports the socket rates, loopback drops and the ingestion stages; verifies
the parse records and both receivers' recovered segments against the oracle
on exactly the datagrams that arrived.

Usage (GPU box): python tools/udp_bench.py [--frames 16384] [--out file.json]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tools")]

from razor_amd.fec import RFEC_UDP_SERVER, WIRE_REC_DTYPE, native, rfec_udp_stats  # noqa: E402
from rx_bench import DSTRIDE, S, STRIDE, stream  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16384)
    ap.add_argument("--loss", type=float, default=0.05)
    ap.add_argument("--window", type=int, default=32)
    ap.add_argument("--chunk", type=int, default=1024, help="datagrams per send call")
    ap.add_argument("--sockbuf", type=int, default=32 << 20)
    ap.add_argument("--batch", type=int, default=4096, help="max datagrams per recvmmsg batch / session push")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    lib = native(1200)
    dgram, dlen, ns, nf = stream(lib, args.frames, args.loss, args.window)
    n = len(dlen)
    rx, rx_addr = lib.udp_open("127.0.0.1", 0, RFEC_UDP_SERVER, args.sockbuf)
    tx, _ = lib.udp_open("127.0.0.1", 0, RFEC_UDP_SERVER, args.sockbuf)
    pin = lib.lib.rfec_pinned_alloc(n * DSTRIDE + n * 2 + 256)
    if not pin:
        raise SystemExit("pinned alloc failed: " + lib.last_error())
    slots = np.ctypeslib.as_array((C.c_uint8 * (n * DSTRIDE)).from_address(pin)).reshape(n, DSTRIDE)
    lens = np.ctypeslib.as_array((C.c_uint16 * n).from_address(pin + n * DSTRIDE))
    st_tx, st_rx = rfec_udp_stats(), rfec_udp_stats()
    times = {}

    def send():
        t0 = time.perf_counter()
        off = 0
        while off < n:
            m = min(args.chunk, n - off)
            off += lib.udp_send(tx, rx_addr, m, DSTRIDE, dgram[off:].ctypes.data, dlen[off:].ctypes.data, 100, st_tx)[1]
        times["send_s"] = time.perf_counter() - t0

    th = threading.Thread(target=send)
    sess = lib.rx_session(STRIDE, S)
    s_out, s_pay, s_recs, s_push = [], [], [], 0.0
    t0 = time.perf_counter()
    th.start()
    got, idle, t_last, batches = 0, 0, t0, 0
    while got < n and idle < 10:
        k = lib.udp_recv(rx, min(args.batch, n - got), DSTRIDE, slots[got:].ctypes.data, lens[got:].ctypes.data, 20,
                         st_rx)
        if k:
            tp = time.perf_counter()
            o, op, _, r = sess.push_datagrams(k, DSTRIDE, slots[got:].ctypes.data, lens[got:].ctypes.data,
                                              max_out=k + 64, want_recs=True)
            s_push += time.perf_counter() - tp
            s_out.append(o)
            s_pay.append(op)
            s_recs.append(r)
            got += k
            batches += 1
            idle, t_last = 0, time.perf_counter()
        else:
            idle += 1
    th.join()
    recv_s = t_last - t0
    s_out, s_pay, s_recs = np.concatenate(s_out), np.concatenate(s_pay), np.concatenate(s_recs)
    sess_info = sess.info()
    sess.close()
    t1 = time.perf_counter()
    out, outp, mts, rep, recs = lib.host_recv_datagrams(got, DSTRIDE, slots.ctypes.data, lens.ctypes.data, STRIDE, S,
                                                        0, 1 << 20, want_recs=True)
    ingest_s = time.perf_counter() - t1
    rbytes = int(lens[:got].astype(np.int64).sum())
    res = {"frames": args.frames, "datagrams_sent": n, "datagrams_received": got, "loopback_dropped": n - got,
           "net_loss": args.loss, "window": args.window, "send_s": times["send_s"], "recv_s": recv_s,
           "send_datagrams_per_s": n / times["send_s"], "recv_datagrams_per_s": got / recv_s,
           "recv_GBps": rbytes / recv_s / 1e9, "tx_stats": st_tx.as_dict(), "rx_stats": st_rx.as_dict(),
           "streaming": {"batches": batches, "session_push_s": s_push,
                         "push_datagrams_per_s": got / s_push, "recovered": len(s_out),
                         "loop_datagrams_per_s": got / recv_s, "session_info": sess_info},
           "ingest_s": ingest_s, "ingest_datagrams_per_s": got / ingest_s, "recovered": len(out),
           "rx_report": {f: getattr(rep, f) for f, _ in rep._fields_}, "max_ts": mts}
    if not args.no_verify:
        from pyoracle import Oracle
        o = Oracle(1200)
        h_dg, h_dl = slots[:got].copy(), lens[:got].copy()
        erecs, epay = o.parse_batch(h_dg, h_dl, STRIDE, S)
        rec_ok = np.array_equal(recs.view(np.uint8).reshape(-1), np.asarray(erecs).view(np.uint8).reshape(-1))
        eo, eop, emts, edrop = o.rx_recover(recs.view(WIRE_REC_DTYPE), epay, S, max_out=1 << 20)
        i = np.argsort(eo["hdr"]["seq"], kind="stable")
        ok = (rec_ok and len(eo) == len(out) and np.array_equal(eo["hdr"][i], out["hdr"]) and
              np.array_equal(eop[i], outp) and emts == mts and edrop == rep.n_fec_dropped)
        k = np.argsort(s_out["hdr"]["seq"], kind="stable")
        s_ok = (np.array_equal(s_recs.view(np.uint8).reshape(-1), np.asarray(erecs).view(np.uint8).reshape(-1)) and
                len(s_out) == len(eo) and np.array_equal(s_out["hdr"][k], eo["hdr"][i]) and
                np.array_equal(s_pay[k], eop[i]) and sess_info["max_ts"] == emts)
        res["verified"] = bool(ok and s_ok)
        res["streaming"]["verified"] = bool(s_ok)
    lib.lib.rfec_pinned_free(pin)
    lib.udp_close(rx)
    lib.udp_close(tx)
    print(json.dumps(res, indent=1))
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1))
    if not res.get("verified", True):
        raise SystemExit("udp verification failed")


if __name__ == "__main__":
    main()
