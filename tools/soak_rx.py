"""Soak of the receiver session path (rfec_rx_session_push_datagrams[_async]) against the oracle's
event-by-event receiver (oracle/rfec_oracle.c rx_recover: sim_fec.c / flex_fec_receiver.c semantics,
pinned by tests/golden/rx.json).  Each round draws a product-sender stream (frame sizes over k choices,
protect fractions), a network (loss, reordering window, duplicates, late parities), datagram slots
pageable or pinned, the push (sync / pipelined), the control-plane shards (1-8), the batch size, and
evictions after every batch or none; the delivered segments (headers, fec_id, payload rows), max_ts and
the dropped-parity count must equal the oracle's over the same arrivals with the same evictions (its
own parse of the same datagrams).

Usage (GPU box): python tools/soak_rx.py [--seconds 180] [--seed 1] [--out f.json]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests")]

import pyoracle as po  # noqa: E402
from razor_amd.fec import native  # noqa: E402

DSTRIDE, STRIDE, CAP = 1280, 1024, 1000


def stream(lib, rng):
    frames_n = int(rng.integers(200, 2500))
    kc = rng.choice([1, 3, 6, 10, 16, 24], size=int(rng.integers(1, 4)), replace=False)
    pfc = rng.choice([20, 50, 80, 100], size=int(rng.integers(1, 3)), replace=False)
    sizes = rng.choice(kc, frames_n) * 1000 - rng.integers(0, 900, frames_n)
    blob = rng.integers(0, 256, int(sizes.sum()), dtype=np.uint8)
    frames = np.zeros(frames_n, po.FRAME)
    frames["data"] = blob.ctypes.data + np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    frames["size"] = sizes
    frames["payload_type"] = 96
    frames["ftype"] = np.arange(frames_n) % 50 == 0
    frames["protect_fraction"] = rng.choice(pfc, frames_n)
    frames["now_ms"] = 1_700_000_000_000 + np.arange(frames_n) * 33
    st = lib.sender_init()
    segs, groups, sdg, sdl, fdg, fdl, _ = lib.send_frames(st, frames, int(rng.integers(1, 1 << 30)), DSTRIDE,
                                                          max_segs=frames_n * 26 + 64, max_groups=frames_n + 64,
                                                          max_parities=frames_n * 40 + 64)
    # send order: a group's parities right after the segment that closes it
    order_k, order_i = [], []
    p = 0
    closes = {}
    for g in groups:
        nl = int(g["n_lines"])
        if int(g["first_seg"]) >= 0:
            closes[int(g["first_seg"]) + int(g["count"]) - 1] = (p, nl)
        p += nl
    for i in range(len(segs)):
        order_k.append(0)
        order_i.append(i)
        if i in closes:
            p0, nl = closes[i]
            order_k += [1] * nl
            order_i += list(range(p0, p0 + nl))
    kind, idx = np.array(order_k, np.int8), np.array(order_i, np.int64)
    net = dict(loss=float(rng.uniform(0, 0.35)), window=int(rng.integers(1, 200)), dup=float(rng.uniform(0, 0.2)),
               late=float(rng.uniform(0, 0.25)) if rng.random() < 0.3 else 0.0, late_by=int(rng.integers(500, 5000)))
    pos = np.arange(len(kind), dtype=np.int64)
    keep = rng.random(len(kind)) >= net["loss"]
    kind, idx, pos = kind[keep], idx[keep], pos[keep]
    key = pos + rng.integers(0, net["window"], len(pos))
    key += ((kind == 1) & (rng.random(len(pos)) < net["late"])) * net["late_by"]
    dup = rng.random(len(pos)) < net["dup"]
    kind = np.concatenate([kind, kind[dup]])
    idx = np.concatenate([idx, idx[dup]])
    key = np.concatenate([key, key[dup] + rng.integers(1, 3 * net["window"] + 1, int(dup.sum()))])
    pos = np.concatenate([pos, pos[dup]])
    o = np.lexsort((pos, key))
    kind, idx = kind[o], idx[o]
    n = len(kind)
    dgram = np.zeros((n, DSTRIDE), np.uint8)
    dlen = np.zeros(n, np.uint16)
    s_m, f_m = kind == 0, kind == 1
    dgram[s_m], dlen[s_m] = sdg[idx[s_m]], sdl[idx[s_m]]
    dgram[f_m], dlen[f_m] = fdg[idx[f_m]], fdl[idx[f_m]]
    return dgram, dlen, dict(frames=frames_n, k=[int(x) for x in kc], pf=[int(x) for x in pfc], **net)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=180.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    lib = native(CAP)
    o = po.Oracle(CAP)
    rng = np.random.default_rng(args.seed)
    t_end = time.time() + args.seconds
    tot = dict(streams=0, datagrams=0, delivered=0, batches=0, mismatches=0, by_mode={})
    fails = []
    while time.time() < t_end:
        dgram, dlen, cfg = stream(lib, rng)
        n = len(dlen)
        mode = str(rng.choice(["sync", "async"]))
        threads = int(rng.integers(1, 9))
        batch = int(rng.choice([int(rng.integers(1, 300)), int(rng.integers(300, 6000))]))
        evict = bool(rng.random() < 0.5)
        pinned = bool(rng.random() < 0.6)
        if pinned:
            dg, k1 = lib.pinned_array((n, DSTRIDE), np.uint8)
            dl, k2 = lib.pinned_array((n,), np.uint16)
            dg[...] = dgram
            dl[...] = dlen
        else:
            dg, dl = dgram, dlen
        erecs, epay = o.parse_batch(dgram, dlen, STRIDE, CAP)
        eo, eop, emts, edrop = o.rx_recover(erecs, epay, CAP, max_out=1 << 20, evict_every=batch if evict else 0)
        sess = lib.rx_session(STRIDE, CAP, threads)
        got, gotp, dropped = [], [], 0
        max_out = 4 * batch + 4096
        for a in range(0, n, batch):
            m = min(batch, n - a)
            push = sess.push_datagrams if mode == "sync" else sess.push_datagrams_async
            out, outp, rep, _ = push(m, DSTRIDE, dg[a:].ctypes.data, dl[a:].ctypes.data, max_out=max_out,
                                     pinned_out=pinned)
            got.append(out)
            gotp.append(outp)
            dropped += rep.n_fec_dropped
            tot["batches"] += 1
            # the heartbeat's eviction once a full batch is ingested (the pipelined push ingests the previous one)
            if evict and (mode == "sync" and m == batch or mode == "async" and a > 0):
                sess.evict()
        if mode == "async":
            out, outp, rep, _ = sess.push_datagrams_async(0, DSTRIDE, 0, 0, max_out=max_out, pinned_out=pinned)
            got.append(out)
            gotp.append(outp)
            dropped += rep.n_fec_dropped
        info = sess.info()
        sess.close()
        out, outp = np.concatenate(got), np.concatenate(gotp)
        i, j = np.argsort(out["hdr"]["seq"], kind="stable"), np.argsort(eo["hdr"]["seq"], kind="stable")
        ok = (len(out) == len(eo) and np.array_equal(out["hdr"][i], eo["hdr"][j]) and
              np.array_equal(out["fec_id"][i], eo["fec_id"][j]) and np.array_equal(outp[i][:, :CAP], eop[j][:, :CAP]) and
              info["max_ts"] == emts and dropped == edrop)
        key = f"{mode}/T{threads}/{'evict' if evict else 'noevict'}"
        tot["by_mode"][key] = tot["by_mode"].get(key, 0) + 1
        tot["streams"] += 1
        tot["datagrams"] += n
        tot["delivered"] += len(out)
        if not ok:
            tot["mismatches"] += 1
            fails.append(dict(cfg, mode=mode, threads=threads, batch=batch, evict=evict, pinned=pinned,
                              got=len(out), want=len(eo), max_ts=[info["max_ts"], emts], dropped=[dropped, edrop]))
            print("MISMATCH", fails[-1], flush=True)
        if tot["streams"] % 10 == 0:
            print(json.dumps({k: v for k, v in tot.items() if k != "by_mode"}), flush=True)
    res = dict(tot, seconds=args.seconds, seed=args.seed, failures=fails[:20])
    print(json.dumps(res, indent=1))
    if args.out:
        Path(args.out).parent.mkdir(parents=True, exist_ok=True)
        Path(args.out).write_text(json.dumps(res, indent=1))
    if tot["mismatches"]:
        raise SystemExit("session soak: mismatches")


if __name__ == "__main__":
    main()
