"""The bench step end to end, host memory in and out (GPU box): the c3 /
c3full workloads (65,536 groups of k = 10 x 1,200 B, the row layer or the
sender's full 3 x 4 plan) as razor's sender and receiver hold them --
sim_segment_t / sim_fec_t structs in host memory (AoS, payload at offset 34).

  encode  rfec_host_encode_groups: gather into pinned SoA -> H2D -> encode
          kernel -> D2H of the parities -> scatter into sim_fec_t
  decode  rfec_host_recover_groups: the received set (2 segments of every
          group lost, the bench's erasure pairs; every parity received)
          gathered -> H2D -> dense decode -> D2H of the recovered slots ->
          scatter into flex_fec_recover-style out_seg structs

Both chunked and double-buffered (copies, kernels and host threads overlap).
--mem pinned: the structs in rfec_pinned_alloc memory, so both directions
take the zero-copy path -- no host gather or scatter, the device reads the
sim_segment_t and writes the sim_fec_t / out_seg structs over PCIe itself
(rfec_hostio.hip); only the pointer tables are staged.
Prints one JSON line per workload: per-stage times (summed over chunks) and
the wall time of each direction, GiB/s over the bench's algorithmic bytes
(bench.py: encode (k + r) S per group, decode the peel's bytes), every
recovered segment checked against the original.  The device-resident rate
is bench.py's `value`; this one is PCIe-bound.

Usage: python tools/e2e_step.py [--groups 65536] [--reps 3] [--config c3|c3full|both]
                                [--mem pageable|pinned|both]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT)]

from bench import distinct_row_pairs, peel_bytes  # noqa: E402
from razor_amd.fec import fec_dtype, native, seg_dtype  # noqa: E402


def alloc(lib, n, dtype, mem, keep):
    if mem != "pinned":
        return np.zeros(n, dtype)
    a, kp = lib.pinned_array((n,), dtype)
    a.view(np.uint8)[...] = 0
    keep.append(kp)
    return a


def run(lib, G, full, reps, mem):
    k, S = 10, 1200
    plan = lib.plan_from_fraction(k, 80, 3 if full else 1)
    n = plan.n_lines
    rng = np.random.default_rng(5)
    keep = []
    segs = alloc(lib, G * k, seg_dtype(1200), mem, keep)
    segs["data"] = rng.integers(0, 256, (G * k, S), dtype=np.uint8)
    gi = np.repeat(np.arange(G, dtype=np.uint64), k)
    ii = np.tile(np.arange(k, dtype=np.uint64), G)
    segs["packet_id"] = (1 + gi * k + ii).astype(np.uint32)
    segs["fid"] = (1 + gi).astype(np.uint32)
    segs["timestamp"] = (33 * gi).astype(np.uint32)
    segs["index"] = ii
    segs["total"] = k
    segs["ftype"] = gi % 60 == 0
    segs["data_size"] = S
    fecs = alloc(lib, G * n, fec_dtype(1200), mem, keep)
    sp = segs.ctypes.data + np.arange(G * k, dtype=np.uint64) * segs.dtype.itemsize
    fp = fecs.ctypes.data + np.arange(G * n, dtype=np.uint64) * fecs.dtype.itemsize
    # the bench's erasures: 2 per group, distinct-row pairs (rows) / every recoverable pair (full plan)
    if full:
        pairs = np.array([(a, b) for a in range(k) for b in range(a + 1, k) if peel_bytes(plan, k, (a, b), S)])
    else:
        pairs = np.array(distinct_row_pairs(plan))
    pick = rng.integers(0, len(pairs), G)
    erased = np.sort(pairs[pick], axis=1)
    pb = np.array([peel_bytes(plan, k, tuple(p), S) for p in pairs.tolist()], np.int64)
    enc_bytes, dec_bytes = G * (k + n) * S, int(pb[pick].sum())
    sp_rx = sp.copy().reshape(G, k)
    sp_rx[np.arange(G), erased[:, 0]] = 0
    sp_rx[np.arange(G), erased[:, 1]] = 0
    out = alloc(lib, G * 2, seg_dtype(1200), mem, keep)
    op = out.ctypes.data + np.arange(G * 2, dtype=np.uint64) * out.dtype.itemsize
    lib.host_encode_groups(plan, G, sp, fp)  # warm: staging
    lib.host_recover_groups(plan, G, sp_rx.reshape(-1), fp, 2, op)
    enc = [lib.host_encode_groups(plan, G, sp, fp) for _ in range(reps)]
    dec = [lib.host_recover_groups(plan, G, sp_rx.reshape(-1), fp, 2, op) for _ in range(reps)]
    oi = dec[-1][0]
    ok = bool(np.array_equal(oi.astype(np.int64), erased))
    want = segs.reshape(G, k)[np.arange(G)[:, None], erased]
    for f in ("packet_id", "fid", "timestamp", "index", "data_size", "data"):
        ok = ok and bool(np.array_equal(out[f].reshape(G, 2, *out[f].shape[1:]), want[f]))
    med = lambda runs, key: float(np.median([r[key] for r in runs]))  # noqa: E731
    e_t = {key: med(enc, key) for key in enc[0] if key.endswith("_us")}
    d_t = {key: med([r[2] for r in dec], key) for key in dec[0][2] if key.endswith("_us")}
    wall = e_t["total_us"] + d_t["total_us"]
    zc = all(r["zero_copy"] for r in enc) and all(r[2]["zero_copy"] for r in dec)
    assert zc == (mem == "pinned") and (zc or not any(r["zero_copy"] for r in enc)), mem
    if zc:  # the structs themselves cross PCIe (16-B chunks from the data's dword), + 8-B pointers
        ss, fs = segs.dtype.itemsize, fecs.dtype.itemsize
        # receive side: whole structs only on the lines the decode reads (row layouts: the lines that hold an
        # erased member; the matrix plan: the first line firing at once per target, else the mask schedule),
        # the rest as a 64-B header
        lm = [set(plan.members(l)) for l in range(n)]
        cnt = {}
        for a, b in erased.tolist():
            cnt[(a, b)] = cnt.get((a, b), 0) + 1
        nseg = nfec = nhdr = 0
        cascade = full  # the sender's matrix plan: the dense cascade decode (rfec_hostmem.c zc_lines_read)
        for (a, b), m in cnt.items():
            held = [l for l in range(n) if a in lm[l] or b in lm[l]]  # received lines holding an erased member
            lines = lines_read(lm, k, {a, b}, 2) if cascade else held
            need = set().union(*(lm[l] for l in lines)) - {a, b}
            nseg += m * len(need)
            nfec += m * len(lines)
            if cascade:  # headers: the rest of the held lines (+ the first parity); nothing else crosses
                hs = set().union(*(lm[l] for l in held)) - {a, b} - need
                hf = (set(held) | {0}) - set(lines)
                nhdr += m * (len(hs) + len(hf))
            else:
                nhdr += m * (k - 2 - len(need) + n - len(lines))
        pcie = {"encode_h2d": G * k * (ss + 8) + G * n * 8, "encode_d2h": G * n * fs,
                "decode_h2d": nseg * ss + nfec * fs + nhdr * 64 + G * ((k + n + 2) * 8 + 24),
                "decode_d2h": G * 2 * ss + 17 * G * 2}
    else:  # decode H2D: the received payloads only, in 1,216-B slots (2 of k lost), + headers, masks, row maps
        pcie = {"encode_h2d": G * k * (S + 20), "encode_d2h": G * n * (S + 23),
                "decode_h2d": G * ((k - 2 + n) * 1216 + k * 20 + n * 22 + 24 + (k + n) * 4),
                "decode_d2h": G * 2 * (S + 21) + 16 * G}
    return {"workload": f"{'c3full' if full else 'c3'}: k10_r{n}_S1200_G{G}, host AoS in / out, {mem}",
            "zero_copy": zc,
            "encode_us": {x: round(v, 1) for x, v in e_t.items()},
            "decode_us": {x: round(v, 1) for x, v in d_t.items()},
            "encode_e2e_gibps": round(enc_bytes / (e_t["total_us"] * 1e-6) / 2**30, 2),
            "decode_e2e_gibps": round(dec_bytes / (d_t["total_us"] * 1e-6) / 2**30, 2),
            "step_e2e_gibps": round((enc_bytes + dec_bytes) / (wall * 1e-6) / 2**30, 2),
            "pcie_bytes": pcie,
            "bytes": {"encode": enc_bytes, "decode": dec_bytes}, "reps": reps, "verified": ok}


def lines_read(lm, k, erased, E):
    """rfec_hostmem.c zc_lines_read with every parity received: per erased member of rank < E, the first
    line (plan order) that fires at once for it; if one has none, every step of the canonical mask schedule."""
    n = len(lm)
    have = set(range(k)) - set(erased)
    lines, casc = set(), False
    for t in sorted(erased)[:E]:
        l = next((l for l in range(n) if t in lm[l] and (lm[l] - have) == {t} and lm[l] & have), None)
        if l is None:
            casc = True
        else:
            lines.add(l)
    if casc:
        h, er, progress = set(have), sorted(erased), True
        while progress:
            progress = False
            for l in range(n):
                x = lm[l] - h
                if len(x) != 1 or not (lm[l] & h):
                    continue
                t = next(iter(x))
                if er.index(t) >= E:
                    continue
                lines.add(l)
                h.add(t)
                progress = True
    return sorted(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--config", default="both", choices=("c3", "c3full", "both"))
    ap.add_argument("--mem", default="pageable", choices=("pageable", "pinned", "both"))
    args = ap.parse_args()
    lib = native(1200)
    for mem in (("pageable", "pinned") if args.mem == "both" else (args.mem,)):
        for full in ((False, True) if args.config == "both" else (args.config == "c3full",)):
            print(json.dumps(run(lib, args.groups, full, args.reps, mem)), flush=True)


if __name__ == "__main__":
    main()
