"""Randomised soak of the batched device API against the oracle (GPU box).

Each iteration draws a configuration -- k in 2..64, the sender's plan for a
random protect fraction (rows only or rows + columns), a payload size, 256-2048
groups, 0-6 erasures per group, lost parities, header corruptions that make
the exact peel reject lines, the generic or the default kernels -- and checks:
  encode: parities, metas, fec_data_size, status == oracle
  recover (in place): recovered masks, headers and data == oracle's peel
  recover_out (dense, E random): out slots, headers, indices, masks == oracle
  recover_packed_out (row layouts of rows <= 4, k <= 64; a third of the
    iterations draw the row layer alone): the same, from packed erasure records
and, every other iteration, the wire codec on a random batch (SIM_SEG or
SIM_FEC, capacity 16-1999, 1-20k datagrams): framed bytes and lengths ==
oracle, then parse of the datagrams with random bytes flipped in ~5 % of them
(records, statuses, payload slots == oracle; the intact ones round-trip).
Runs for --seconds (default 120), prints one line per iteration (so a hang
is visible), and writes a JSON summary; exit 1 on any mismatch.

    python tools/soak.py [--seconds 120] [--seed 1] [--out gpurun_out/soak.json]
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
from gpu_engine import GpuEngine  # noqa: E402
from gpu_engine import GpuWire  # noqa: E402
from test_gpu_parity import _lossy_rx  # noqa: E402
import wire_cases as wc  # noqa: E402


def check_wire(o, gw, rng):
    capacity = int(rng.integers(16, 2000))
    stride = (capacity + 15) // 16 * 16 + 16 * int(rng.integers(0, 3))
    N = int(rng.integers(1, 20001))
    seg = bool(rng.random() < 0.5)
    data, hdr, sizes, stamps = wc.random_batch(rng, N, stride, capacity, seg=seg)
    over = 36 if seg else 49
    dstride = min(2048, (capacity + over + 15) // 16 * 16)
    if seg:
        g, gl = gw.frame_seg(data, hdr, stamps, capacity, dstride)
        e, el = o.frame_seg_batch(data, hdr, stamps, capacity, dstride)
    else:
        g, gl = gw.frame_fec(data, hdr, sizes, None, stamps, capacity, dstride)
        e, el = o.frame_fec_batch(data, hdr, sizes, None, stamps, capacity, dstride)
    if not (np.array_equal(gl, el) and np.array_equal(g, e)):
        return f"frame {'seg' if seg else 'fec'} N={N} cap={capacity}", (capacity, N, seg)
    bad = rng.random(N) < 0.05
    for i in np.nonzero(bad)[0]:
        L = int(gl[i])
        if L:
            g[i, int(rng.integers(L))] ^= np.uint8(1 << int(rng.integers(8)))
    recs, pay = gw.parse(g, gl, stride, capacity)
    orecs, opay = o.parse_batch(g, gl, stride, capacity)
    if not (np.array_equal(recs.view(np.uint8), orecs.view(np.uint8)) and np.array_equal(pay, opay)):
        return f"parse N={N} cap={capacity}", (capacity, N, seg)
    ok = ~bad
    if not (np.array_equal(pay[ok], data.reshape(N, -1)[ok]) and (recs["status"][ok] == 0).all()):
        return f"roundtrip N={N} cap={capacity}", (capacity, N, seg)
    if bad.any() and not (recs["status"][bad] != 0).all():
        return f"a flipped bit passed the CRC N={N}", (capacity, N, seg)
    return None, (capacity, N, seg)


def check_encode(o, eng, plan, shards, hdr, cap):
    """as tests/test_gpu_parity.py: status and sizes everywhere, metas and
    parity bytes (up to fec_data_size) of the lines the reference emits"""
    e_p, e_m, e_f, e_s = o.encode_batch(plan, shards, hdr, cap)
    p, m, f, st = eng.encode(plan, shards, hdr, cap)
    if not (np.array_equal(st, e_s) and np.array_equal(f, e_f)):
        return "encode status / sizes"
    ok = e_s == 0
    if not np.array_equal(m[ok], e_m[ok]):
        return "encode meta"
    for g, l in zip(*np.nonzero(ok)):
        L = int(e_f[g, l])
        if not np.array_equal(p[g, l, :L], e_p[g, l, :L]):
            return f"encode parity g{g} l{l}"
    return None


def check_recover(o, eng, plan, k, args):
    rx, rh, present, parity, meta, fs, pp, cap = args
    e_s, e_h, e_rec = o.recover_batch(plan, rx, rh, present, parity, meta, fs, pp, cap)
    g_s, g_h, g_rec = eng.recover(plan, rx, rh, present, parity, meta, fs, pp, cap)
    if not np.array_equal(g_rec, e_rec):
        return "recovered masks"
    G = rx.shape[0]
    for gi in range(G):
        m = int(e_rec[gi, 0]) | (int(e_rec[gi, 1]) << 64)
        for i in range(k):
            if (m >> i) & 1:
                if g_h[gi, i] != e_h[gi, i]:
                    return f"header g{gi} s{i}"
                L = int(e_h[gi, i]["size"])
                if not np.array_equal(g_s[gi, i, :L], e_s[gi, i, :L]):
                    return f"data g{gi} s{i}"
    return None


def check_dense(o, eng, plan, E, args):
    rx, rh, present, parity, meta, fs, pp, cap = args
    e_s, e_h, e_i, e_rec = o.recover_batch_out(plan, rx, rh, present, parity, meta, fs, pp, cap, E)
    g_s, g_h, g_i, g_rec = eng.recover_out(plan, rx, rh, present, parity, meta, fs, pp, cap, E)
    if not np.array_equal(g_rec, e_rec):
        return "dense recovered masks"
    if not np.array_equal(g_i, e_i):
        return "dense out_index"
    for gi in range(rx.shape[0]):
        for e in range(E):
            if e_i[gi, e] == 0xFF:
                continue
            if g_h[gi, e] != e_h[gi, e]:
                return f"dense header g{gi} e{e}"
            L = int(e_h[gi, e]["size"])
            if not np.array_equal(g_s[gi, e, :L], e_s[gi, e, :L]):
                return f"dense data g{gi} e{e}"
    return None


def check_packed(o, eng, plan, E, args):
    """rfec_pack_erasures + rfec_recover_packed_out == the oracle's dense recovery"""
    rx, rh, present, parity, meta, fs, pp, cap = args
    e_s, e_h, e_i, e_rec = o.recover_batch_out(plan, rx, rh, present, parity, meta, fs, pp, cap, E)
    g_s, g_h, g_i, g_rec, _ = eng.recover_packed(plan, rx, rh, present, parity, meta, fs, pp, cap, E)
    if not np.array_equal(g_rec, e_rec):
        return "packed recovered masks"
    if not np.array_equal(g_i, e_i):
        return "packed out_index"
    for gi, e in zip(*np.nonzero(e_i != 0xFF)):
        if g_h[gi, e] != e_h[gi, e]:
            return f"packed header g{gi} e{e}"
        L = int(e_h[gi, e]["size"])
        if not np.array_equal(g_s[gi, e, :L], e_s[gi, e, :L]):
            return f"packed data g{gi} e{e}"
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    rng = np.random.default_rng(args.seed)
    o = po.Oracle(1000)
    engines = {t: GpuEngine(1000, tuning=t) for t in (0, 1)}
    gw = GpuWire(1000)
    t0 = time.time()
    it, fails, groups, cfgs, wit, dgrams, pk_groups = 0, [], 0, set(), 0, 0, 0
    while time.time() - t0 < args.seconds:
        if (it + wit) % 2 == 1:
            what, (cap_w, N, seg) = check_wire(o, gw, rng)
            wit += 1
            dgrams += N
            line = f"wire {wit} {'SIM_SEG' if seg else 'SIM_FEC'} cap={cap_w} N={N} " + ("ok" if not what
                                                                                     else "FAIL " + what)
            print(line, flush=True)
            if what:
                fails.append(line)
            continue
        k = int(rng.integers(2, 65))
        pf = int(rng.choice([5, 10, 20, 40, 80, 120, 200, 255]))
        plan = o.plan_from_fraction(k, pf, 1 if rng.random() < 1 / 3 else 3)
        if plan.n_lines == 0:
            continue
        S = int(rng.choice([16, 64, 200, 256, 512, 1000]))
        G = int(rng.choice([256, 512, 1024, 2048]))
        tuning = int(rng.integers(0, 2))
        eng = engines[tuning]
        top = int(min(6, k))
        shards, hdr, rx, rh, present, parity, meta, fs, pp, cap = _lossy_rx(
            o, plan, k, G, S, rng, lambda r: r.integers(0, top + 1), p_lost_parity=float(rng.random() * 0.4),
            corrupt=float(rng.choice([0.0, 0.2, 0.45])))
        rargs = (rx, rh, present, parity, meta, fs, pp, cap)
        E = int(rng.integers(1, min(k, 6) + 1))
        packed = eng.lib.packed_stride(plan, E) > 0
        what = (check_encode(o, eng, plan, shards, hdr, cap) or check_recover(o, eng, plan, k, rargs)
                or check_dense(o, eng, plan, E, rargs) or (packed and check_packed(o, eng, plan, E, rargs)) or None)
        pk_groups += G if packed else 0
        it += 1
        groups += G
        cfgs.add((k, plan.n_lines))
        line = (f"{it} k={k} pf={pf} lines={plan.n_lines} S={S} G={G} E={E} tuning={tuning} packed={int(packed)} "
                + ("ok" if not what else "FAIL " + what))
        print(line, flush=True)
        if what:
            fails.append(line)
    out = {"iterations": it, "groups": groups, "packed_groups": pk_groups, "distinct_k_lines": len(cfgs),
           "wire_iterations": wit,
           "datagrams": dgrams, "seconds": round(time.time() - t0, 1), "seed": args.seed, "failures": fails}
    print(json.dumps(out))
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1))
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
