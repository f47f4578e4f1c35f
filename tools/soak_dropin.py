"""Randomised soak of the group-level drop-in (include/razor_flex.h through the
resident service) against the oracle (GPU box).

Each iteration: a group of k = 2..160 ragged segments and a random protect
fraction; flex_fec_sender_update's parities (count, line index, meta,
fec_data_size, payload) == the oracle's encode of the sender's plan; then,
when every line was emitted and k <= 128, a random erasure pattern (0-6 segments, a lost
parity with probability 0.3) through the flex receiver (segments, then
parities, then the recovered ones cascading back in), whose recovered set ==
the oracle's peel.  Prints a line per iteration; JSON summary; exit 1 on a
mismatch.

    python tools/soak_dropin.py [--seconds 120] [--seed 1] [--out file.json]
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
from test_flex_dropin import bind_flex, make_segments, run_receiver, sender_group  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    rng = np.random.default_rng(args.seed)
    o = po.Oracle(1000)
    lib = bind_flex(native(1000))
    snd = lib.lib.flex_fec_sender_create()
    t0 = time.time()
    it, rx_it, fails, lines = 0, 0, [], 0
    try:
        while time.time() - t0 < args.seconds:
            k = int(rng.integers(2, 161))
            pf = int(rng.choice([1, 5, 10, 20, 40, 80, 120, 200, 255]))
            shards, hdr = o.fill_groups(int(rng.integers(100, 100000)), 1, k, 1000, ragged=True)
            plan = o.plan_from_fraction(k, pf, 3)
            e_p, e_m, e_f, e_s = o.encode_batch(plan, shards, hdr, 1000)
            segs = make_segments(lib, shards[0], hdr[0])
            fecs = sender_group(lib, snd, segs, pf)
            emitted = [l for l in range(plan.n_lines) if e_s[0, l] == 0]
            what = None
            if len(fecs) != len(emitted):
                what = f"{len(fecs)} parities, oracle {len(emitted)}"
            else:
                for f, l in zip(fecs, emitted):
                    L = int(e_f[0, l])
                    meta = np.frombuffer(bytes(f.fec_meta), po.HDR_DTYPE)[0]
                    if f.index != plan.line[l].index or f.fec_data_size != L:
                        what = f"line {l}: index / size"
                    elif meta.tobytes() != e_m[0, l].tobytes():
                        what = f"line {l}: meta"
                    elif bytes(f.fec_data)[:L] != e_p[0, l, :L].tobytes():
                        what = f"line {l}: payload"
                    if what:
                        break
            lines += len(fecs)
            it += 1
            tag = f"{it} k={k} pf={pf} lines={plan.n_lines} emitted={len(fecs)}"
            if not what and len(emitted) == plan.n_lines and plan.n_lines and k <= 128:  # (128-bit masks)
                # the receiver: a random erasure pattern against the oracle's peel
                m = (1 << k) - 1
                er = rng.choice(k, int(rng.integers(0, min(6, k) + 1)), replace=False)
                for i in er:
                    m &= ~(1 << int(i))
                pp = (1 << plan.n_lines) - 1
                if rng.random() < 0.3:
                    pp &= ~(1 << int(rng.integers(plan.n_lines)))
                present = [m & (2**64 - 1), m >> 64]
                fresh = make_segments(lib, shards[0], hdr[0])
                got, _ = run_receiver(lib, fresh, fecs, present, pp, fresh[0].packet_id)
                rx, rh = shards.copy(), hdr.copy()
                for i in er:
                    rx[0, int(i)] = 0
                    rh[0, int(i)] = np.zeros((), po.HDR_DTYPE)
                pr = np.array([present], np.uint64)
                _, _, e_rec = o.recover_batch(plan, rx, rh, pr, e_p, e_m, e_f, np.array([pp], np.uint64), 1000)
                exp = [int(e_rec[0, 0]), int(e_rec[0, 1])]
                rx_it += 1
                tag += f" erased={len(er)} rx"
                if got != exp:
                    what = f"receiver recovered {got} != oracle {exp}"
            line = tag + (" ok" if not what else " FAIL " + what)
            print(line, flush=True)
            if what:
                fails.append(line)
    finally:
        lib.lib.flex_fec_sender_destroy(snd)
    out = {"sender_groups": it, "parities": lines, "receiver_patterns": rx_it, "seconds": round(time.time() - t0, 1),
           "seed": args.seed, "failures": fails}
    print(json.dumps(out))
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1))
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
