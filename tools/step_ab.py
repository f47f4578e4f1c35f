"""Interleaved A/B of encode / decode kernel flags in bench.py's own step
(encode then decode, disjoint buffer sets rotated per step so no operand is
MALL-resident), per-kernel HIP events on the launch stream, medians.

Usage (GPU box): python tools/step_ab.py [--rounds 6] [--reps 10] [--variants name,...]
                 [--k 32 --payload 256 --col 4] [--full-plan] [--cold]
--cold decodes the set encoded one step earlier (bench.py's receiver-realistic
order), so the decode's parity operand has been pushed out of the MALL.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from bench import Workload  # noqa: E402
from razor_amd.fec import native  # noqa: E402

FLAT, META_TAIL, NT, WT, WTNT, PLAIN, FLATDEC = 65536, 131072, 512, 64, 64 | 128, 4, 262144
VARIANTS = {
    "default": (0, 0),
    "enc flat (r01 default)": (FLAT, 0),
    "enc out nt": (NT, 0),
    "enc out wtnt": (WTNT, 0),
    "enc out plain": (PLAIN, 0),
    "enc out meta_tail": (META_TAIL, 0),
    "enc out meta_tail nt": (META_TAIL | NT, 0),
    "enc flat nt": (FLAT | NT, 0),
    "dec flat (r01 default)": (0, FLATDEC),
    "dec out wt": (0, WT),
    "dec out plain": (0, PLAIN),
    "dec out wtnt": (0, WTNT),
    "dec lds hdr peel": (0, 32768),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--groups", type=int, default=65536)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--payload", type=int, default=1200)
    ap.add_argument("--col", type=int, default=0)
    ap.add_argument("--full-plan", action="store_true")
    ap.add_argument("--sets", type=int, default=2)
    ap.add_argument("--cold", action="store_true")
    ap.add_argument("--variants", default="")
    ap.add_argument("--extra", default="", help="name=enc_flags:dec_flags;...")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    variants = dict(VARIANTS)
    if args.variants:
        variants = {k: variants[k] for k in args.variants.split(",")}
    for item in filter(None, args.extra.split(";")):  # extras always run
        name, fl = item.split("=")
        e, d = fl.split(":")
        variants[name] = (int(e, 0), int(d, 0))
    dev = torch.device("cuda", 0)
    lib = native(1000)
    sets = [Workload(lib, args.groups, args.k, args.payload, 80, dev, 0, seed=11 + i, col=args.col,
                     full_plan=args.full_plan) for i in range(args.sets)]
    w = sets[0]
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    te = {k: [] for k in variants}
    td = {k: [] for k in variants}
    n = len(sets)
    for r in range(args.rounds + 1):
        for name, (fe, fd) in variants.items():
            ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.reps)]
            for i in range(args.reps):
                a, b, c = ev[i]
                a.record(stream)
                lib.set_tuning(fe)
                sets[i % n].encode(sp)
                b.record(stream)
                lib.set_tuning(fd)
                sets[(i - 1) % n if args.cold else i % n].decode(sp)
                c.record(stream)
            torch.cuda.synchronize()
            if r == 0:
                continue  # warm-up round
            te[name] += [a.elapsed_time(b) * 1e3 for a, b, _ in ev]
            td[name] += [b.elapsed_time(c) * 1e3 for _, b, c in ev]
    lib.set_tuning(0)
    res = {}
    print(f"{'variant':28s} {'enc_us':>8s} {'enc_min':>8s} {'frac':>6s} {'dec_us':>8s} {'dec_min':>8s} {'frac':>6s} {'step GiB/s':>10s}")
    for name in variants:
        e, d = float(np.median(te[name])), float(np.median(td[name]))
        fe, fd = w.enc_bytes / e / 8e6, w.dec_bytes / d / 8e6
        step = (w.enc_bytes + w.dec_bytes) / ((e + d) * 1e-6) / 2**30
        res[name] = {"enc_us": e, "enc_min_us": min(te[name]), "enc_frac": fe, "dec_us": d, "dec_min_us": min(td[name]),
                     "dec_frac": fd, "step_gibps": step, "flags": variants[name]}
        print(f"{name:28s} {e:8.1f} {min(te[name]):8.1f} {fe:6.3f} {d:8.1f} {min(td[name]):8.1f} {fd:6.3f} {step:10.1f}")
    ok = all(s.verify() for s in sets)
    print("verified", ok)
    if args.out:
        Path(args.out).parent.mkdir(parents=True, exist_ok=True)
        Path(args.out).write_text(json.dumps({"results": res, "verified": ok, "args": vars(args)}, indent=1))


if __name__ == "__main__":
    main()
