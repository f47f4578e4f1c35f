"""Interleaved A/B of the encode / decode kernel variants and the HBM ceiling
probes on one GPU, one process (cdna_hip_programming.md §5.4 rule 24).

Usage (GPU box): python tools/ab_encode.py [--rounds 5] [--reps 20] [--out gpurun_out/ab.json]
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

ENC_VARIANTS = {
    "default(nt_ld+wt_st)": 0,
    "nt_st": 512,
    "plain_st": 4,
    "wt_nt_st": 192,
    "plain_ld": 2,
    "items2": 8,
    "generic": 1,
    "diag_no_meta": 256,
    "group_wave": 8192,
    "group_wave_xcd": 8192 | 16384,
    "xcd": 16384,
}
DEC_VARIANTS = {"fused(default nt_st)": 0, "fused_wt_st": 64, "fused_plain_st": 4, "fused_plain_ld": 2,
                "two_kernel": 4096, "two_kernel_wt_st": 4096 | 64, "diag_const_sched": 4096 | 1024, "wave": 16,
                "pipe": 32, "fused_items2": 8, "fused_items2_wt": 8 | 64, "fused_group_wave": 8192, "fused_group_wave_xcd": 8192 | 16384}
# (encode flags, decode flags)
STEP_VARIANTS = {"default (enc wt, dec nt)": (0, 0), "enc nt, dec nt": (512, 512), "enc nt, dec wt": (512, 64),
                 "enc wt, dec wt": (64, 64), "enc items2": (8, 0), "dec pipe": (0, 32), "dec diag const sched": (0, 4096 | 1024), "dec two-kernel": (0, 4096), "dec wave": (0, 16),
                 "group_wave both": (8192, 8192), "dec items2": (0, 8), "dec items2 plain st": (0, 8 | 4),
                 "dec plain st": (0, 4), "group_wave+xcd both": (8192 | 16384, 8192 | 16384)}


def timeit(fn, reps, stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--groups", type=int, default=65536)
    ap.add_argument("--out", default="gpurun_out/ab.json")
    ap.add_argument("--stride", type=int, default=0)
    ap.add_argument("--step-only", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = native(1000)
    w = Workload(lib, args.groups, 10, 1200, 80, dev, 0, seed=5, stride=args.stride or None)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    nb = 1 << 30
    a = torch.empty(nb, dtype=torch.uint8, device=dev)
    b = torch.empty(nb, dtype=torch.uint8, device=dev)
    sink = torch.zeros(16384, dtype=torch.uint8, device=dev)
    a.random_(0, 255)

    def enc(flags):
        def f():
            lib.set_tuning(flags)
            w.encode(sp)
        return f

    def dec(flags):
        def f():
            lib.set_tuning(flags)
            w.decode(sp)
        return f

    def probe(kind, flags):
        L = lib.lib
        if kind == "read":
            return lambda: L.rfec_probe_read(a.data_ptr(), nb, sink.data_ptr(), flags, sp)
        if kind == "copy":
            return lambda: L.rfec_probe_copy(a.data_ptr(), b.data_ptr(), nb // 2, flags, sp)
        return lambda: L.rfec_probe_write(b.data_ptr(), nb, flags, sp)

    cases = {}
    for k, f in ENC_VARIANTS.items():
        cases[f"enc/{k}"] = (enc(f), w.enc_bytes)
    for k, f in DEC_VARIANTS.items():
        cases[f"dec/{k}"] = (dec(f), w.dec_bytes)
    for kind, bytes_ in (("read", nb), ("copy", nb), ("write", nb)):
        for fl, name in ((0, "plain"), (1, "nt"), (2, "plain_x4"), (3, "nt_x4")):
            cases[f"probe_{kind}/{name}"] = (probe(kind, fl), bytes_)
    if args.step_only:
        cases = {}
    res = {k: [] for k in cases}
    for k, (fn, _) in cases.items():  # warm
        fn()
    torch.cuda.synchronize()
    for r in range(args.rounds):
        for k, (fn, _) in cases.items():
            res[k].append(timeit(fn, args.reps, stream))
    # step mode, as bench.py runs it: encode then decode, alternating, with
    # per-kernel events (what one kernel leaves dirty in L2/MALL is paid by the next)
    step_res = {}
    for name, (fe, fd) in STEP_VARIANTS.items():
        te, td = [], []
        for r in range(args.rounds):
            ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.reps)]
            for i in range(args.reps):
                ev[i][0].record(stream)
                lib.set_tuning(fe)
                w.encode(sp)
                ev[i][1].record(stream)
                lib.set_tuning(fd)
                w.decode(sp)
                ev[i][2].record(stream)
            torch.cuda.synchronize()
            te += [a.elapsed_time(b) / 1e3 for a, b, _ in ev[2:]]
            td += [b.elapsed_time(c) / 1e3 for _, b, c in ev[2:]]
        step_res[name] = (float(np.median(te)), float(np.median(td)))
    lib.set_tuning(0)
    out = {}
    print(f"{'case':32s} {'median_us':>10s} {'min_us':>10s} {'GB/s(med)':>10s} {'frac8T':>7s}")
    for k, (_, bytes_) in cases.items():
        t = np.array(res[k])
        med, mn = float(np.median(t)), float(t.min())
        gbs = bytes_ / med / 1e9
        out[k] = {"median_us": med * 1e6, "min_us": mn * 1e6, "GBps": gbs, "frac_of_8TBps": gbs / 8000, "bytes": bytes_}
        print(f"{k:32s} {med * 1e6:10.1f} {mn * 1e6:10.1f} {gbs:10.1f} {gbs / 8000:7.3f}")
    print(f"\nstep mode (encode -> decode alternating), medians:")
    print(f"{'flags':32s} {'enc_us':>8s} {'enc_GB/s':>9s} {'dec_us':>8s} {'dec_GB/s':>9s} {'step_GiB/s':>10s}")
    for name, (te, td) in step_res.items():
        stepg = (w.enc_bytes + w.dec_bytes) / (te + td) / 2**30
        out[f"step/{name}"] = {"enc_us": te * 1e6, "dec_us": td * 1e6, "enc_GBps": w.enc_bytes / te / 1e9,
                               "dec_GBps": w.dec_bytes / td / 1e9, "step_GiBps": stepg}
        print(f"{name:32s} {te * 1e6:8.1f} {w.enc_bytes / te / 1e9:9.1f} {td * 1e6:8.1f} "
              f"{w.dec_bytes / td / 1e9:9.1f} {stepg:10.1f}")
    ok = w.verify()
    print("verify", ok)
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps({"results": out, "verified": ok,
                                          "device": torch.cuda.get_device_name(0)}, indent=1))


if __name__ == "__main__":
    main()
