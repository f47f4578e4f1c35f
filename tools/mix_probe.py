"""HBM ceiling of the encodes' read / write mixes (GPU box): rfec_probe_mix
over r read : w write streams of the c3 group count (65,536 x 1,200 B per
stream), two rotated buffer sets (MALL-proof), 30 timed launches each,
event-timed.  Prints one JSON line per mix: the launch time, the bytes it
moves and the fraction of 8 TB/s -- the bound the FEC kernel of the same mix
is measured against (10 : 3 row encode, 10 : 7 full 3 x 4 plan, 4 : 1 the c5 rows of 4).

    python tools/mix_probe.py [--groups 65536] [--payload 1200]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from razor_amd.fec import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=65536)
    ap.add_argument("--payload", type=int, default=1200)
    ap.add_argument("--reps", type=int, default=30)
    args = ap.parse_args()
    lib = native(1000)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    for r, w, S in ((10, 3, args.payload), (10, 7, args.payload), (4, 1, 256 * 8), (1, 1, args.payload)):
        sb = args.groups * S
        sets = [(torch.empty(r * sb, dtype=torch.uint8, device=dev), torch.empty(w * sb, dtype=torch.uint8, device=dev))
                for _ in range(2)]
        for a, b in sets:
            a.fill_(1)

        def run(i):
            a, b = sets[i % 2]
            rc = lib.lib.rfec_probe_mix(a.data_ptr(), b.data_ptr(), sb, r, w, st)
            if rc:
                raise RuntimeError(f"rfec_probe_mix {r}:{w} -> {rc}")

        for i in range(4):
            run(i)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
        torch.cuda.synchronize()
        for i, (e0, e1) in enumerate(ev):
            e0.record()
            run(i)
            e1.record()
        torch.cuda.synchronize()
        ts = sorted(e0.elapsed_time(e1) * 1e3 for e0, e1 in ev)
        us = ts[len(ts) // 2]
        nbytes = (r + w) * sb
        print(json.dumps({"mix": f"{r}:{w}", "stream_bytes": sb, "bytes": nbytes, "median_us": round(us, 2),
                          "min_us": round(ts[0], 2), "TBps": round(nbytes / us / 1e6, 3),
                          "frac_of_8TBps": round(nbytes / us / 1e6 / 8.0, 4)}), flush=True)
        del sets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
