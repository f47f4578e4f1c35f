"""Per-phase kernel statistics from a rocprofv3 kernel trace of `python
bench.py` (the driver's default command): the FEC kernels' launches grouped
into the blocks they run in -- the headline's primed / warm-up / timed steps,
then (after the verification kernels) the c4_strong sub-object's 65,536-group
launches -- with calls / mean / median per kernel in each block, next to the
whole-run rocprofv3 --stats summary that averages both.

    python tools/phase_stats.py gpurun_out/<tag>/prof/run_kernel_trace.csv [--out stats.json]
"""
import argparse
import csv
import json
import re
import statistics as st

FEC = re.compile(r"(k_(?:encode|decode|cascade|peel|recover)\w*(?:<[^>]*>)?)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out", default="")
    ap.add_argument("--min-block", type=int, default=20, help="FEC launches that make a block")
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    blocks, cur, gap = [], [], 0
    for r in rows:
        m = FEC.search(r["Kernel_Name"])
        if m:
            cur.append((m.group(1), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
            gap = 0
        else:
            gap += 1
            if gap > 8 and cur:  # a run of other kernels (verification, fills) ends a block
                blocks.append(cur)
                cur = []
    if cur:
        blocks.append(cur)
    blocks = [b for b in blocks if len(b) >= args.min_block]
    names = ["headline (prime, warm-up, timed steps)", "c4_strong (65,536-group launches)", "c5 sub-object",
             "c5 sub-object, packed-record decode", "c3full sub-object"]
    out = []
    for i, b in enumerate(blocks):
        per = {}
        for n, us in b:
            per.setdefault(n, []).append(us)
        out.append({"block": names[i] if i < len(names) else f"block {i}",
                    "kernels": {n: {"calls": len(v), "mean_us": round(st.mean(v), 2), "median_us": round(st.median(v), 2),
                                    "min_us": round(min(v), 2), "max_us": round(max(v), 2)} for n, v in per.items()}})
    print(json.dumps(out, indent=1))
    if args.out:
        open(args.out, "w").write(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
