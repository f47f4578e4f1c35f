"""Per-kernel SQ / TCC counter averages from one rocprofv3 --pmc pass (the
instruction mix and LDS cycles behind a kernel's time).  The counter pass is
a child process; this parent never touches the GPU.

Usage (GPU box):
  python tools/pmc_sq.py --tag NAME --counters "SQ_WAVES SQ_INSTS_VALU ..." \
      --match k_frame_seg,k_parse -- python tools/wire_bench.py --reps 3
Writes gpurun_out/pmc_sq/NAME.json: {kernel: {counter: mean per dispatch}}.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import subprocess
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def main():
    argv = sys.argv[1:]
    cmd = argv[argv.index("--") + 1:] if "--" in argv else []
    argv = argv[:argv.index("--")] if "--" in argv else argv
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--counters", required=True)
    ap.add_argument("--match", required=True)
    ap.add_argument("--timeout", type=int, default=120)
    ap.add_argument("--by-grid", action="store_true", help="one entry per (kernel, grid size): launches of one "
                    "kernel over different batches (e.g. the SIM_FEC and SIM_SEG parses) kept apart")
    args = ap.parse_args(argv)
    d = ROOT / "gpurun_out" / "pmc_sq" / args.tag
    d.mkdir(parents=True, exist_ok=True)
    full = ["rocprofv3", "--pmc", *args.counters.split(), "--kernel-trace", "--output-format", "csv", "-d", str(d),
            "-o", "run", "--", *cmd]
    print(" ".join(full), flush=True)
    r = subprocess.run(full, cwd=ROOT, timeout=args.timeout, capture_output=True, text=True)
    (d / "stdout.log").write_text(r.stdout + "\n" + r.stderr)
    if r.returncode != 0:
        raise SystemExit(f"rocprofv3 failed with {r.returncode}; see {d}/stdout.log")
    pats = args.match.split(",")
    acc = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> summed over instances
    for f in glob.glob(str(d / "**" / "*counter_collection.csv"), recursive=True):
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                pat = next((p for p in pats if p in name), None)
                if pat is None:
                    continue
                if args.by_grid:
                    pat = f"{pat}@grid{row.get('Grid_Size', row.get('Grid_Size_X', ''))}"
                acc[(pat, row.get("Dispatch_Id", ""))][row["Counter_Name"]] += float(row["Counter_Value"])
    out = defaultdict(lambda: defaultdict(list))
    for (pat, _), cs in acc.items():
        for c, v in cs.items():
            out[pat][c].append(v)
    res = {k: {c: sum(v) / len(v) for c, v in cs.items()} | {"dispatches": len(next(iter(cs.values())))}
           for k, cs in out.items()}
    print(json.dumps(res, indent=1))
    (ROOT / "gpurun_out" / "pmc_sq" / f"{args.tag}.json").write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
