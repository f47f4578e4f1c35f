"""HBM traffic per launch from rocprofv3 PMC counters, for bench.py's
roofline.traffic.  Runs on the GPU box:

    python tools/pmc_traffic.py --out gpurun_out/<tag>/traffic.json [-- bench args]

Two separate counter passes of the same bench command (FETCH_SIZE and
WRITE_SIZE do not fit one pass on gfx950), each `rocprofv3 --pmc X
--kernel-trace --output-format csv -- python bench.py ...` started as a child
process (this parent never touches the GPU).  Corrections as
MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced streaming
read, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

KERNELS = {"encode": ("k_encode",), "decode": ("k_decode_rows", "k_decode_out", "k_decode_disjoint", "k_decode_cascade",
                                              "k_decode_matrix"),
           "check": ("k_cascade_check",), "peel": ("k_peel",), "recover": ("k_recover",)}


def run_pass(counter, outdir, bench_args, timeout):
    d = Path(outdir) / f"pmc_{counter}"
    d.mkdir(parents=True, exist_ok=True)
    cmd = ["rocprofv3", "--pmc", counter, "--kernel-trace", "--output-format", "csv", "-d", str(d), "-o", "run",
           "--", sys.executable, str(ROOT / "bench.py"), "--no-cpu"] + bench_args
    print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, cwd=ROOT, timeout=timeout, capture_output=True, text=True)
    (d / "stdout.log").write_text(r.stdout + "\n" + r.stderr)
    if r.returncode != 0:
        raise SystemExit(f"rocprofv3 pass {counter} failed with {r.returncode}; see {d}/stdout.log")
    files = glob.glob(str(d / "**" / "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    return files, (json.loads(line[-1]) if line else None)


def per_kernel(files, counter):
    vals = defaultdict(list)
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                for key, pats in KERNELS.items():
                    if any(p in name for p in pats):
                        vals[key].append(float(row["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--timeout", type=int, default=400)
    ap.add_argument("bench_args", nargs="*", default=[])
    args = ap.parse_args()
    bench_args = args.bench_args or ["--steps", "10", "--warmup", "2"]
    outdir = Path(args.out).parent
    ffiles, bench_line = run_pass("FETCH_SIZE", outdir, bench_args, args.timeout)
    fetch = per_kernel(ffiles, "FETCH_SIZE")
    write = per_kernel(run_pass("WRITE_SIZE", outdir, bench_args, args.timeout)[0], "WRITE_SIZE")
    # the workload the bench ran
    groups = 65536
    for i, a in enumerate(bench_args):
        if a == "--groups":
            groups = int(bench_args[i + 1])
    S, k, r = 1200, 10, 3
    enc_alg = groups * (k + r) * S
    cfg = (bench_line or {}).get("config", {})
    groups = cfg.get("groups_per_gpu", groups)
    if cfg.get("bytes_per_step_per_gpu", {}).get("encode"):  # the bench's own workload (any plan)
        enc_alg = cfg["bytes_per_step_per_gpu"]["encode"]
        S, k, r = cfg.get("payload_bytes", S), cfg.get("k", k), cfg.get("r", r)
    res = {}
    for key in KERNELS:
        f, w = fetch.get(key, []), write.get(key, [])
        if not f or not w:
            continue
        fb = sum(f) / len(f) * 1024
        wb = sum(w) / len(w) * 1024
        res[key] = {"launches": len(f), "fetch_size_kib_avg": fb / 1024, "write_size_kib_avg": wb / 1024,
                    "hbm_read_bytes_corrected": 2 * fb, "hbm_write_bytes": wb, "hbm_bytes": 2 * fb + wb}
    entry = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), FETCH doubled (gfx950)",
             "bench_args": bench_args, "kernels": res}
    if "encode" in res:
        entry["encode_hbm_bytes_per_launch"] = res["encode"]["hbm_bytes"]
        entry["encode_algorithmic_bytes"] = enc_alg
        entry["encode_traffic_over_algorithmic"] = res["encode"]["hbm_bytes"] / enc_alg
    dec_alg = (bench_line or {}).get("config", {}).get("bytes_per_step_per_gpu", {}).get("decode")
    if "recover" in res and dec_alg:  # two-kernel decode (plans with columns)
        entry["recover_traffic_over_algorithmic"] = res["recover"]["hbm_bytes"] / dec_alg
    if "decode" in res and dec_alg:
        entry["decode_hbm_bytes_per_launch"] = res["decode"]["hbm_bytes"]
        entry["decode_algorithmic_bytes"] = dec_alg
        entry["decode_traffic_over_algorithmic"] = res["decode"]["hbm_bytes"] / dec_alg
        if "check" in res:  # the cascade decode's two launches together
            entry["decode_with_check_traffic_over_algorithmic"] = (res["decode"]["hbm_bytes"] +
                                                                   res["check"]["hbm_bytes"]) / dec_alg
    name = f"k{k}_r{r}_S{S}_G{groups}" + ("+packed" if "--packed-decode" in bench_args else "")
    Path(args.out).write_text(json.dumps({name: entry}, indent=1))
    print(json.dumps({name: entry}, indent=1))


if __name__ == "__main__":
    main()
