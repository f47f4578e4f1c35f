"""One-screen summary of a tools/gcmd_rx.sh directory: per run, datagrams/s and the per-batch stage split,
then the kernel table of the trace (rocprofv3 sqlite).  python tools/rx_summary.py gpurun_out/<tag>"""
import json
import sqlite3
import sys
from pathlib import Path

d = Path(sys.argv[1])
for f in sorted(d.glob("rx_*.json")):
    r = json.loads(f.read_text())
    for k, v in r.items():
        if isinstance(v, dict) and "threads" in v:
            c = v["calls"]
            st = {a: round(b / c, 1) for a, b in v["stage_us_sum"].items()}
            print(f"{f.stem:12s} {k:9s} {v['datagrams_per_s'] / 1e6:6.2f} M/s  wall/batch {v['wall_s'] / c * 1e6:6.1f} us  "
                  f"host {st['host_us']} kernel {st['kernel_us']} total {st['total_us']}  ok={v['verified_vs_oracle']}")
            print("      split/batch", v["host_split_us_per_batch"])
for log in sorted(d.glob("rx_*.log")):
    sh = [l.strip() for l in log.read_text().splitlines() if l.startswith("rx shard")]
    if sh:
        print(log.stem, *sh[-8:], sep="\n   ")
db = next(d.glob("rxprof/*.db"), None)
if db:
    c = sqlite3.connect(db)
    for n, cnt, avg, tot in c.execute("select name, count(*), avg(end-start)/1000.0, sum(end-start)/1e6 from kernels "
                                      "group by name order by 4 desc limit 10"):
        print(f"{cnt:5d} {avg:8.1f} us {tot:7.2f} ms  {n[:80]}")
