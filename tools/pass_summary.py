"""One-screen summary of a tools/measure.sh pass (container side):

    python tools/pass_summary.py gpurun_out/<tag>     (or profiles/r05/final)

Prints the numbers DESIGN.md §5 quotes: the default line (headline, c4_strong,
c5 with its packed-record decode, c3full), the --config c3full / c5 lines, the
traffic ratios, the r:w probes, end to end, wire and the drop-in group bench.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path


def last_json(p: Path):
    if p.suffix == ".json" and p.exists():
        lines = [l for l in p.read_text().splitlines() if l.startswith("{")]
        return json.loads(lines[-1]) if lines and len(lines) == 1 else json.loads(p.read_text())
    lines = [l for l in p.read_text().splitlines() if l.startswith("{")]
    return json.loads(lines[-1])


def main():
    d = Path(sys.argv[1])
    src = (lambda n: d / f"{n}.log") if (d / "bench.log").exists() else (lambda n: d / f"{n}.json")
    b = last_json(src("bench"))
    r, dr = b["roofline"], b["decode_roofline"]
    print(f"headline value {b['value']} GiB/s, {b['ms_per_step']} ms/step; encode {r['launch_us']} us {r['frac']} "
          f"(x{r['mix_ceiling']['kernel_vs_ceiling']} of {r['mix_ceiling']['frac_of_peak']}); decode "
          f"{dr['launch_us']} us {dr['frac']}")
    print(f"c4_strong {b['c4_strong']['value']}")
    for s in ("c5", "c3full"):
        c = b[s]
        pk = c.get("decode_packed") or {}
        print(f"{s} sub {c['value']}; encode {c['encode']['launch_us']} us {c['encode']['frac']} "
              f"(x{c['encode']['mix_ceiling']['kernel_vs_ceiling']}); decode {c['decode']['launch_us']} us "
              f"{c['decode']['frac']}; packed {pk.get('launch_us')} {pk.get('frac')}; verified {c['verified']} "
              f"digest {c['verified_vs_reference_digest']}")
    cb = b.get("cpu_baseline") or {}
    print(f"cpu {cb.get('value')} / {cb.get('all_cores_O2_gibps')} ({cb.get('all_cores_threads')} thr) / "
          f"{cb.get('reference_flags_O0_1core_gibps')} (-O0)")
    for s in ("bench_c3full", "bench_c5"):
        x = last_json(src(s))
        print(f"{s} {x['value']}; encode {x['roofline']['launch_us']} us {x['roofline']['frac']} "
              f"(x{x['roofline']['mix_ceiling']['kernel_vs_ceiling']}); decode {x['decode_roofline']['launch_us']} "
              f"us {x['decode_roofline']['frac']}")
    for f in ("traffic_c3", "traffic_c5", "traffic_c3full", "traffic_c5p"):
        p = d / f"{f}.json"
        if p.exists():
            for k, v in json.loads(p.read_text()).items():
                print(f"{f} {k}: encode {v.get('encode_traffic_over_algorithmic', 0):.4f} decode "
                      f"{v.get('decode_traffic_over_algorithmic', 0):.4f}")
    mix = d / ("mix.log" if (d / "mix.log").exists() else "mix.json")
    for l in mix.read_text().splitlines():
        if l.startswith("{"):
            m = json.loads(l)
            print(f"mix {m['mix']} {m['median_us']} us {m['frac_of_8TBps']}")
    e2e = d / ("e2e.log" if (d / "e2e.log").exists() else "e2e_step.json")
    for l in e2e.read_text().splitlines():
        if l.startswith("{"):
            e = json.loads(l)
            print(f"e2e {e['workload'].split(',')[0][:6]} {e['workload'].split(', ')[-1]} zc={e['zero_copy']} "
                  f"enc {e['encode_e2e_gibps']} dec {e['decode_e2e_gibps']} step {e['step_e2e_gibps']}")
    w = json.loads((d / "wire.json").read_text())
    print("wire", {k: (v["median_us"], v["frac_of_hbm_peak"]) for k, v in w["kernels"].items()})
    g = (d / "group_bench.log").read_text()
    print("group_bench", " ".join(l.strip() for l in g.splitlines() if "median" in l or "line_level" in l))


if __name__ == "__main__":
    main()
