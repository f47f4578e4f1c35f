"""Prints one wire_bench result (gpurun_out/wst/w_<stride>.json) as one line (lab helper)."""
import json
import sys

s = sys.argv[1]
d = json.load(open(f"gpurun_out/wst/w_{s}.json"))
print(s, {k: (v["median_us"], v["frac_of_hbm_peak"]) for k, v in d["kernels"].items()})
