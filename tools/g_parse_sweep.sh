#!/bin/bash
# Smoke, then the wire kernels' time against batch size (the per-launch fixed cost of the persistent parse / framing).
set -o pipefail
mkdir -p gpurun_out/psweep
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/psweep/smoke.log 2>&1 || { tail -30 gpurun_out/psweep/smoke.log; exit 1; }
tail -4 gpurun_out/psweep/smoke.log
for G in ${GROUPS_LIST:-8192 16384 32768 65536 131072 262144}; do
  timeout -k 10 120 python -u tools/wire_bench.py --groups $G --reps 10 --out gpurun_out/psweep/w$G.json > gpurun_out/psweep/w$G.log 2>&1 || { tail -20 gpurun_out/psweep/w$G.log; exit 1; }
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/psweep/w*.json"), key=lambda p:int(p.split("/w")[-1][:-5])):
    d=json.load(open(f)); print(d["groups"], {k: (v["median_us"], v["frac_of_hbm_peak"]) for k, v in d["kernels"].items()})
PY
# A/B (AB_LIBS: names under tools/bin/ab), interleaved, at the bench's size
for r in 1 2 3; do
  for L in ${AB_LIBS:-}; do
    timeout -k 10 120 python -u tools/wire_bench.py --reps 10 --lib tools/bin/abx/librazor_fec_v1200_$L.so --out gpurun_out/psweep/ab_${L}_$r.json > gpurun_out/psweep/ab_${L}_$r.log 2>&1 || { tail -20 gpurun_out/psweep/ab_${L}_$r.log; exit 1; }
  done
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/psweep/ab_*.json")):
    d=json.load(open(f)); print(f.split("/")[-1], {k: v["median_us"] for k, v in d["kernels"].items()}, d.get("verified"))
PY
