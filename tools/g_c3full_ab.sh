#!/bin/bash
# GPU box: interleaved A/B of librazor_fec.so builds (AB_LIBS, under tools/bin/abx/) on the c3full config
# (bench.py --config c3full, no wire / CPU legs).  bash tools/g_c3full_ab.sh TAG
set -o pipefail
TAG=${1:-c3ab}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in 1 2 3; do
  for L in ${AB_LIBS:-}; do
    timeout -k 10 150 python -u bench.py --lib tools/bin/abx/librazor_fec_$L.so --config c3full --steps 80 --warmup 5 --no-wire --no-cpu > $OUT/${L}_$r.json 2> $OUT/${L}_$r.err || { tail -20 $OUT/${L}_$r.err; exit 1; }
  done
done
python - "$OUT" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["config"]["workload"], "enc", d["roofline"]["launch_us"], "dec", d["decode_roofline"]["launch_us"],
          d["decode_roofline"]["frac"], "verified", d["verified"], d.get("verified_vs_reference_digest"))
PY
