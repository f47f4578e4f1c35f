#!/bin/bash
# GPU box: interleaved A/B of librazor_fec.so builds (AB_LIBS, under tools/bin/abx/) on the bench's c3full and
# c5 sub-objects (headline steps kept short, no c4 / wire / CPU legs).  bash tools/g_c3full_ab.sh TAG
set -o pipefail
TAG=${1:-c3ab}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in 1 2 3; do
  for L in ${AB_LIBS:-}; do
    timeout -k 10 150 python -u bench.py --lib tools/bin/abx/librazor_fec_$L.so --steps 20 --warmup 5 --c4-steps 0 --no-wire --no-cpu > $OUT/${L}_$r.json 2> $OUT/${L}_$r.err || { tail -20 $OUT/${L}_$r.err; exit 1; }
  done
done
python - "$OUT" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    c = d["c3full"]; c5 = d["c5"]
    print(f.split("/")[-1], "c3 dec", d["decode_roofline"]["launch_us"], "c3full dec", c["decode"]["launch_us"], c["decode"]["frac"],
          "c5 dec", c5["decode"]["launch_us"], "verified", d["verified"], c["verified"])
PY
